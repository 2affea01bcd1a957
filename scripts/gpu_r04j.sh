#!/bin/bash
# r04j: the GPU suite + smoke, then benches of the batched state loads
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
scripts/gpu_round.sh $TAG tests smoke env || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || exit $?
cd $R && timeout -k 10 200 python -u profiles/prof_lanes.py 2v2 65536 20 > $O/prof_lanes_2v2.txt 2>&1 || exit $?
echo r04j ok
