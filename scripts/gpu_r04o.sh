#!/bin/bash
# r04o: the GPU suite + smoke, env / driver benches, and the env-only 2v2 WRITE_SIZE pass
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export TMPDIR=/tmp
scripts/gpu_round.sh $TAG tests smoke env || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
    -d $O/pmc_${c}_2v2 -o run -- python3 $R/bench.py --mode env --config 2v2 --envs 65536 --steps 40 --warmup 10 --no-cpu-baseline > $O/pmc_${c}_2v2.log 2>&1 || exit 1
done
echo r04o ok
