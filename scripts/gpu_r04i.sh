#!/bin/bash
# r04i: PMC passes (driver-shaped PPO bench: SQ mix, FETCH, WRITE; env-only
# 2v2: FETCH, WRITE) and the phase timers of the lane kernels and the general path
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export TMPDIR=/tmp
cd $R && timeout -k 10 200 python -u profiles/prof_lanes.py 2v2 65536 20 > $O/prof_lanes_2v2.txt 2>&1 || exit $?
cd $R && timeout -k 10 300 python -u profiles/prof_general.py 65536 20 --ppo > $O/prof_general.log 2>&1 || exit $?
bash $R/scripts/gpu_pmc_round.sh $TAG || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
    -d $O/pmc_${c}_2v2 -o run -- python3 $R/bench.py --mode env --config 2v2 --envs 65536 --steps 40 --warmup 10 --no-cpu-baseline > $O/pmc_${c}_2v2.log 2>&1 || exit 1
done
echo r04i ok
