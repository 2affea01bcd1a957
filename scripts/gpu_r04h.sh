#!/bin/bash
# r04h: the round's measurement pass on the default library -- benches
# (driver window with the CPU baseline, long window, env-only 2v2 / FFA4 /
# 1v1, the full C4 / C5 sizes), kernel traces, and the PMC passes (SQ mix +
# FETCH_SIZE / WRITE_SIZE of the driver-shaped PPO bench; FETCH / WRITE of
# the env-only 2v2 bench)
#   scripts/gpu_r04h.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export TMPDIR=/tmp
scripts/gpu_round.sh $TAG bench env full profd envprof2 envprof || exit $?
scripts/gpu_pmc_round.sh $TAG || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
    -d $O/pmc_${c}_2v2 -o run -- python3 $R/bench.py --mode env --config 2v2 --envs 65536 --steps 40 --warmup 10 --no-cpu-baseline > $O/pmc_${c}_2v2.log 2>&1 || exit 1
done
cd $R && timeout -k 10 300 python -u profiles/prof_general.py 65536 20 --ppo > $O/prof_general.log 2>&1 || exit $?
cd $R && timeout -k 10 200 python -u profiles/prof_lanes.py 2v2 65536 20 > $O/prof_lanes_2v2.txt 2>&1 || exit $?
echo r04h ok
