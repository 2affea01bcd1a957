#!/bin/bash
# r04s: the round's final measurement pass (after the fused general-path launch) on the default library --
# GPU suite + smoke + A/B golden, benches (driver window with the CPU
# baseline, long window, env-only 2v2 / FFA4 / 1v1, the full C4 / C5 sizes),
# kernel traces, PMC passes (PPO: SQ mix + FETCH / WRITE; env-only 2v2, FFA4,
# 1v1: FETCH / WRITE), phase timers
#   scripts/gpu_r04q.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export TMPDIR=/tmp
scripts/gpu_round.sh $TAG tests smoke ab bench env full profd envprof2 envprof || exit $?
bash $R/scripts/gpu_pmc_round.sh $TAG || exit $?
for cfg in "2v2 65536 40 10" "ffa4 16384 40 10" "1v1 4096 60 10"; do
  set -- $cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
      -d $O/pmc_${c}_$1 -o run -- python3 $R/bench.py --mode env --config $1 --envs $2 --steps $3 --warmup $4 --no-cpu-baseline > $O/pmc_${c}_$1.log 2>&1 || exit 1
  done
done
cd $R && timeout -k 10 200 python -u profiles/prof_lanes.py 2v2 65536 20 > $O/prof_lanes_2v2.txt 2>&1 || exit $?
cd $R && timeout -k 10 300 python -u profiles/prof_general.py 65536 20 --ppo > $O/prof_general.log 2>&1 || exit $?
echo r04s ok
