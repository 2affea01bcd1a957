#!/bin/bash
# per-kernel stats of the env-only and PPO benches + PPO phase breakdown
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/ppo_breakdown.py > $O/ppo_breakdown.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/env -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 20 --no-cpu-baseline > $O/env.log 2>&1 || exit $?
echo ok
