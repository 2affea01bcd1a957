#!/bin/bash
# PPO regime over many iterations: per-iteration env step cost and a kernel
# trace to attribute it (scripts/ppo_breakdown.py)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trend
mkdir -p $O
cd $R
timeout -k 10 200 python -u scripts/ppo_breakdown.py 65536 ${1:-12} > $O/breakdown.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/scripts/ppo_breakdown.py 65536 ${1:-12} > $O/prof.log 2>&1 || exit $?
echo ok
