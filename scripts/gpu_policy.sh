#!/bin/bash
# fused policy kernels: tests, then the PPO breakdown and bench
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pol
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_breakdown.py > $O/ppo_breakdown.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
echo ok
