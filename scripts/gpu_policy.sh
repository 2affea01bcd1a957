#!/bin/bash
# fused policy kernels: tests, then the PPO breakdown, bench and kernel stats
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pol
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_ppo.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/policy_bench.py > $O/polbench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_breakdown.py > $O/ppo_breakdown.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 64 --warmup 64 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
echo ok
