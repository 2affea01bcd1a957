#!/bin/bash
# quick re-validation: GPU parity tests, smoke, env + PPO bench lines
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
echo ok
