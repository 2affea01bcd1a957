#!/bin/bash
# re-validation: GPU tests, smoke, env + PPO bench lines, kernel stats of both benches
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_breakdown.py > $O/ppo_breakdown.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 20 --no-cpu-baseline > $O/prof_env.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ppo -o run -- python3 $R/bench.py --steps 64 --warmup 64 --no-cpu-baseline > $O/prof_ppo.log 2>&1 || exit $?
echo ok
