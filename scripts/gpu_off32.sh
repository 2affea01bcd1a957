#!/bin/bash
# policy train kernel with 32-bit store offsets: GPU tests, policy micro-bench,
# driver-shaped bench; every step under its own time limit
R=$GRAFT_REPO_ROOT
TAG=${1:-off32}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/policy_bench.py > $O/polbench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit $?
echo ok
