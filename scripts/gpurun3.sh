#!/bin/bash
# split-kernel version: parity tests, bench (ppo + env), kernel stats
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --mode env --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env -o run -- python3 $R/bench.py --mode env --steps 50 --warmup 5 --no-cpu-baseline > $O/prof_env.log 2>&1
echo "prof rc=$?"
