#!/bin/bash
# first GPU session: parity tests then bench then profile
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1
timeout -k 10 700 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "prof rc=$?"
