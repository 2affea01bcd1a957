#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ppo.log 2>&1 || exit $?
rm -rf $O/ab; $R/scripts/gpurun_ab.sh base || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ppo -o run -- python3 $R/bench.py --steps 64 --warmup 64 --no-cpu-baseline > $O/prof_ppo.log 2>&1
echo "prof rc=$?"
