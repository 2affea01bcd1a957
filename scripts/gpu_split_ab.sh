#!/bin/bash
# A/B of the split step (side stream for the general path + its envs' post
# phases) against the one-stream order, same library, MAS_SPLIT=0/1/2:
#   scripts/gpu_split_ab.sh <tag> [tests]
# env-only 2v2 x65536, FFA4 x16384, 1v1 x4096 and the driver window, each
# under its own time limit; stops at the first failing step.
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$1" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
  echo "tests ok"
fi
for sp in 0 1 2; do
  MAS_SPLIT=$sp timeout -k 10 200 python bench.py --mode env --steps 128 --warmup 64 --no-cpu-baseline > $O/env_2v2_s$sp.log 2>&1 || exit $?
  MAS_SPLIT=$sp timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline > $O/env_ffa_s$sp.log 2>&1 || exit $?
  MAS_SPLIT=$sp timeout -k 10 200 python bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline > $O/env_1v1_s$sp.log 2>&1 || exit $?
  MAS_SPLIT=$sp timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_s$sp.log 2>&1 || exit $?
  echo "split=$sp ok"
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit $?
echo ok
