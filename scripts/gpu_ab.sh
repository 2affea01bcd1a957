#!/bin/bash
# A/B pass: parity of the current build, then the single-env SolveTOI latency
# replay and the PPO bench for the current build and libmas_prev.so.
#   scripts/gpu_ab.sh <tag>
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
PREV=gym-ma-survival-2d_amd/masurvival/_lib/libmas_prev.so
MAS_DUMP_DIR=$O timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_regimes.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
timeout -k 10 200 python -u scripts/toi_latency.py --lib $PREV > $O/lat_prev.log 2>&1
timeout -k 10 200 python -u scripts/toi_latency.py > $O/lat_new.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --lib $PREV > $O/bench_prev.log 2>&1
echo done
