#!/bin/bash
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r02j; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_regimes.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
bash scripts/gpu_ktrace.sh r02j main prev
