#!/bin/bash
# GPU tests, then the per-kernel instruction mix of the env-step kernels
# (SQ counters, one rocprofv3 pass) on the driver-shaped bench window.
#   scripts/gpu_tests_pmc.sh <tag>
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_sq -o run \
  -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_sq.log 2>&1
echo done
