#!/bin/bash
# PMC passes of the driver-shaped bench (each pass its own run): SQ
# instruction mix of the env kernels, then HBM FETCH_SIZE and WRITE_SIZE.
#   scripts/gpu_pmc_round.sh <tag>
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || exit 1
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv \
  -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit 1
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv \
  -d $O/pmc_write -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit 1
echo pmc ok
