#!/bin/bash
# A/B pass plus HBM traffic of the current build (FETCH_SIZE / WRITE_SIZE in
# separate passes over the driver-shaped window).   scripts/gpu_ab_pmc.sh <tag>
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
bash $R/scripts/gpu_ab.sh $1
bash $R/scripts/gpu_ktrace.sh $1 main prev
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv \
  -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv \
  -d $O/pmc_write -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_write.log 2>&1
echo done
