#!/bin/bash
# Kernel traces of the PPO bench for several builds (A/B):
#   scripts/gpu_ktrace.sh <tag> <lib-name>...   (libmas.so = "main")
set -e
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = main ]; then LIB=""; else LIB="--lib $R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"; fi
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline $LIB > $O/kt_$v.log 2>&1
done
echo done
