#!/bin/bash
# Kernel traces of the random-action env bench for several builds (A/B):
#   scripts/gpu_ktrace_env.sh <tag> <config> <steps> <lib-name>...   (libmas.so = "main")
set -e
R=$GRAFT_REPO_ROOT; TAG=$1; CFG=$2; ST=$3; shift 3; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = main ]; then LIB=""; else LIB="--lib $R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"; fi
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${CFG}_$v -o run -- \
    python3 $R/bench.py --mode env --config $CFG --steps $ST --warmup 10 --no-cpu-baseline $LIB > $O/kt_${CFG}_$v.log 2>&1
done
echo done
