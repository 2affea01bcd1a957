#!/bin/bash
# A/B: per-kernel times of library variants, interleaved
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
i=0
for v in "$@"; do
  i=$((i+1))
  lib=$L/libmas${v:+_$v}.so; [ "$v" = base ] && lib=$L/libmas.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${i}_$v -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 40 --no-cpu-baseline --lib $lib > $O/${i}_$v.log 2>&1 || exit $?
done
echo done
