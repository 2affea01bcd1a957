#!/bin/bash
# per-kernel stats of the env-only bench for libmas.so and the variants named on the command line
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abenv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
for v in base "$@"; do
  lib=$L/libmas_$v.so; [ "$v" = base ] && lib=$L/libmas.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 20 --no-cpu-baseline --lib $lib > $O/$v.log 2>&1 || exit $?
done
echo ok
