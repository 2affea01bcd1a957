#!/bin/bash
# A/B: env-only bench per library variant (base = libmas.so) + per-kernel stats;
# then the GPU parity tests on libmas.so
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abenv
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
for v in base "$@" base; do
  lib=$L/libmas_$v.so; [ "$v" = base ] && lib=$L/libmas.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/bench.py --mode env --steps 128 --warmup 64 --no-cpu-baseline --lib $lib > $O/$v.log 2>&1 || exit $?
done
echo ok
