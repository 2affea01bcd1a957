#!/bin/bash
# A/B builds of the fused policy kernels: libmas_<name>.so = the base objects
# with mas_policy.hip recompiled under extra -D flags.  usage: NAME "FLAGS" ...
set -e
C=$(dirname $0)/../gym-ma-survival-2d_amd/csrc
cd $C
L=../masurvival/_lib
FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Wno-unused-result -Wno-pass-failed -mllvm -pragma-unroll-threshold=200000"  # (the Makefile's)
while [ $# -gt 0 ]; do
  n=$1; f=$2; shift 2
  mkdir -p build_pv
  /opt/rocm/bin/hipcc $FLAGS $f -c -o build_pv/mas_policy_$n.o mas_policy.hip &
done
wait
for o in build_pv/mas_policy_*.o; do
  n=${o#build_pv/mas_policy_}; n=${n%.o}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/libmas_$n.so build/mas_k_*.o build/mas_capi.o $o
done
