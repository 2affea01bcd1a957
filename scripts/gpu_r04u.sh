#!/bin/bash
# r04u: split-K chunk count of the layer-1 weight-gradient GEMM (hipBLASLt
# batched GEMM over K chunks, MAS_SPLITK_CAP) -- policy_bench per cap,
# alternating processes
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
for cap in 64 32 128 256 64 32 128 256; do
  echo -n "cap $cap: " >> $O/polbench.log
  MAS_SPLITK_CAP=$cap timeout -k 10 300 python -u scripts/policy_bench.py 2>/dev/null | grep libmas >> $O/polbench.log || exit $?
done
echo ok
