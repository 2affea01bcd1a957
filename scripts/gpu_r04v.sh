#!/bin/bash
# r04v: row-stride padding of the feature-major activation buffers
# (MAS_ACT_PAD) -- policy_bench per pad, alternating processes
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
for pad in 64 32 128 256 64 32 128 256; do
  echo -n "pad $pad: " >> $O/polbench.log
  MAS_ACT_PAD=$pad timeout -k 10 300 python -u scripts/policy_bench.py 2>/dev/null | grep libmas >> $O/polbench.log || exit $?
done
echo ok
