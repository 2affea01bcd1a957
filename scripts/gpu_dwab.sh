#!/bin/bash
# weight-gradient kernel A/B: scripts/policy_bench.py per library, one process each (run-order bias)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
for v in "$@"; do
  timeout -k 10 200 python -u scripts/policy_bench.py $L/libmas$v.so >> $O/polbench.log 2>&1 || exit $?
done
echo ok
