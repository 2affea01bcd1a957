#!/bin/bash
# policy A/B (r04): GPU policy tests on the default library, then
# scripts/policy_bench.py over the variant libraries under MAS_POL_CW=1 / 0
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for cw in 1 0; do
  MAS_POL_CW=$cw timeout -k 10 300 python -u scripts/policy_bench.py "$@" > $O/polbench_cw$cw.log 2>&1 || exit $?
done
echo ok
