#!/bin/bash
# policy kernel A/B: GPU policy tests on the default library, then
# scripts/policy_bench.py over the variant libraries (build_policy_variants.sh)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/polab
mkdir -p $O
cd $R
L=gym-ma-survival-2d_amd/masurvival/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/policy_bench.py "$@" > $O/polbench.log 2>&1 || exit $?
echo ok
