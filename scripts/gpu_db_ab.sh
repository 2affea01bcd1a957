#!/bin/bash
# A/B of the double-buffered train-kernel weight stages (MAS_POL_DB variants
# from build_policy_variants.sh): policy numerics tests per library, the
# policy micro-bench over all, then the driver-shaped bench per library.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dbab
mkdir -p $O
cd $R
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
for v in dbB dbC; do
  MAS_LIB=$L/libmas_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_ppo.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
done
timeout -k 10 300 python -u scripts/policy_bench.py $L/libmas.so $L/libmas_dbA.so $L/libmas_dbB.so $L/libmas_dbC.so > $O/polbench.log 2>&1 || exit $?
for v in "" _dbC; do
  MAS_LIB=$L/libmas$v.so timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver$v.log 2>&1 || exit $?
done
echo ok
