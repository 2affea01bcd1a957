#!/bin/bash
# r04g: the GPU suite on the default library (sequential obs rows, k_post_lanes
# at 3 waves / SIMD, policy biases in LDS), env-bench A/B of the obs writers
# (libmas_tile: LDS tile windows at 2 waves; libmas_seq2: sequential rows at
# 2 waves) and the policy A/B (libmas_nolds, libmas_nodefer; MAS_POL_CW 1 / 0)
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
scripts/gpu_round.sh $TAG tests || exit $?
for v in "" _tile _seq2; do
  timeout -k 10 200 python bench.py --mode env --no-cpu-baseline --lib $L/libmas$v.so > $O/bench_env$v.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --lib $L/libmas$v.so > $O/bench_ffa$v.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline --lib $L/libmas$v.so > $O/bench_1v1$v.log 2>&1 || exit $?
done
for v in "MAS_POL_DB=1 MAS_POL_CW=1" "MAS_POL_DB=0 MAS_POL_CW=1" "MAS_POL_DB=0 MAS_POL_CW=0"; do
  env $v timeout -k 10 300 python -u scripts/policy_bench.py $L/libmas.so $L/libmas_nolds.so >> $O/polbench.log 2>&1 || exit $?
  echo "^ $v" >> $O/polbench.log
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || exit $?
MAS_POL_DB=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_db0.log 2>&1 || exit $?
echo ok
