#!/bin/bash
# r04r: the train kernel's transposed activation stores (MAS_POL_TR), the
# persistent act kernel (MAS_POL_ACT_DB) and the
# fused two-world-step general-path launch (MAS_GEN_FUSE2): GPU policy tests
# and the general-path parity tests, policy_bench under MAS_POL_TR=1 / 0 in
# alternating processes, then env-only and driver benches under each knob
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
export MAS_POL_TR=1 MAS_POL_ACT_DB=1 MAS_GEN_FUSE2=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py -x -v --timeout 120 --timeout-method thread > $O/tests_pol.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_policy.py > $O/tests_env.log 2>&1 || exit $?
for tr in 1 0 1 0; do
  MAS_POL_TR=$tr MAS_POL_ACT_DB=$tr timeout -k 10 300 python -u scripts/policy_bench.py >> $O/polbench_tr$tr.log 2>&1 || exit $?
done
for f in 1 0 1 0; do
  MAS_GEN_FUSE2=$f timeout -k 10 300 python -u bench.py --mode env --no-cpu-baseline >> $O/bench_env_f$f.json 2>> $O/bench_env.err || exit $?
done
for f in 1 0; do
  MAS_GEN_FUSE2=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline >> $O/bench_driver_f$f.json 2>> $O/bench_driver.err || exit $?
done
MAS_POL_TR=0 MAS_POL_ACT_DB=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline >> $O/bench_driver_tr0.json 2>> $O/bench_driver.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --shards 2 >> $O/bench_driver_sh2.json 2>> $O/bench_driver.err || exit $?
echo ok
