#!/bin/bash
# r04t: the seen rows of k_post_lanes as LDS bytes (MAS_POST_SEEN8, 12 instead
# of 11 workgroups per CU for 2v2): GPU suite on the default library, then
# env-only 2v2 / 1v1 and driver benches against libmas_s0.so (seen words) in
# alternating processes
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
S0=gym-ma-survival-2d_amd/masurvival/_lib/libmas_s0.so
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --mode env --no-cpu-baseline >> $O/bench_env_s8.json 2>> $O/err.log || exit $?
  timeout -k 10 300 python -u bench.py --mode env --no-cpu-baseline --lib $S0 >> $O/bench_env_s0.json 2>> $O/err.log || exit $?
done
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --mode env --config 1v1 --envs 4096 --steps 100 --warmup 20 --no-cpu-baseline >> $O/bench_1v1_s8.json 2>> $O/err.log || exit $?
  timeout -k 10 300 python -u bench.py --mode env --config 1v1 --envs 4096 --steps 100 --warmup 20 --no-cpu-baseline --lib $S0 >> $O/bench_1v1_s0.json 2>> $O/err.log || exit $?
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_driver_s8.json 2>> $O/err.log || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --lib $S0 >> $O/bench_driver_s0.json 2>> $O/err.log || exit $?
echo ok
