#!/bin/bash
# r04 perf pass: benches (driver window, long window, env-only 2v2 / FFA4 /
# 1v1, the full C4 / C5 sizes), kernel traces, and the k_pre_lanes
# occupancy A/B (libmas_p3.so: MAS_PRE_OCC=3)
#   scripts/gpu_r04_perf.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
scripts/gpu_round.sh $TAG t:test_gpu_policy.py bench benchcw0 env full profd envprof2 envprof || exit $?
if [ -f $L/libmas_p3.so ]; then
  timeout -k 10 200 python bench.py --mode env --no-cpu-baseline --lib $L/libmas_p3.so > $O/bench_env_p3.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --lib $L/libmas_p3.so > $O/bench_ffa_p3.log 2>&1 || exit $?
fi
echo perf ok
