#!/bin/bash
# r04b: the reconstructed short-circuit sleep loop (1v1 A/B build) probe, then
# the agent-lane kernels (quick 1v1 + 2v2 build): parity, graph replay, bench
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04b; mkdir -p $O; cd $R
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
export MAS_LIB=$L/libmas_q.so
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_facade.py tests/test_gpu_split.py tests/test_gpu_full_size.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_q.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline --lib $L/libmas_q.so > $O/bench_env_q.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline --lib $L/libmas.so > $O/bench_env_old.log 2>&1 || exit 1
echo ok
