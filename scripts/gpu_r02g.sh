set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r02g; mkdir -p $O; cd $R
timeout -k 10 200 python -u scripts/toi_latency.py --lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_base.so > $O/lat_base.log 2>&1
timeout -k 10 200 python -u scripts/toi_latency.py > $O/lat_new.log 2>&1
MAS_DUMP_DIR=$O timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_regimes.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_base.so > $O/bench_base.log 2>&1
echo done
