#!/bin/bash
# round measurement: tests, smoke, PMC traffic, headline bench, kernel stats
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 20 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 20 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
cd $R
python profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/r01_pmc_traffic.json 2v2:65536 > /dev/null || exit $?
cp $O/r01_pmc_traffic.json profiles/r01_pmc_traffic.json
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_ffa.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_1v1.log 2>&1 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1
echo "prof rc=$?"
