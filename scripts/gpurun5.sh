#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --mode env --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env -o run -- python3 $R/bench.py --mode env --steps 50 --warmup 5 --no-cpu-baseline > $O/prof_env.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH --kernel-include-regex "mas::" --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_sq.log 2>&1
echo "sq rc=$?"
