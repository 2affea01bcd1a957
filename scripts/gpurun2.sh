#!/bin/bash
# GPU session 2: phase profile, parity + PPO tests, PPO bench, kernel stats, HBM counters
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python profiles/prof_phases.py 2v2 65536 20 > $O/phases.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_ppo.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ppo -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_ppo.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex k_step --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_sq.log 2>&1
echo "sq rc=$?"
