#!/bin/bash
# round measurement: GPU tests, smoke, PMC HBM traffic of the env step,
# bench lines (headline PPO + env-only + other configs), kernel stats
# usage: scripts/gpu_measure.sh <round tag, e.g. r01>
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/measure
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 20 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 20 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
cd $R
python profiles/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/${TAG}_pmc_traffic.json 2v2:65536 > /dev/null || exit $?
cp $O/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_traffic.json
cd /tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_fetch_ppo -o run -- python3 $R/bench.py --no-cpu-baseline > $O/pmc_fetch_ppo.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_write_ppo -o run -- python3 $R/bench.py --no-cpu-baseline > $O/pmc_write_ppo.log 2>&1 || exit $?
cd $R
python profiles/pmc_traffic.py $O/pmc_fetch_ppo/run_counter_collection.csv $O/pmc_write_ppo/run_counter_collection.csv $O/${TAG}_pmc_traffic_ppo.json 2v2:65536:ppo > /dev/null || exit $?
cp $O/${TAG}_pmc_traffic_ppo.json profiles/${TAG}_pmc_traffic_ppo.json
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --no-cpu-baseline > $O/bench_env.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_ffa.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_1v1.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_breakdown.py > $O/ppo_breakdown.log 2>&1 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env -o run -- python3 $R/bench.py --mode env --no-cpu-baseline > $O/prof_env.log 2>&1 || exit $?
cd $R
python profiles/stats_summary.py $O/prof_bench/run_kernel_stats.csv profiles/${TAG}_kernel_stats.txt "round ${TAG#r}: rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (MI355X, 2v2 N_envs=65536, PPO: 64 warmup + 128 timed steps, 3 updates)" 192 $O/prof_bench/run_kernel_trace.csv 128 || exit $?
python profiles/stats_summary.py $O/prof_env/run_kernel_stats.csv profiles/${TAG}_kernel_stats_env.txt "round ${TAG#r}: rocprofv3 --kernel-trace --stats -- python3 bench.py --mode env --no-cpu-baseline (MI355X, 2v2 N_envs=65536, random policy: 64 warmup + 128 timed steps)" 192 $O/prof_env/run_kernel_trace.csv 128 || exit $?
echo ok
