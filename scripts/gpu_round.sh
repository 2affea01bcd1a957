#!/bin/bash
# One GPU measurement pass (run via gpurun from the repo root):
#   scripts/gpu_round.sh <tag> <step>...   (steps: the case labels below, e.g.
#   tests t:<files> testslib:<variant> gaebench ab regimes smoke bench benchq benchcw0 shards env full
#   c4rank envprof2 prof profd envprof pmc pmcenv sqmix profenv profwaves split0ab slowkab
#   libab:<variant> trafab:<libs> ktrace:<libs> ktraced:<libs> ktraceenv:<cfg>:<steps>:<libs> dist
#   polab[:<libs>] polpmc trend[:<iterations>])
# writes gpurun_out/<tag>/...; every GPU step has its own time limit and the
# script stops at the first failing step.
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; } ;;
    testslib:*)
      # testslib:<variant>: the GPU suite on masurvival/_lib/libmas_<variant>.so (MAS_LIB)
      cd $R && MAS_LIB=$R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_${step#testslib:}.so timeout -k 10 900 \
        python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/gpu_tests_${step#testslib:}.log 2>&1 || { echo "tests failed"; exit 1; } ;;
    testsv:*)
      # testsv:<variant>: the GPU suite on a narrowed variant library (MAS_CLASSES="2v2 ffa": other classes skip)
      cd $R && MAS_CLASSES="2v2 ffa" MAS_LIB=$R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_${step#testsv:}.so timeout -k 10 900 \
        python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/gpu_tests_${step#testsv:}.log 2>&1 || { echo "tests failed"; exit 1; } ;;
    t:*)
      # t:<file.py>[,<file.py>...]: those GPU test files only
      F=$(echo ${step#t:} | tr ',' ' ' | sed 's#\([^ ]*\)#tests/\1#g')
      cd $R && timeout -k 10 900 python -u -m pytest $F -m gpu -x -v -s --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $O/gpu_tests_sel.log 2>&1 || { echo "selected tests failed"; exit 1; } ;;
    gaebench*)
      # gaebench[:<variant>,...]: mas_gae timing on the default library, then on each variant (MAS_LIB)
      cd $R && timeout -k 10 200 python -u scripts/gae_bench.py > $O/gae_bench.txt 2>&1 || exit 1
      if [ "$step" != gaebench ]; then
        for v in $(echo ${step#gaebench:} | tr ',' ' '); do
          cd $R && MAS_LIB=$R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so timeout -k 10 200 python -u scripts/gae_bench.py \
            >> $O/gae_bench.txt 2>&1 || exit 1
        done
      fi ;;
    py:*)
      # py:<script>[,arg...]: one python script (repo-relative), output to <tag>/py_<name>.txt
      IFS=, read -r SCR ARGS <<< "${step#py:}"
      cd $R && timeout -k 10 300 python -u $SCR $(echo $ARGS | tr ',' ' ') > $O/py_$(basename $SCR .py).txt 2>&1 || exit 1 ;;
    ab)
      cd $R && timeout -k 10 600 python -u scripts/ab_solve_golden.py all > $O/ab_golden.log 2>&1 || { echo "A/B differs"; exit 1; } ;;
    regimes)
      cd $R && MAS_DUMP_DIR=$O timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_regimes.py -x -v -s \
        --timeout 600 --timeout-method thread -p no:cacheprovider > $O/regimes.log 2>&1 || { echo "regimes failed"; exit 1; } ;;
    smoke)
      cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $? ;;
    bench)
      cd $R && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit $?
      cd $R && timeout -k 10 400 python bench.py --no-cpu-baseline --no-live-traffic > $O/bench.log 2>&1 || exit $? ;;
    benchcw0)
      # the PPO update on k_policy_train (MAS_POL_CW=0): the counted-wait kernel's A/B
      cd $R && MAS_POL_CW=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/bench_driver_cw0.log 2>&1 || exit $? ;;
    benchq)
      cd $R && timeout -k 10 400 python bench.py --no-cpu-baseline --no-live-traffic > $O/bench.log 2>&1 || exit $?
      cd $R && timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/bench_driver.log 2>&1 || exit $? ;;
    shards)
      cd $R && timeout -k 10 400 python bench.py --steps 20 --warmup 5 --shards 2 --no-cpu-baseline --no-live-traffic > $O/bench_driver_shards2.log 2>&1 || exit $?
      cd $R && timeout -k 10 400 python bench.py --shards 2 --no-cpu-baseline --no-live-traffic > $O/bench_shards2.log 2>&1 || exit $? ;;
    shardab)
      # env handles per GPU on concurrent streams (bench.py --shards): 1, 2, 4, alternating, twice; driver window
      for k in 1 2; do
        for sh in 1 2 4; do
          cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --shards $sh --no-cpu-baseline --no-live-traffic >> $O/shardab_driver_sh$sh.json 2>> $O/shardab.err || exit 1
        done
      done ;;
    env)
      cd $R && timeout -k 10 200 python bench.py --mode env --no-cpu-baseline --no-live-traffic > $O/bench_env.log 2>&1 || exit $?
      cd $R && timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic > $O/bench_ffa.log 2>&1 || exit $?
      cd $R && timeout -k 10 200 python bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline --no-live-traffic > $O/bench_1v1.log 2>&1 || exit $? ;;
    full)
      # the C4 / C5 workloads at their configured env counts on one GPU
      cd $R && timeout -k 10 300 python bench.py --mode env --envs 262144 --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic > $O/bench_env_c4full.log 2>&1 || exit $?
      cd $R && timeout -k 10 300 python bench.py --mode env --config ffa4 --envs 131072 --steps 30 --warmup 10 --no-cpu-baseline --no-live-traffic > $O/bench_env_c5full.log 2>&1 || exit $? ;;
    c4rank)
      # the C4 per-rank workload of the 8-GPU target (2v2 x 262144 over 8 GPUs = 32768 per rank) in the
      # driver-shaped PPO window: bench line, kernel trace, FETCH / WRITE passes
      cd $R && timeout -k 10 300 python bench.py --envs 32768 --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/bench_driver_c4rank.log 2>&1 || exit $?
      cd $R && timeout -k 10 300 python bench.py --envs 32768 --no-cpu-baseline --no-live-traffic > $O/bench_c4rank.log 2>&1 || exit $?
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4rank -o run -- \
        python3 $R/bench.py --envs 32768 --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/prof_c4rank.log 2>&1 || exit $?
      for c in FETCH_SIZE WRITE_SIZE; do
        cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
          -d $O/pmc_${c}_c4rank -o run -- python3 $R/bench.py --envs 32768 --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/pmc_${c}_c4rank.log 2>&1 || exit $?
      done ;;
    envprof2)
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env -o run -- \
        python3 $R/bench.py --mode env --no-cpu-baseline --no-live-traffic > $O/prof_env.log 2>&1 || exit $? ;;
    prof)
      cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
        python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/prof_bench.log 2>&1 || exit $?
      cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench128 -o run -- \
        python3 $R/bench.py --no-cpu-baseline --no-live-traffic > $O/prof_bench128.log 2>&1 || exit $? ;;
    profd)
      cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
        python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/prof_bench.log 2>&1 || exit $? ;;
    pmc)
      cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mas::k_" --output-format csv \
        -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/pmc_fetch.log 2>&1 || exit $?
      cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mas::k_" --output-format csv \
        -d $O/pmc_write -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/pmc_write.log 2>&1 || exit $? ;;
    envprof)
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ffa -o run -- \
        python3 $R/bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic > $O/prof_ffa.log 2>&1 || exit $?
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_1v1 -o run -- \
        python3 $R/bench.py --mode env --config 1v1 --steps 100 --warmup 20 --no-cpu-baseline --no-live-traffic > $O/prof_1v1.log 2>&1 || exit $? ;;
    profenv)
      # phase timers of the env kernels (libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc prof`)
      cd $R && timeout -k 10 300 python -u profiles/prof_env.py 2v2 65536 20 --ppo > $O/prof_env_ppo.txt 2>&1 || exit $?
      cd $R && timeout -k 10 200 python -u profiles/prof_env.py 2v2 65536 20 > $O/prof_env_2v2.txt 2>&1 || exit $? ;;
    profwaves)
      # per-wave span distribution of the env kernels (profiling build), PPO and random regimes
      cd $R && timeout -k 10 300 python -u profiles/prof_env.py 2v2 65536 20 --ppo --waves > $O/prof_waves_ppo.txt 2>&1 || exit $?
      cd $R && timeout -k 10 200 python -u profiles/prof_env.py 2v2 65536 20 --waves > $O/prof_waves_2v2.txt 2>&1 || exit $? ;;
    split0ab)
      # the slow split (default) vs one stream (MAS_SPLIT=0), alternating processes: driver window, env-only 2v2
      for sp in 2 0 2 0; do
        cd $R && MAS_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic >> $O/split0ab_driver_sp$sp.json 2>> $O/split0ab.err || exit 1
        cd $R && MAS_SPLIT=$sp timeout -k 10 200 python -u bench.py --mode env --no-cpu-baseline --no-live-traffic >> $O/split0ab_env_sp$sp.json 2>> $O/split0ab.err || exit 1
      done ;;
    slowkab*)
      # MAS_SLOW_K (TOI events of an env's step that send it to the slow list next step), alternating:
      # slowkab = 4 (default) vs 2 vs 1; slowkab:<k>,<k>,... those values
      KS="4 2 1"; [ "$step" != slowkab ] && KS=$(echo ${step#slowkab:} | tr ',' ' ')
      for k in $KS $KS; do
        cd $R && MAS_SLOW_K=$k timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic >> $O/slowkab_driver_k$k.json 2>> $O/slowkab.err || exit 1
      done ;;
    libab:*)
      # libab:<variant>: driver window + env-only 2v2, default library vs masurvival/_lib/libmas_<variant>.so, alternating
      V=${step#libab:}
      for k in 1 2; do
        for lib in default $V; do
          L=""; [ $lib != default ] && L="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$lib.so"
          cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic $L >> $O/libab_driver_$lib.json 2>> $O/libab.err || exit 1
          cd $R && timeout -k 10 200 python -u bench.py --mode env --no-cpu-baseline --no-live-traffic $L >> $O/libab_env_$lib.json 2>> $O/libab.err || exit 1
        done
      done ;;
    varab:*)
      # varab:<lib>:<VAR>:<v1>,<v2>,...: one library (main = libmas.so), the environment variable VAR at
      # each value, alternating, twice: driver window, env-only 2v2 and FFA4 x16384
      IFS=: read -r _ V VAR VALS <<< "$step"
      LIB=""; [ "$V" != main ] && LIB="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$V.so"
      for k in 1 2; do
        for val in $(echo $VALS | tr ',' ' '); do
          cd $R && env $VAR=$val timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic $LIB >> $O/varab_${V}_driver_$VAR$val.json 2>> $O/varab.err || exit 1
          cd $R && env $VAR=$val timeout -k 10 200 python -u bench.py --mode env --no-cpu-baseline --no-live-traffic $LIB >> $O/varab_${V}_env_$VAR$val.json 2>> $O/varab.err || exit 1
          cd $R && env $VAR=$val timeout -k 10 200 python -u bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic $LIB >> $O/varab_${V}_ffa_$VAR$val.json 2>> $O/varab.err || exit 1
        done
      done ;;
    libabx:*)
      # libabx:<lib>,<lib>,...: driver window, env-only 2v2 and FFA4 x16384 per library (main = libmas.so), alternating, twice
      for k in 1 2; do
        for v in $(echo ${step#libabx:} | tr ',' ' '); do
          LIB=""; [ "$v" != main ] && LIB="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
          cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic $LIB >> $O/libabx_driver_$v.json 2>> $O/libabx.err || exit 1
          cd $R && timeout -k 10 200 python -u bench.py --mode env --no-cpu-baseline --no-live-traffic $LIB >> $O/libabx_env_$v.json 2>> $O/libabx.err || exit 1
          cd $R && timeout -k 10 200 python -u bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic $LIB >> $O/libabx_ffa_$v.json 2>> $O/libabx.err || exit 1
        done
      done ;;
    trafab:*)
      # trafab:<lib>[,<lib>...]: the driver window with its live FETCH / WRITE passes (roofline.traffic) per library
      for v in $(echo ${step#trafab:} | tr ',' ' '); do
        LIB=""; [ "$v" != main ] && LIB="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
        cd $R && timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $LIB > $O/trafab_driver_$v.json 2>> $O/trafab.err || exit 1
      done ;;
    pmcenv)
      # FETCH_SIZE / WRITE_SIZE passes of the env-only workloads (2v2, FFA4 shard, 1v1, C4 / C5 full)
      for cfg in "2v2 65536 40 10" "ffa4 16384 40 10" "1v1 4096 60 10" "2v2 262144 20 10" "ffa4 131072 15 10"; do
        set -- $cfg
        for c in FETCH_SIZE WRITE_SIZE; do
          cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
            -d $O/pmc_${c}_$1_$2 -o run -- python3 $R/bench.py --mode env --config $1 --envs $2 --steps $3 --warmup $4 --no-cpu-baseline --no-live-traffic > $O/pmc_${c}_$1_$2.log 2>&1 || exit 1
        done
      done ;;
    sqmix)
      # SQ instruction mix of the env kernels in the driver-shaped bench (one counter set, its own run)
      cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > $O/pmc_sq.log 2>&1 || exit 1 ;;
    ktrace:*)
      # ktrace:<lib>[,<lib>...]: kernel traces of the PPO bench per library (main = libmas.so)
      for v in $(echo ${step#ktrace:} | tr ',' ' '); do
        LIB=""; [ "$v" != main ] && LIB="--lib $R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
        cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
          python3 $R/bench.py --no-cpu-baseline --no-live-traffic $LIB > $O/kt_$v.log 2>&1 || exit 1
      done ;;
    ktraced:*)
      # ktraced:<lib>[,<lib>...]: kernel traces of the driver-window bench (20 steps, 1 update) per library
      for v in $(echo ${step#ktraced:} | tr ',' ' '); do
        LIB=""; [ "$v" != main ] && LIB="--lib $R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
        cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktd_$v -o run -- \
          python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic $LIB > $O/ktd_$v.log 2>&1 || exit 1
      done ;;
    ktraceenv:*)
      # ktraceenv:<config>:<steps>:<lib>[,<lib>...]: kernel traces of the env-only bench per library
      IFS=: read -r _ CFG ST LIBS <<< "$step"
      for v in $(echo $LIBS | tr ',' ' '); do
        LIB=""; [ "$v" != main ] && LIB="--lib $R/gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
        cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${CFG}_$v -o run -- \
          python3 $R/bench.py --mode env --config $CFG --steps $ST --warmup 10 --no-cpu-baseline --no-live-traffic $LIB > $O/kt_${CFG}_$v.log 2>&1 || exit 1
      done ;;
    dist)
      # multi-rank rehearsal on one GPU: 2 ranks over gloo (test + bench launch path)
      cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread \
        -p no:cacheprovider > $O/dist_test.log 2>&1 || exit 1
      cd $R && MAS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 16 --warmup 16 --horizon 16 --envs 4096 \
        > $O/dist_bench2.log 2>&1 || exit 1 ;;
    polab*)
      # polab[:<lib>,...]: GPU policy tests, then scripts/policy_bench.py over the default library and
      # the variant libraries (scripts/build_policy_variants.sh)
      L=gym-ma-survival-2d_amd/masurvival/_lib
      LIBS=""; [ "$step" != polab ] && LIBS=$(echo ${step#polab:} | tr ',' '\n' | sed "s#^#$L/libmas_#; s#\$#.so#" | tr '\n' ' ')
      cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 120 --timeout-method thread \
        -p no:cacheprovider > $O/polab_tests.log 2>&1 || exit 1
      cd $R && timeout -k 10 300 python -u scripts/policy_bench.py $L/libmas.so $LIBS > $O/polbench.log 2>&1 || exit 1 ;;
    polpmc)
      # PMC passes over the policy micro-bench (default library): HBM bytes, then two SQ sets
      L=$R/gym-ma-survival-2d_amd/masurvival/_lib
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "pol::k_" --output-format csv -d $O/pol_fetch -o run -- \
        python3 $R/scripts/policy_bench.py $L/libmas.so > $O/pol_fetch.log 2>&1 || exit 1
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "pol::k_" --output-format csv -d $O/pol_write -o run -- \
        python3 $R/scripts/policy_bench.py $L/libmas.so > $O/pol_write.log 2>&1 || exit 1
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
        --kernel-include-regex "k_policy" --output-format csv -d $O/pol_p1 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/pol_p1.log 2>&1 || exit 1
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM \
        --kernel-include-regex "k_policy" --output-format csv -d $O/pol_p2 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/pol_p2.log 2>&1 || exit 1 ;;
    trend*)
      # trend[:<iterations>]: PPO regime over many iterations, per-iteration env step cost + kernel trace
      IT=12; [ "$step" != trend ] && IT=${step#trend:}
      cd $R && timeout -k 10 200 python -u scripts/ppo_breakdown.py 65536 $IT > $O/trend_breakdown.log 2>&1 || exit 1
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trend_prof -o run -- \
        python3 $R/scripts/ppo_breakdown.py 65536 $IT > $O/trend_prof.log 2>&1 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
echo ok
