#!/bin/bash
# r04 diagnosis pass of the agent-lane kernels: phase timers (profiling
# build), the SQ instruction mix and wait counters of the env-only bench, and
# the HBM traffic passes of the env-only workloads (2v2 x65536, FFA4 x16384,
# 1v1 x4096)
#   scripts/gpu_r04_diag.sh <tag> [phases] [sq] [traffic]
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    phases)
      cd $R && timeout -k 10 200 python -u profiles/prof_lanes.py 2v2 65536 20 > $O/prof_lanes_2v2.txt 2>&1 || exit 1 ;;
    sq)
      cd /tmp && timeout -s KILL 120 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
      cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_sq_env -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_sq_env.log 2>&1 || exit 1
      cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU \
        --kernel-include-regex "mas::k_" --output-format csv -d $O/pmc_sqw_env -o run -- python3 $R/bench.py --mode env --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_sqw_env.log 2>&1 || exit 1 ;;
    traffic)
      for cfg in "2v2 65536 40 10" "ffa4 16384 40 10" "1v1 4096 60 10"; do
        set -- $cfg
        for c in FETCH_SIZE WRITE_SIZE; do
          cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "mas::k_" --output-format csv \
            -d $O/pmc_${c}_$1 -o run -- python3 $R/bench.py --mode env --config $1 --envs $2 --steps $3 --warmup $4 --no-cpu-baseline > $O/pmc_${c}_$1.log 2>&1 || exit 1
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
echo ok
