#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/misc
mkdir -p $O
cd $R
for c in 16 32 64 128 256; do
  MAS_SPLITK_CAP=$c timeout -k 10 120 python scripts/policy_bench.py > $O/splitk_$c.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex "mas::k_" --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 64 --no-cpu-baseline > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM --kernel-include-regex "mas::k_" --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --mode env --steps 40 --warmup 64 --no-cpu-baseline > $O/p2.log 2>&1 || exit $?
echo ok
