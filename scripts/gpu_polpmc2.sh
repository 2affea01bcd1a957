#!/bin/bash
# r04 policy PMC passes over scripts/policy_bench.py (default library: the
# double-buffered train kernel): SQ wave cycles / waits / instruction mix,
# LDS, and MFMA busy cycles; one counter set per run
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex "k_policy" --output-format csv -d $O/p1 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA --kernel-include-regex "k_policy" --output-format csv -d $O/p2 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM --kernel-include-regex "k_policy" --output-format csv -d $O/p3 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/p3.log 2>&1 || exit $?
echo ok
