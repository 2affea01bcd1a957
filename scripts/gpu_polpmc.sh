#!/bin/bash
# PMC passes over the policy micro-bench (scripts/policy_bench.py, default
# library): HBM fetch / write bytes of the policy kernels, then two SQ passes
# (wave cycles, waits, instruction mix, LDS bank conflicts); one counter set
# per run, each under its own time limit.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/polpmc
mkdir -p $O
L=$R/gym-ma-survival-2d_amd/masurvival/_lib
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "pol::k_" --output-format csv -d $O/fetch -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "pol::k_" --output-format csv -d $O/write -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex "k_policy" --output-format csv -d $O/p1 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM --kernel-include-regex "k_policy" --output-format csv -d $O/p2 -o run -- python3 $R/scripts/policy_bench.py $L/libmas.so > $O/p2.log 2>&1 || exit $?
echo ok
