#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python profiles/prof_phases.py 2v2 65536 20 > $O/phases.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "mas::" --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --mode env --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_sq.log 2>&1
echo "sq rc=$?"
