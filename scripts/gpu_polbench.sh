#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/polbench
mkdir -p $O
cd $R
L=gym-ma-survival-2d_amd/masurvival/_lib
timeout -k 10 300 python scripts/policy_bench.py $L/libmas_old.so $L/libmas_old.so $L/libmas_dma.so $L/libmas_old.so $L/libmas_dma.so > $O/polbench.log 2>&1 || exit $?
echo ok
