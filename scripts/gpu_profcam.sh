#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profcam
mkdir -p $O
cd $R
timeout -k 10 200 python profiles/prof_general.py > $O/prof_general.log 2>&1 && timeout -k 10 300 python profiles/prof_general.py 65536 20 --ppo > $O/prof_general_ppo.log 2>&1 || exit $?
echo ok
