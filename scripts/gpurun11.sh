#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
$R/scripts/gpurun_ab.sh base nofast base
