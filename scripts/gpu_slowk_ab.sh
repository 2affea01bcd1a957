#!/bin/bash
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/slowk; mkdir -p $O; cd $R
for k in 4 2 3 8 4; do
  MAS_SLOW_K=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_k$k.log 2>&1 || exit $?
  MAS_SLOW_K=$k timeout -k 10 200 python bench.py --mode env --steps 128 --warmup 64 --no-cpu-baseline > $O/env_k$k.log 2>&1 || exit $?
  echo "k=$k ok"
done
