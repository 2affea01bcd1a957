#!/bin/bash
# r04w: the slow split (MAS_SPLIT=2, default) vs one stream (MAS_SPLIT=0)
# with the fused general-path launch: driver-window benches, alternating
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
for sp in 2 0 2 0; do
  MAS_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/bench_driver_sp$sp.json 2>> $O/err.log || exit $?
done
for sp in 2 0; do
  MAS_SPLIT=$sp timeout -k 10 300 python -u bench.py --mode env --no-cpu-baseline >> $O/bench_env_sp$sp.json 2>> $O/err.log || exit $?
done
echo ok
