#!/bin/bash
# A/B of the side stream's priority (MAS_SIDE_PRIO=0 default priority, 1 highest):
# driver-window and env-only benches, alternating, each under its own limit
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prio; mkdir -p $O; cd $R
for r in a b; do
  for p in 0 1; do
    MAS_SIDE_PRIO=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_p${p}_$r.log 2>&1 || exit $?
    MAS_SIDE_PRIO=$p timeout -k 10 200 python bench.py --mode env --config ffa4 --steps 50 --warmup 10 --no-cpu-baseline > $O/ffa_p${p}_$r.log 2>&1 || exit $?
  done
  echo "round $r ok"
done
MAS_SIDE_PRIO=1 timeout -k 10 200 python -u scripts/toi_tail_probe.py 65536 40 > $O/probe_p1.log 2>&1 || exit $?
echo ok
