#!/bin/bash
# A/B of variant libraries (masurvival/_lib/libmas_<v>.so) on the env-only and
# the driver-shaped PPO bench.   scripts/gpu_libab.sh <tag> <v1> <v2> ...
# (v = main: libmas.so itself)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
for rep in 1 2; do for v in "$@"; do
  L="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
  [ "$v" = main ] && L=""  # the in-tree product library
  timeout -k 10 200 python bench.py --mode env --no-cpu-baseline $L > $O/env_$v.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $L > $O/drv_$v.log 2>&1 || exit 1
  python - "$v" "$O" <<'PY'
import json, sys
v, o = sys.argv[1], sys.argv[2]
d = [json.loads(l) for k in ('env', 'drv') for l in open(f'{o}/{k}_{v}.log') if l.startswith('{')]
print(v, 'env-only env_step %.4f ms' % d[0]['config']['breakdown_ms']['env_step'],
      '| driver env_step %.4f ms, ms/step %.4f' % (d[1]['config']['breakdown_ms']['env_step'], d[1]['ms_per_step']))
PY
done; done
