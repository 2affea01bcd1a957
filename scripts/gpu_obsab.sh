cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/obsab && for v in base obsskip1 obsskip2; do
  L=""; [ $v != base ] && L="--lib gym-ma-survival-2d_amd/masurvival/_lib/libmas_$v.so"
  timeout -k 10 200 python bench.py --mode env --no-cpu-baseline $L > gpurun_out/obsab/$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/obsab/$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['config']['breakdown_ms']['env_step'])"
done
