"""Summarise gpurun_ab.sh output: per-variant kernel averages (us) and bench line."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/ab'
for d in sorted(glob.glob(os.path.join(root, '*/')), key=lambda p: int(os.path.basename(p.rstrip('/')).split('_')[0])):
    name = os.path.basename(d.rstrip('/'))
    ks = {}
    for r in csv.DictReader(open(os.path.join(d, 'run_kernel_stats.csv'))):
        if 'mas::' in r['Name']:
            ks[r['Name'].split('<')[0].replace('void mas::', '')] = float(r['AverageNs']) / 1000
    ms = float('nan')
    for ln in open(d.rstrip('/') + '.log'):
        if ln.startswith('{"metric"'):
            ms = json.loads(ln)['ms_per_step']
    tot = sum(ks.values())
    print(f'{name:14s} ms/step={ms:.3f} kernels_sum={tot:.1f}us ' + ' '.join(f'{k}={v:.1f}' for k, v in sorted(ks.items())))
