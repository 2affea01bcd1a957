"""Summarise scripts/gpu_ab_env.sh: bench ms/step and steady-state per-kernel
times (median over the last half of the trace) for each variant.
usage: python profiles/ab_env.py gpurun_out/abenv base variant..."""
import collections
import csv
import json
import os
import statistics
import sys


def main(d, *names):
    for v in names:
        line = [l for l in open(os.path.join(d, v + '.log')) if l.startswith('{')]
        ms = json.loads(line[-1])['ms_per_step'] if line else float('nan')
        rows = list(csv.DictReader(open(os.path.join(d, v, 'run_kernel_trace.csv'))))
        rows.sort(key=lambda r: int(r['Start_Timestamp']))
        rows = rows[len(rows) // 2:]
        t = collections.defaultdict(list)
        for r in rows:
            if 'mas::' in r['Kernel_Name']:
                k = r['Kernel_Name'].split('<')[0].replace('void mas::', '')
                t[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
        ks = {k: round(statistics.median(x), 1) for k, x in t.items()}
        per_step = sum(statistics.median(x) * len(x) for x in t.values()) / max(1, len(t.get('k_pre', [1])))
        print(f'{v:8s} ms/step {ms:.4f}  env kernels/step {per_step:.1f} us  {ks}')


if __name__ == '__main__':
    main(*sys.argv[1:])
