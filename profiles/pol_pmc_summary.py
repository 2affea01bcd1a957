"""Per-kernel averages (per dispatch) of the rocprofv3 PMC passes that
`scripts/gpu_round.sh <tag> polpmc` collects over scripts/policy_bench.py.
usage: python profiles/pol_pmc_summary.py <gpurun_out/polpmc> <out.json>
FETCH_SIZE / WRITE_SIZE are KB (reported here in bytes)."""
import collections
import csv
import json
import os
import sys


def main(d, out):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ('fetch', 'write', 'p1', 'p2'):
        path = os.path.join(d, sub, 'run_counter_collection.csv')
        if not os.path.exists(path):  # (the gpu_round.sh step's directory names)
            path = os.path.join(d, 'pol_' + sub, 'run_counter_collection.csv')
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')
            acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    res = {}
    for k, cs in sorted(acc.items()):
        res[k] = {}
        for c, v in sorted(cs.items()):
            m = sum(v) / len(v)
            res[k][c + ('_bytes' if c in ('FETCH_SIZE', 'WRITE_SIZE') else '')] = m * 1024 if c in ('FETCH_SIZE', 'WRITE_SIZE') else m
        res[k]['dispatches'] = max(len(v) for v in cs.values())
    json.dump(res, open(out, 'w'), indent=1)
    for k, v in res.items():
        print(k, {c: f'{x:.4g}' for c, x in v.items()})


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
