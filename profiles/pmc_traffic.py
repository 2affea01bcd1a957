"""HBM traffic of one mas_step from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected in separate runs, MI355X_MICROARCH.md HBM section).

usage: python profiles/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json> <workload>

Sums the env-step kernels (mas::k_*, excluding k_seed/k_stats and the
policy kernels mas::pol::*) per step
(steps = number of k_pre dispatches).  FETCH_SIZE / WRITE_SIZE are in KB.
The guide's x2 FETCH_SIZE correction is calibrated for 16-B-per-lane
streaming reads; the state loads here are 4 B per lane (uncalibrated width),
so the raw value is reported and the corrected one alongside it."""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter or 'mas::' not in r['Kernel_Name'] or '::pol::' in r['Kernel_Name']:
            continue
        k = r['Kernel_Name'].split('<')[0].replace('void mas::', '')
        acc[k] += float(r['Counter_Value']) * 1024.0
        n[k] += 1
    return acc, n


def main(fetch_csv, write_csv, out, workload):
    f, nf = per_kernel(fetch_csv, 'FETCH_SIZE')
    w, nw = per_kernel(write_csv, 'WRITE_SIZE')
    steps = max(nf.get('k_pre', 0), 1)
    fetch = sum(f.values()) / steps
    write = sum(w.values()) / steps
    res = {
        'workload': workload, 'steps_profiled': steps,
        'fetch_bytes_per_step': fetch, 'write_bytes_per_step': write,
        'traffic_bytes_per_step': fetch + write,
        'traffic_bytes_per_step_fetch_x2': 2 * fetch + write,
        'per_kernel_fetch_bytes_per_launch': {k: f[k] / nf[k] for k in f},
        'per_kernel_write_bytes_per_launch': {k: w[k] / nw[k] for k in w},
        'note': 'FETCH_SIZE+WRITE_SIZE (KB->B) summed over the env-step kernels per mas_step; '
                'dword state loads (4 B/lane): the x2 FETCH correction of the guide is calibrated for 16-B lanes only',
    }
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:5])
