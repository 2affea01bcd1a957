"""HBM traffic of one mas_step from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected in separate runs, MI355X_MICROARCH.md HBM section).

usage: python profiles/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>
                                      <workload key> [last_steps]

Sums the env-step kernels (mas::k_*, excluding k_seed/k_stats and the
policy kernels mas::pol::*) per step.  A step is the launch group that starts
at a k_pre dispatch (dispatch order); with last_steps only the last that many
steps count -- bench.py's timed window, so the traffic comes from the same
regime as the bench line's achieved bandwidth (not the pre-roll's episode
start).  FETCH_SIZE / WRITE_SIZE are in KB.  The guide's x2 FETCH_SIZE
correction is calibrated for 16-B-per-lane streaming reads; most state loads
here are 4 B per lane (uncalibrated width), so the raw value is reported and
the corrected one alongside it."""
import collections
import csv
import json
import sys


def per_step(path, counter, last):
    rows = [r for r in csv.DictReader(open(path))
            if r['Counter_Name'] == counter and 'mas::' in r['Kernel_Name'] and '::pol::' not in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    steps = []
    for r in rows:
        k = r['Kernel_Name'].split('<')[0].replace('void mas::', '')
        if k in ('k_pre', 'k_pre_lanes'):
            steps.append(collections.defaultdict(float))
        if not steps or k in ('k_seed', 'k_stats'):
            continue
        steps[-1][k] += float(r['Counter_Value']) * 1024.0
    if last:
        steps = steps[-int(last):]
    tot = collections.defaultdict(float)
    for s in steps:
        for k, v in s.items():
            tot[k] += v
    n = max(len(steps), 1)
    return {k: v / n for k, v in tot.items()}, len(steps)


def kernel_bytes(path, counter, name):
    """The counter's bytes (KB -> B) summed over every dispatch of kernel `name`
    (e.g. k_stats, the calibration kernel of bench.py's live_traffic)."""
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter and (name + '(') in r['Kernel_Name']:
            tot += float(r['Counter_Value']) * 1024.0
    return tot


def main(fetch_csv, write_csv, out, workload, last=None):
    f, nf = per_step(fetch_csv, 'FETCH_SIZE', last)
    w, nw = per_step(write_csv, 'WRITE_SIZE', last)
    fetch, write = sum(f.values()), sum(w.values())
    res = {
        'workload': workload, 'steps_profiled': min(nf, nw),
        'fetch_bytes_per_step': fetch, 'write_bytes_per_step': write,
        'traffic_bytes_per_step': fetch + write,
        'traffic_bytes_per_step_fetch_x2': 2 * fetch + write,
        'per_kernel_fetch_bytes_per_step': dict(f),
        'per_kernel_write_bytes_per_step': dict(w),
        'note': 'FETCH_SIZE+WRITE_SIZE (KB->B) summed over the env-step kernels per mas_step'
                + (f' over the last {last} steps (the bench timed window)' if last else '')
                + '; mostly dword state loads (4 B/lane): the x2 FETCH correction of the guide is calibrated '
                  'for 16-B lanes only',
    }
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:6])
