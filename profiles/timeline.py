"""Per-step timeline of the env step's kernels from a rocprofv3 kernel trace
(run_kernel_trace.csv): for each of the last `steps` launch groups (k_pre
start -> last env kernel end), every env kernel's queue, start and end
relative to the k_pre start (us), then per-kernel means.
usage: python profiles/timeline.py <run_kernel_trace.csv> [steps] [--show K]"""
import collections
import csv
import sys


def groups(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    out, cur = [], None
    for r in rows:
        n = r['Kernel_Name']
        if 'mas::' not in n or '::pol::' in n or 'k_stats' in n or 'k_seed' in n:
            continue
        short = n.split('(')[0].replace('void mas::', '').replace('mas::Cap<4, 4, 4, 4, 4>', 'C')
        if 'k_pre_lanes<' in n:
            cur = {'t0': int(r['Start_Timestamp']), 'k': []}
            out.append(cur)
        if cur is None:
            continue
        q = r.get('Queue_Id', r.get('Stream_Id', '?'))
        cur['k'].append((short, q, (int(r['Start_Timestamp']) - cur['t0']) / 1e3,
                         (int(r['End_Timestamp']) - cur['t0']) / 1e3))
    return out


def main():
    a = [x for x in sys.argv[1:] if not x.startswith('--')]
    steps = int(a[1]) if len(a) > 1 else 20
    show = int(sys.argv[sys.argv.index('--show') + 1]) if '--show' in sys.argv else 3
    g = groups(a[0])[-steps:]
    for s in g[:show]:
        print('step:')
        for k in s['k']:
            print(f'  {k[0]:45s} q{k[1]:>3} {k[2]:8.1f} {k[3]:8.1f}  ({k[3] - k[2]:.1f})')
    agg = collections.defaultdict(list)
    span = []
    for s in g:
        span.append(max(k[3] for k in s['k']))
        seen = collections.Counter()
        for k in s['k']:
            key = f'{k[0]}#{seen[k[0]]}'
            seen[k[0]] += 1
            agg[key].append(k)
    print(f'# mean over {len(g)} steps: kernel, start, end, duration (us)')
    for key, v in agg.items():
        n = len(v)
        print(f'  {key:47s} n={n:3d} {sum(x[2] for x in v) / n:8.1f} {sum(x[3] for x in v) / n:8.1f} '
              f'{sum(x[3] - x[2] for x in v) / n:8.1f}')
    print(f'# span mean {sum(span) / len(span):.1f} us')


if __name__ == '__main__':
    main()
