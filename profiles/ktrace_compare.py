"""Per-step kernel time of the env step from rocprofv3 kernel traces (A/B of
builds on the same workload: the builds are bit-identical, so every trace
replays the same envs).  For the last `steps` env steps (k_pre .. k_obs
launch groups): mean / p50 / p90 / max per kernel family, and the launch
group span.
usage: python profiles/ktrace_compare.py <run_kernel_trace.csv>... [--steps 128]"""
import csv
import sys

import numpy as np

FAMILIES = [('general', ('k_gen<', 'k_gen_solve<', 'k_toi_list<', 'k_gen_toi<')), ('k_pre', ('k_pre<',)),
            ('k_phys_fast', ('k_phys_fast<',)), ('k_boxes', ('k_boxes<',)), ('k_cameras', ('k_cameras<',)),
            ('k_post', ('k_post<',)), ('k_reset', ('k_reset<',)), ('k_obs', ('k_obs<',))]


def steps_of(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    steps, cur = [], None
    for r in rows:
        n = r['Kernel_Name']
        if 'mas::' not in n or '::pol::' in n:
            continue
        if 'mas::k_pre<' in n:
            cur = {'t0': int(r['Start_Timestamp']), 'k': {}}
            steps.append(cur)
        if cur is None:
            continue
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        for fam, keys in FAMILIES:
            if any('mas::' + k in n for k in keys):
                cur['k'][fam] = cur['k'].get(fam, 0.0) + d
        if 'mas::k_obs<' in n:
            cur['span'] = (int(r['End_Timestamp']) - cur['t0']) / 1e3
    return [s for s in steps if 'span' in s]


def main():
    args = sys.argv[1:]
    n = 128
    if '--steps' in args:
        i = args.index('--steps')
        n = int(args[i + 1])
        del args[i:i + 2]
    for path in args:
        st = steps_of(path)[-n:]
        print(f'{path}: {len(st)} steps (us per step: mean p50 p90 max)')
        for fam, _ in FAMILIES + [('span', None)]:
            v = np.array([s['span'] if fam == 'span' else s['k'].get(fam, 0.0) for s in st])
            print(f'  {fam:12s} {v.mean():8.1f} {np.percentile(v, 50):8.1f} {np.percentile(v, 90):8.1f} {v.max():8.1f}')


if __name__ == '__main__':
    main()
