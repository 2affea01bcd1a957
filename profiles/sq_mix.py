"""Per-kernel instruction mix of the env-step kernels from one rocprofv3 PMC
pass (SQ_WAVES, SQ_INSTS_VALU / SALU / VMEM_RD / VMEM_WR / LDS,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES) over bench.py's last `steps` env steps:
instructions per wave and wave-cycles per wave, averaged per kernel.
usage: python profiles/sq_mix.py <counter_collection.csv> [steps]"""
import collections
import csv
import sys


def main(path, steps=20):
    steps = int(steps)
    rows = [r for r in csv.DictReader(open(path)) if 'mas::' in r['Kernel_Name'] and '::pol::' not in r['Kernel_Name']]
    disp = collections.defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r['Dispatch_Id'])
        disp[d][r['Counter_Name']] = disp[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
        names[d] = r['Kernel_Name'].split('<')[0].replace('void mas::', '')
    order = sorted(disp)
    starts = [d for d in order if names[d] in ('k_pre', 'k_pre_lanes')]
    keep = set(d for d in order if d >= starts[-steps]) if len(starts) >= steps else set(order)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in keep:
        for c, v in disp[d].items():
            agg[names[d]][c] += v
        agg[names[d]]['launches'] += 1
    cols = ['SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR', 'SQ_INSTS_LDS', 'SQ_WAVE_CYCLES']
    print('%-12s %8s %9s ' % ('kernel', 'launches', 'waves/l') + ' '.join('%12s' % c.replace('SQ_', '').replace('INSTS_', '')
                                                                         for c in cols) + '   (per wave)')
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES']):
        w = max(a['SQ_WAVES'], 1.0)
        print('%-12s %8d %9.0f ' % (k, a['launches'], w / a['launches']) + ' '.join('%12.0f' % (a[c] / w) for c in cols))


if __name__ == '__main__':
    main(*sys.argv[1:])
