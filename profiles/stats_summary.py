"""Summarise a rocprofv3 --stats kernel table (run_kernel_stats.csv) into text.
usage: python profiles/stats_summary.py <run_kernel_stats.csv> <out.txt> "<header line>" [steps] [trace.csv timed]
With [steps], adds the per-step share (total / steps) of each kernel.  With
the kernel trace and the number of timed steps, adds the duration of the env
step's launch group (k_pre start -> k_obs end, what bench.py times with HIP
events as `roofline.kernel_ms`) over the last `timed` steps."""
import csv
import sys


def step_spans(trace):
    """k_pre start -> the last end of the step's env kernels (mas::k_*, not
    the policy's mas::pol::*) before the next k_pre: with the split step the
    side stream's kernels can end after the caller's k_obs."""
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp']))
    spans, t0, t1 = [], None, None
    for r in rows:
        n = r['Kernel_Name']
        if 'mas::k_pre<' in n or 'mas::k_pre_lanes<' in n:
            if t0 is not None and t1 is not None:
                spans.append((t1 - t0) / 1e6)
            t0, t1 = int(r['Start_Timestamp']), None
        elif t0 is not None and 'mas::k_' in n and 'mas::pol::' not in n and 'k_stats' not in n:
            t1 = max(t1 or 0, int(r['End_Timestamp']))
    if t0 is not None and t1 is not None:
        spans.append((t1 - t0) / 1e6)
    return spans


def main(path, out, header, steps=None, trace=None, timed=None):
    rows = list(csv.DictReader(open(path)))
    lines = ['# ' + header, '# durations in ns; one row per kernel name (first 100 chars)',
             'name | calls | total_ns | avg_ns | min_ns | max_ns | pct' + (' | us_per_step' if steps else '')]
    for r in rows:
        x = [r['Name'][:100], r['Calls'], r['TotalDurationNs'], r['AverageNs'], r['MinNs'], r['MaxNs'],
             r['Percentage'][:6]]
        if steps:
            x.append('%.1f' % (float(r['TotalDurationNs']) / 1e3 / float(steps)))
        lines.append(' | '.join(x))
    if trace:
        sp = step_spans(trace)
        k = int(timed)
        lines.append('# mas_step launch group (k_pre start -> last env kernel end): mean %.4f ms over the last %d steps '
                     '(the timed region), %.4f ms over all %d steps' % (sum(sp[-k:]) / k, k, sum(sp) / len(sp), len(sp)))
    open(out, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main(*sys.argv[1:])
