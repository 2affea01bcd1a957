"""Summarise a rocprofv3 --stats kernel table (run_kernel_stats.csv) into text.
usage: python profiles/stats_summary.py <run_kernel_stats.csv> <out.txt> "<header line>" [steps]
With [steps], adds the per-step share (total / steps) of each kernel."""
import csv
import sys


def main(path, out, header, steps=None):
    rows = list(csv.DictReader(open(path)))
    lines = ['# ' + header, '# durations in ns; one row per kernel name (first 100 chars)',
             'name | calls | total_ns | avg_ns | min_ns | max_ns | pct' + (' | us_per_step' if steps else '')]
    for r in rows:
        x = [r['Name'][:100], r['Calls'], r['TotalDurationNs'], r['AverageNs'], r['MinNs'], r['MaxNs'],
             r['Percentage'][:6]]
        if steps:
            x.append('%.1f' % (float(r['TotalDurationNs']) / 1e3 / float(steps)))
        lines.append(' | '.join(x))
    open(out, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main(*sys.argv[1:])
