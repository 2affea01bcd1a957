"""Summarise a rocprofv3 --stats kernel table (run_kernel_stats.csv) into text.
usage: python profiles/stats_summary.py <run_kernel_stats.csv> <out.txt> "<header line>" [trace.csv timed]
The table's columns cover the whole profiled run (pre-roll, warm-up and timed
steps).  With the kernel trace and the number of timed steps, adds
  - us_per_step: each kernel's time inside the timed window (from the k_pre
    launch of the first timed env step to the end of the trace) divided by
    the timed steps -- the per-step cost the bench's ms_per_step contains
    (round 4's column divided whole-run totals by the step argument instead);
  - calls_in_window;
  - the duration of the env step's launch group (k_pre start -> last env
    kernel end, what bench.py times with HIP events as `roofline.kernel_ms`)
    over the last `timed` steps."""
import csv
import sys


def _is_pre(n):
    return 'mas::k_pre<' in n or 'mas::k_pre_lanes<' in n


def step_spans(rows):
    """k_pre start -> the last end of the step's env kernels (mas::k_*, not
    the policy's mas::pol::*) before the next k_pre: with the split step the
    side streams' kernels can end after the caller's last kernel."""
    spans, t0, t1 = [], None, None
    for r in rows:
        n = r['Kernel_Name']
        if _is_pre(n):
            if t0 is not None and t1 is not None:
                spans.append((t1 - t0) / 1e6)
            t0, t1 = int(r['Start_Timestamp']), None
        elif t0 is not None and 'mas::k_' in n and 'mas::pol::' not in n and 'k_stats' not in n:
            t1 = max(t1 or 0, int(r['End_Timestamp']))
    if t0 is not None and t1 is not None:
        spans.append((t1 - t0) / 1e6)
    return spans


def window_per_kernel(rows, timed):
    """{kernel name[:100]: (total ns, calls)} inside the timed window."""
    pre = [int(r['Start_Timestamp']) for r in rows if _is_pre(r['Kernel_Name'])]
    w0 = pre[-timed]
    out = {}
    for r in rows:
        if int(r['Start_Timestamp']) < w0:
            continue
        k = r['Kernel_Name'][:100]
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        t, c = out.get(k, (0, 0))
        out[k] = (t + d, c + 1)
    return out


def main(path, out, header, trace=None, timed=None):
    rows = list(csv.DictReader(open(path)))
    tr = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp'])) if trace else None
    k = int(timed) if timed else 0
    win = window_per_kernel(tr, k) if tr else {}
    lines = ['# ' + header,
             '# durations in ns over the whole profiled run; one row per kernel name (first 100 chars)' +
             (f'; us_per_step / calls_in_window: the timed window of {k} steps only' if tr else ''),
             'name | calls | total_ns | avg_ns | min_ns | max_ns | pct' +
             (' | us_per_step | calls_in_window' if tr else '')]
    for r in rows:
        x = [r['Name'][:100], r['Calls'], r['TotalDurationNs'], r['AverageNs'], r['MinNs'], r['MaxNs'],
             r['Percentage'][:6]]
        if tr:
            t, c = win.get(r['Name'][:100], (0, 0))
            x += ['%.1f' % (t / 1e3 / k), str(c)]
        lines.append(' | '.join(x))
    if tr:
        sp = step_spans(tr)
        lines.append('# mas_step launch group (k_pre start -> last env kernel end): mean %.4f ms over the last %d steps '
                     '(the timed region), %.4f ms over all %d steps' % (sum(sp[-k:]) / k, k, sum(sp) / len(sp), len(sp)))
        tot = sum(t for t, _ in win.values())
        lines.append('# kernel time inside the timed window: %.1f us per step (all streams summed)' % (tot / 1e3 / k))
    open(out, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main(*sys.argv[1:])
