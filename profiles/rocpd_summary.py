"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a text table.
usage: python profiles/rocpd_summary.py <run_results.db> <out.txt> "<header line>" """
import sqlite3
import sys


def main(db, out, header):
    c = sqlite3.connect(db)
    rows = ['# ' + header, '# durations in ns; one row per kernel name (first 110 chars)',
            'name | calls | total_ns | avg_ns | min_ns | max_ns | arch_vgpr | accum_vgpr | scratch_B/lane | lds_B']
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), max(vgpr_count), "
         "max(accum_vgpr_count), max(scratch_size), max(lds_size) from kernels group by name order by sum(duration) desc")
    for r in c.execute(q):
        r = (r[0][:110],) + tuple(round(x, 1) if isinstance(x, float) else x for x in r[1:])
        rows.append(' | '.join(str(x) for x in r))
    open(out, 'w').write('\n'.join(rows) + '\n')
    print('\n'.join(rows))


if __name__ == '__main__':
    main(*sys.argv[1:4])
