"""Idle time of the GPU inside the bench's timed window, from a rocprofv3
kernel trace of `KFAC_PROFILE_MARKER=1 python bench.py ...`.

    python scripts/probes/trace_gaps.py <kernel_trace.csv> [min_gap_us]

Prints the union of busy intervals (over all queues), the idle total, and the
idle gaps longer than `min_gap_us` with the kernels on both sides -- host-bound
stretches (eager launches, Python, host syncs) show up as gaps.  The inverse
step is located by its tridiagonal-reduction kernels (red_*).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if 'sleep' in r[2].lower() or 'spin' in r[2].lower()]
    if len(marks) >= 2:
        rows = rows[marks[0] + 1:marks[1]]
    elif marks:
        rows = rows[marks[0] + 1:]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy, gaps = 0, []
    cur_s, cur_e, last = rows[0][0], rows[0][1], rows[0][2]
    for s, e, name in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, last, name))
            cur_s, cur_e = s, e
        elif e > cur_e:
            cur_e = e
        if e >= cur_e:
            last = name
    busy += cur_e - cur_s
    red = [r for r in rows if 'red_' in r[2]]
    inv0 = red[0][0] if red else None
    inv1 = red[-1][1] if red else None
    span = (t1 - t0) / 1e6
    print('window %.2f ms, busy %.2f ms, idle %.2f ms (%d dispatches)' % (
        span, busy / 1e6, span - busy / 1e6, len(rows)))
    if red:
        def idle_in(a, b):
            return sum(g for g, at, _, _ in gaps if a <= at < b) / 1e6
        print('inverse-step reduction span %.2f ms; idle before it %.2f ms, during %.2f ms, '
              'after %.2f ms' % ((inv1 - inv0) / 1e6, idle_in(t0, inv0), idle_in(inv0, inv1),
                                 idle_in(inv1, t1 + 1)))
    big = sorted((g for g in gaps if g[0] / 1e3 >= min_gap), key=lambda g: -g[0])
    print('%d gaps >= %.0f us, %.2f ms in total; the 40 longest:' % (
        len(big), min_gap, sum(g[0] for g in big) / 1e6))
    for g, at, a, b in big[:40]:
        print('  %8.1f us at %9.3f ms  after %-50.50s before %-50.50s' % (
            g / 1e3, (at - t0) / 1e6, a, b))


if __name__ == '__main__':
    main()
