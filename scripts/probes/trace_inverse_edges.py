"""The kernels around the inverse update in a rocprofv3 kernel trace of the
bench window: everything from the window start to the first tridiagonal-
reduction launch, and from the last one on for `after_ms`, one line per
dispatch with the idle gap before it -- where the inverse step's host-bound
stretches (eager launches, Python) sit.

    python3 scripts/probes/trace_inverse_edges.py <kernel_trace.csv> [after_ms]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    after_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if 'sleep' in r[2].lower() or 'spin' in r[2].lower()]
    if len(marks) >= 2:
        rows = rows[marks[0] + 1:marks[1]]
    red = [i for i, r in enumerate(rows) if 'red_' in r[2]]
    if not red:
        print('no reduction launches in the window')
        return
    t0 = rows[0][0]

    def dump(lo, hi):
        prev_end = rows[lo - 1][1] if lo > 0 else rows[lo][0]
        for s, e, name in rows[lo:hi]:
            gap = max(0, s - prev_end) / 1e3
            print('%9.3f ms  gap %8.1f us  dur %8.1f us  %s' % (
                (s - t0) / 1e6, gap, (e - s) / 1e3, name[:90]))
            prev_end = max(prev_end, e)

    print('== window start .. first reduction launch')
    dump(0, red[0] + 1)
    end = rows[red[-1]][1] + after_ms * 1e6
    hi = red[-1] + 1
    while hi < len(rows) and rows[hi][0] < end:
        hi += 1
    print('== last reduction launch .. +%.0f ms' % after_ms)
    dump(red[-1], hi)


if __name__ == '__main__':
    main()
