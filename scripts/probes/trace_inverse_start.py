"""Where the inverse step's eigensolve starts relative to its forward/backward
(rocprofv3 --kernel-trace CSV of bench.py under KFAC_PROFILE_MARKER=1).

    python scripts/probes/trace_inverse_start.py <kernel_trace.csv>

Prints, for the first inverse step of the timed window: the first and last
dispatch of the step, the first tridiagonal-reduction kernel, the last model
(conv / BN) kernel of the backward, per-queue dispatch counts, and the
kernels around the first reduction launch (time offset, queue, name)."""
import collections
import csv
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '')
    return n[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'sleep' in r['Kernel_Name'].lower()
             or 'spin' in r['Kernel_Name'].lower()]
    lo = marks[-2] if len(marks) >= 2 else 0
    hi = marks[-1] if len(marks) >= 2 else len(rows)
    win = rows[lo + 1:hi]
    red = [i for i, r in enumerate(win) if 'red_' in r['Kernel_Name']]
    if not red:
        print('no reduction kernel in the window')
        return
    i0 = red[0]
    # the inverse step starts after the previous plain step: walk back to the
    # first kernel after a >= 0.3 ms idle gap before the first reduction
    t = lambda r: int(r['Start_Timestamp'])
    e = lambda r: int(r['End_Timestamp'])
    s = i0
    while s > 0 and t(win[s]) - e(win[s - 1]) < 300000:
        s -= 1
    step0 = t(win[s])
    qcol = 'Queue_Id' if 'Queue_Id' in win[0] else None
    model = [r for r in win[s:i0 + 20000] if 'bn_' in r['Kernel_Name'] or 'igemm' in r['Kernel_Name']
             or 'ck::' in r['Kernel_Name'] or 'conv' in r['Kernel_Name'].lower()]
    last_model = max(e(r) for r in model) if model else step0
    reds = [win[i] for i in red]
    print('inverse step from %.3f ms (window offset)' % ((step0 - t(win[0])) / 1e6))
    print('first reduction kernel at +%.3f ms; last model kernel ends +%.3f ms; '
          'last reduction kernel ends +%.3f ms' % ((t(win[i0]) - step0) / 1e6,
                                                  (last_model - step0) / 1e6,
                                                  (max(e(r) for r in reds) - step0) / 1e6))
    if qcol:
        c = collections.Counter(r[qcol] for r in reds)
        print('reduction dispatches per queue:', dict(c))
        firsts = {}
        for r in reds:
            firsts.setdefault(r[qcol], t(r))
        print('first reduction dispatch per queue: ' + ', '.join(
            'q%s +%.3f' % (q, (v - step0) / 1e6) for q, v in firsts.items()))
    for r in win[max(s, i0 - 12):i0 + 12]:
        print('  +%8.3f  q%-4s %s' % ((t(r) - step0) / 1e6, r.get(qcol, '?') if qcol else '?',
                                     short(r['Kernel_Name'])))


if __name__ == '__main__':
    main()
