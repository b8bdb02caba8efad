"""Per-queue timing of the tridiagonal-reduction launch chains in a rocprofv3
kernel trace of probe_eig_stream_ends.py (or any run of the eigensolver):
for each hardware queue that ran red_* kernels, over the LAST solve in the
trace, the chain's span, the summed kernel durations and the summed gaps
between one launch's end and the next launch's start on that queue, per
quarter of the chain -- whether a concurrent chain lengthens this chain's
kernels or the gaps between them.

    python3 scripts/probes/trace_reduce_queues.py <kernel_trace.csv> [solves]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    solves = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    by_q = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if '_red_' in r['Kernel_Name'] or 'red_fin' in r['Kernel_Name'] or \
                    'red_symv' in r['Kernel_Name'] or 'red_upd' in r['Kernel_Name']:
                q = r.get('Queue_Id') or r.get('Stream_Id') or '0'
                by_q[q].append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                                r['Kernel_Name']))
    for q, rows in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        rows.sort()
        n = len(rows) // solves
        last = rows[-n:] if n else rows
        t0 = last[0][0]
        print('queue %s: %d reduction launches (%d per solve), last solve span %.2f ms' % (
            q, len(rows), n, (last[-1][1] - t0) / 1e6))
        k = len(last)
        for part in range(4):
            seg = last[part * k // 4:(part + 1) * k // 4]
            dur = sum(e - s for s, e, _ in seg) / 1e6
            gaps = sum(max(0, seg[i][0] - seg[i - 1][1]) for i in range(1, len(seg))) / 1e6
            kinds = collections.Counter(('fin' if 'fin' in nm else 'symv' if 'symv' in nm else 'upd')
                                        for _, _, nm in seg)
            mean = {kd: sum(e - s for s, e, nm in seg if kd in nm) / max(1, c) / 1e3
                    for kd, c in kinds.items()}
            print('  quarter %d: %5d launches from %7.2f ms: kernels %6.2f ms, gaps %6.2f ms; '
                  'mean us %s' % (part, len(seg), (seg[0][0] - t0) / 1e6, dur, gaps,
                                  ' '.join('%s %.2f' % kv for kv in sorted(mean.items()))))


if __name__ == '__main__':
    main()
