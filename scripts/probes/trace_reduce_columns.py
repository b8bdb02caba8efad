"""Per-column view of the one-stage tridiagonal reduction (csrc/eig_reduce.hip)
from a rocprofv3 kernel trace: the F / S / U launches of the LAST inverse
update in the trace, binned by column, with the S launches' streamed bytes
(32 KB per half-tile workgroup) and bandwidth.

    rocprofv3 --kernel-trace -d /tmp/t -o run --output-format csv -- \
        python3 scripts/probes/probe_eig_resnet50.py default
    python3 scripts/probes/trace_reduce_columns.py /tmp/t/.../run_kernel_trace.csv [runs]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            kind = ('S' if 'red_symv' in name else 'F' if 'red_fin' in name
                    else 'U' if 'red_upd' in name else None)
            if kind is None:
                continue
            grid = int(r.get('Grid_Size_X') or r.get('Grid_Size') or 0)
            wg = int(r.get('Workgroup_Size_X') or r.get('Workgroup_Size') or 256)
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), kind, grid // max(wg, 1)))
    rows.sort()
    nf = sum(1 for r in rows if r[2] == 'F')
    per = nf // runs
    # the last run: its F launches are columns 0 .. per-1
    fseen, start = 0, 0
    for i, r in enumerate(rows):
        if r[2] == 'F':
            if fseen == nf - per:
                start = i
                break
            fseen += 1
    last = rows[start:]
    span = (last[-1][1] - last[0][0]) / 1e6
    print('reduction launches in the last run: %d (F %d), span %.2f ms' % (len(last), per, span))
    bins = 16
    width = max(1, per // bins)
    col = -1
    acc = {}
    for t0, t1, kind, wgs in last:
        if kind == 'F':
            col += 1
        b = min(col // width, bins - 1)
        a = acc.setdefault(b, {'F': [0.0, 0], 'S': [0.0, 0, 0], 'U': [0.0, 0], 'gap': 0.0})
        a[kind][0] += (t1 - t0) / 1e3
        a[kind][1] += 1
        if kind == 'S':
            a['S'][2] += wgs
    tot = {'F': 0.0, 'S': 0.0, 'U': 0.0}
    print('%-13s %8s %8s %8s %8s %9s %9s' % ('columns', 'F ms', 'S ms', 'U ms', 'F us/col',
                                              'S us/col', 'S GB/s'))
    for b in sorted(acc):
        a = acc[b]
        sb = a['S'][2] * 32768.0
        for k in tot:
            tot[k] += a[k][0] / 1e3
        print('%5d-%-7d %8.2f %8.2f %8.2f %8.2f %9.2f %9.0f' % (
            b * width, (b + 1) * width - 1, a['F'][0] / 1e3, a['S'][0] / 1e3, a['U'][0] / 1e3,
            a['F'][0] / max(a['F'][1], 1), a['S'][0] / max(a['S'][1], 1),
            sb / max(a['S'][0] * 1e3, 1e-9)))
    print('total  F %.2f ms  S %.2f ms  U %.2f ms  (kernel time; span %.2f ms)' % (
        tot['F'], tot['S'], tot['U'], span))


if __name__ == '__main__':
    main()
