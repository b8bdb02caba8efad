"""Per-launch view of the fused BatchNorm kernels (csrc/bn.hip) of ONE step
from a rocprofv3 kernel trace of the bench: the BN launches of the last
`per_step` in the timed window (between the KFAC_PROFILE_MARKER spin kernels),
in launch order, with their grids and durations, and the per-kind totals.

    python3 scripts/probes/bn_layer_stats.py <kernel_trace.csv> [per_step]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    for k in ('bn_stats', 'bn_finalize', 'bn_apply_kernel<true, true>', 'bn_apply_kernel<true, false>',
              'bn_apply_kernel<false, true>', 'bn_apply_kernel<false, false>',
              'bn_bwd_reduce_kernel<true>', 'bn_bwd_reduce_kernel<false>', 'bn_bwd_finalize',
              'bn_bwd_apply_kernel<true, true>', 'bn_bwd_apply_kernel<true, false>',
              'bn_bwd_apply_kernel<false, true>', 'bn_bwd_apply_kernel<false, false>'):
        if k in name:
            return k.replace('_kernel', '')
    return None


def main():
    path = sys.argv[1]
    per_step = int(sys.argv[2]) if len(sys.argv) > 2 else 318
    rows, marks = [], []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            if 'sleep' in name.lower() or 'spin' in name.lower():
                marks.append(s)
                continue
            k = short(name)
            if k is None:
                continue
            gx = int(r.get('Grid_Size_X') or 0) // max(int(r.get('Workgroup_Size_X') or 256), 1)
            gy = int(r.get('Grid_Size_Y') or 1)
            rows.append((s, e, k, gx, gy))
    rows.sort()
    marks.sort()
    if len(marks) >= 2:
        rows = [r for r in rows if marks[0] < r[0] < marks[1]]
    last = rows[-per_step:]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    print('%-34s %6s %6s %9s' % ('kernel', 'gx', 'gy', 'us'))
    for s, e, k, gx, gy in last:
        us = (e - s) / 1e3
        tot[k] += us
        cnt[k] += 1
        print('%-34s %6d %6d %9.2f' % (k, gx, gy, us))
    print()
    for k in sorted(tot, key=lambda k: -tot[k]):
        print('%-34s %4d launches %9.1f us  (%.2f us each)' % (k, cnt[k], tot[k], tot[k] / cnt[k]))
    print('total %.1f us over %d launches' % (sum(tot.values()), sum(cnt.values())))


if __name__ == '__main__':
    main()
