"""Probe: stage-2 bulge chasing (csrc/eig_sb2st.hip) timeline.  Runs stage 1
once, then sb2st on copies of the band under each KFAC_SB2ST_DBG setting
given, with per-workgroup s_memrealtime stamps (dbg bit 8): total time,
workgroup lifetime (ticks x tick time), and the start-to-start distance of
consecutive groups of one matrix (the pipeline's per-group lag).

    python scripts/probes/probe_sb2st_timeline.py --n 4608 --b 2 --dbg 8,24,9
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import _lib, eigen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4608)
    ap.add_argument('--b', type=int, default=2)
    ap.add_argument('--dbg', default='8,24,9')
    a = ap.parse_args()
    dev = torch.device('cuda')
    n, b = a.n, a.b
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    mats = []
    for _ in range(b):
        x = torch.randn(n, n // 3, device=dev, generator=g)
        mats.append(0.3 * torch.eye(n, device=dev) + x @ x.t() / x.shape[1])
    B = eigen._ts_buffers(dev, n, b, slot=7)
    cs = _lib.c_vp(torch.cuda.current_stream(dev).cuda_stream)
    r1 = (_lib.Sy2sbRecord * b)()
    for i, A in enumerate(mats):
        B['A'][i, :n, :n].copy_(A)
        r = r1[i]
        r.A, r.lda, r.tau = B['A'][i].data_ptr(), B['lda'], B['tau'][i].data_ptr()
        r.band, r.ws, r.n = B['band'][i].data_ptr(), B['syws'][i].data_ptr(), n
    _lib.check(L.kfac_sy2sb_batched(r1, b, 0, cs), 'sy2sb')
    band0 = B['band'].clone()
    ref = [torch.linalg.eigvalsh(A.double().cpu()) for A in mats]
    for d in [int(x) for x in a.dbg.split(',')]:
        os.environ['KFAC_SB2ST_DBG'] = str(d)
        r2 = (_lib.Sb2stRecord * b)()
        for i in range(b):
            q = r2[i]
            q.band_in = q.band = B['band'][i].data_ptr()
            q.v2, q.d, q.e = B['v2'][i].data_ptr(), B['d'][i].data_ptr(), B['e'][i].data_ptr()
            q.ldv2, q.n = B['ldv2'], n
        ts = []
        for rep in range(3):
            B['band'].copy_(band0)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.check(L.kfac_sb2st_batched(r2, b, 0, cs), 'sb2st')
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        err = 0.0
        for i in range(b):
            dd = B['d'][i].double().cpu()
            ee = B['e'][i][:n - 1].double().cpu()
            T = torch.diag(dd) + torch.diag(ee, -1) + torch.diag(ee, 1)
            err = max(err, float((torch.linalg.eigvalsh(T) - ref[i]).abs().max() / ref[i].abs().max()))
        line = 'dbg=%d sb2st %.2f ms (min of 3), tridiag eig err %.1e' % (d, min(ts), err)
        if d & 8:
            mx = 4 * 20000
            buf = (ctypes.c_longlong * mx)()
            nw = L.kfac_sb2st_debug_stamps(buf, mx // 4)
            rows = [(buf[4 * k], buf[4 * k + 1], buf[4 * k + 2], buf[4 * k + 3]) for k in range(nw)]
            rows = [r for r in rows if r[0] >= 0]
            t0 = min(r[2] for r in rows)
            life = sorted((r[3] - r[2]) / 100.0 for r in rows)          # us (100 MHz)
            per = {}
            for m, gi, st, en in rows:
                per.setdefault(m, {})[gi] = (st, en)
            lags = []
            for m, d2 in per.items():
                for gi in sorted(d2):
                    if gi + 1 in d2:
                        lags.append((d2[gi + 1][0] - d2[gi][0]) / 100.0)
            lags.sort()
            span = (max(r[3] for r in rows) - t0) / 100.0
            line += ('; span %.0f us, wg lifetime median %.1f us (max %.1f), group start lag '
                     'median %.2f us (p10 %.2f, p90 %.2f)' % (
                         span, life[len(life) // 2], life[-1], lags[len(lags) // 2],
                         lags[len(lags) // 10], lags[9 * len(lags) // 10]))
        print(line, flush=True)
        if d & 128:
            ph = (ctypes.c_longlong * 64)()
            L.kfac_sb2st_debug_phases(ph)
            names = ['fill', 'loads', 'house', 'dot', 'update', 'outputs', 'barrier']
            for t in range(8):
                row = [ph[8 * t + k] for k in range(8)]
                if row[0] == 0:
                    continue
                dl = ['%s %d' % (names[k], row[k + 1] - row[k]) for k in range(7)
                      if row[k + 1] and row[k]]
                print('  tick %d cycles: total %d | %s' % (20 + t, row[7] - row[0], ', '.join(dl)))


if __name__ == '__main__':
    main()
