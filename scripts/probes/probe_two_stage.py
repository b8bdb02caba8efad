"""Probe: the two-stage eigensolver stage by stage (csrc/eig_sy2sb.hip,
eig_sb2st.hip, eig_dc.hip, eig_q2.hip, eig_backtransform.hip shift 16).

For each size: random K-FAC-like SPD factors (identity remnant + low-rank
data); after every stage the intermediate result is checked in fp64 against
torch.linalg.eigvalsh (band after stage 1, tridiagonal after stage 2, full
eigendecomposition at the end) and each stage is timed (events, after a
warm-up run).  Then the ResNet-50 factor set, two-stage group vs the
one-stage path.

    python scripts/probes/probe_two_stage.py [--sizes 64,200,1024] [--resnet50]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import _lib, eigen  # noqa: E402


def factor(n, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(n, max(8, n // 3), device=dev, generator=g)
    return 0.3 * torch.eye(n, device=dev) + x @ x.t() / x.shape[1]


def band_dense(bs, n):
    W = 32
    D = torch.zeros(n, n, dtype=torch.float64)
    b = bs.view(-1, W)[:n].double().cpu()
    for o in range(W):
        off = W - 1 - o
        if off >= n:
            continue
        vals = b[off:, o]
        idx = torch.arange(off, n)
        D[idx, idx - off] = vals
        D[idx - off, idx] = vals
    return D


def run_size(n, dev, reps=3):
    L = _lib.lib()
    mats = [factor(n, dev, s) for s in range(2)]
    B = eigen._ts_buffers(dev, n, len(mats), slot=7)
    b = len(mats)
    cur = torch.cuda.current_stream(dev)
    cs = _lib.c_vp(cur.cuda_stream)
    r1 = (_lib.Sy2sbRecord * b)()
    r2 = (_lib.Sb2stRecord * b)()
    r4 = (_lib.Q2Record * b)()
    r3 = eigen._dc_records(B, n, b)
    for i, A in enumerate(mats):
        r = r1[i]
        r.A, r.lda, r.tau = B['A'][i].data_ptr(), B['lda'], B['tau'][i].data_ptr()
        r.band, r.ws, r.n = B['band'][i].data_ptr(), B['syws'][i].data_ptr(), n
        q = r2[i]
        q.band_in = q.band = B['band'][i].data_ptr()
        q.v2, q.d, q.e = B['v2'][i].data_ptr(), B['d'][i].data_ptr(), B['e'][i].data_ptr()
        q.ldv2, q.n = B['ldv2'], n
        z = r4[i]
        z.Z, z.v2, z.ldz, z.ldv2, z.n = B['Z'][i].data_ptr(), B['v2'][i].data_ptr(), B['lda'], \
            B['ldv2'], n
    lda = B['lda']
    stages = [
        ('sy2sb', lambda: _lib.check(L.kfac_sy2sb_batched(r1, b, 1, cs), 'sy2sb')),
        ('sb2st', lambda: _lib.check(L.kfac_sb2st_batched(r2, b, 1, cs), 'sb2st')),
        ('dc', lambda: _lib.check(L.kfac_dc_batched(r3, b, 1, cs), 'dc')),
        ('q2', lambda: _lib.check(L.kfac_q2_batched(r4, b, 1, cs), 'q2')),
        ('q1', lambda: _lib.check(L.kfac_band_backtransform(
            _lib.ptr(B['A']), lda, B['sA'], _lib.ptr(B['tau']), _lib.ptr(B['Z']), lda, n * lda,
            n, b, _lib.ptr(B['T']), _lib.ptr(B['W1']), _lib.ptr(B['W2']), _lib.ptr(B['Vt']),
            eigen.SB2, 1, cs), 'q1')),
    ]
    ref = [torch.linalg.eigvalsh(A.double().cpu()) for A in mats]
    times = {k: [] for k, _ in stages}
    for rep in range(reps):
        for i, A in enumerate(mats):
            B['A'][i, :n, :n].copy_(A)
        for name, fn in stages:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1))
            if rep == 0:
                for i in range(b):
                    sc = float(ref[i].abs().max())
                    if name == 'sy2sb':
                        ev = torch.linalg.eigvalsh(band_dense(B['band'][i], n))
                        print('  n=%d mat %d sy2sb: band eig err %.1e' %
                              (n, i, float((ev - ref[i]).abs().max()) / sc), flush=True)
                    elif name == 'sb2st':
                        d = B['d'][i].double().cpu()
                        e = B['e'][i][:n - 1].double().cpu()
                        T = torch.diag(d) + torch.diag(e, -1) + torch.diag(e, 1)
                        ev = torch.linalg.eigvalsh(T)
                        print('  n=%d mat %d sb2st: tridiag eig err %.1e' %
                              (n, i, float((ev - ref[i]).abs().max()) / sc), flush=True)
                    elif name == 'q1':
                        Q = B['Z'][i, :, :n].t().double().cpu()
                        w = B['w'][i].double().cpu()
                        A = mats[i].double().cpu()
                        res = float((A @ Q - Q * w).abs().max()) / sc
                        orth = float((Q.t() @ Q - torch.eye(n, dtype=torch.float64)).abs().max())
                        print('  n=%d mat %d final: eig err %.1e resid %.1e orth %.1e' %
                              (n, i, float((w - ref[i]).abs().max()) / sc, res, orth), flush=True)
    print('n=%d x%d ms: ' % (n, b) + ' '.join('%s %.2f' % (k, min(v)) for k, v in times.items()) +
          ' total %.2f' % sum(min(v) for v in times.values()), flush=True)


def resnet50(dev):
    sys.path.insert(0, os.path.join(os.getcwd(), 'scripts', 'probes'))
    import probe_eig_resnet50 as pr
    ns = pr.sizes()
    mats = [factor(n, dev, i) for i, n in enumerate(ns)]
    variants = [(0, 0)] + [(1, c) for c in
                           [int(x) for x in os.environ.get('TS_COUNTS', '0').split(',')]]
    for flag, cnt in variants:
        eigen.TWO_STAGE = bool(flag)
        eigen.TWO_STAGE_COUNT = cnt
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = eigen.symeig_many(mats)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t) * 1e3
        worst = 0.0
        for A, (Q, d) in zip(mats[:12], out[:12]):
            Ad = A.double()
            sc = float(d.abs().max())
            worst = max(worst, float((Ad @ Q.double() - Q.double() * d.double()).abs().max()) / sc)
        print('resnet50 set (%d factors) two_stage=%d count=%d: %.1f ms, worst resid (first 12) '
              '%.1e' % (len(mats), flag, cnt, el, worst), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='33,64,200,1024')
    ap.add_argument('--resnet50', action='store_true')
    a = ap.parse_args()
    dev = torch.device('cuda')
    for n in [int(x) for x in a.sizes.split(',') if x]:
        run_size(n, dev)
    if a.resnet50:
        resnet50(dev)


if __name__ == '__main__':
    main()
