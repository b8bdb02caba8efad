"""Probe: the fused one-launch-per-column reduction (csrc/eig_reduce.hip) per
size class and for the whole ResNet-50 ragged batch, next to the round-1
3-launch reduction; plus the D&C and back-transform stages of the fused path."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from distributed_kfac_pytorch_amd.ops import eigen, _lib  # noqa: E402
from probe_eig_resnet50 import sizes  # noqa: E402


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best * 1e3


def records(classes, dev):
    total = sum(len(v) for v in classes.values())
    rr = (_lib.ReduceRecord * total)()
    dr = (_lib.DcRecord * total)()
    k = 0
    bts = []
    for n, mats in sorted(classes.items(), key=lambda kv: -kv[0]):
        b = len(mats)
        B = eigen._tri_buffers(dev, n, b, slot=7)
        for i, m in enumerate(mats):
            B['A'][i, :n, :n].copy_(m)
        dcr = eigen._dc_records(B, n, b)
        for i in range(b):
            r = rr[k]
            r.A, r.lda, r.d = B['A'][i].data_ptr(), B['lda'], B['d'][i].data_ptr()
            r.e, r.tau = B['e'][i].data_ptr(), B['tau'][i].data_ptr()
            r.ws, r.n = B['rws'].data_ptr() + 4 * i * B['rwsf'], n
            dr[k] = dcr[i]
            k += 1
        bts.append((B, n, b))
    return rr, dr, bts, total


def main():
    dev = torch.device('cuda')
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    L = _lib.lib()
    cs = _lib.stream()

    def mk(n, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        X = torch.randn(n, n // 3 + 1, device=dev, generator=g)
        return X @ X.t() / X.shape[1] + 1e-3 * torch.eye(n, device=dev)

    cases = [('4608x1', {4608: 1}), ('4608x3', {4608: 3}), ('2304x6', {2304: 6}),
             ('2048x4', {2048: 4}), ('1152x4', {1152: 4})]
    ns = [n for n in sizes() if n > eigen.SMALL_N]
    full = {}
    for n in ns:
        full[n] = full.get(n, 0) + 1
    cases.append(('resnet50_all_large(%d)' % len(ns), full))
    for name, spec in cases:
        classes = {n: [mk(n, 13 * n + i) for i in range(b)] for n, b in spec.items()}
        rr, dr, bts, total = records(classes, dev)
        t_red = timeit(lambda: _lib.check(L.kfac_reduce_batched(rr, total, 1, cs), 'reduce'))
        t_dc = timeit(lambda: _lib.check(L.kfac_dc_batched(dr, total, 1, cs), 'dc'))

        def bt():
            for B, n, b in bts:
                _lib.check(L.kfac_tridiag_backtransform(*eigen._bt_args(B, n, b), 1, cs), 'bt')
        t_bt = timeit(bt)
        cols = max(spec)
        print('%-26s fused reduction %8.2f ms (%5.2f us/col)  dc %7.2f ms  backtransform %7.2f ms'
              % (name, t_red, 1e3 * t_red / cols, t_dc, t_bt), flush=True)


if __name__ == '__main__':
    main()
