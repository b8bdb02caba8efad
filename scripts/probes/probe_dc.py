"""Probe: wall time of the batched divide-and-conquer tridiagonal solver alone
(csrc/eig_dc.hip) and of rocSOLVER stedc, per ResNet-50 size class."""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen, _lib  # noqa: E402


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


def main():
    dev = torch.device('cuda')
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    for n, b in [(4608, 1), (4608, 3), (2304, 6), (2048, 4), (1152, 4), (576, 3)]:
        g = torch.Generator(device=dev).manual_seed(n)
        X = torch.randn(b, n, n // 3, device=dev, generator=g)
        A = (X @ X.transpose(1, 2) / X.shape[2] + 1e-3 * torch.eye(n, device=dev))
        B = eigen._tri_buffers(dev, n, b)
        lda = B['lda']
        B['A'][:, :n, :n].copy_(A)
        L = _lib.lib()
        _lib.check(L.kfac_sytrd_batched(_lib.ptr(B['A']), lda, B['sA'], n, b, _lib.ptr(B['d']),
                                        _lib.ptr(B['e']), _lib.ptr(B['tau']), _lib.ptr(B['ws']),
                                        0, _lib.stream()), 'sytrd')
        recs = eigen._dc_records(B, n, b)
        cs = _lib.stream()
        t_dc = timeit(lambda: _lib.check(L.kfac_dc_batched(recs, b, 1, cs), 'dc'))
        d0, e0 = B['d'].clone(), B['e'].clone()

        def stedc():
            B['d'].copy_(d0)
            B['e'].copy_(e0)
            _lib.check(L.kfac_stedc_batched(_lib.ptr(B['d']), _lib.ptr(B['e']), _lib.ptr(B['Z']),
                                            lda, n * lda, n, b, _lib.ptr(B['info']), cs), 'stedc')
        t_st = timeit(stedc)
        t_bt = timeit(lambda: _lib.check(L.kfac_tridiag_backtransform(
            *eigen._bt_args(B, n, b), 1, cs), 'bt'))
        t_red = timeit(lambda: _lib.check(L.kfac_sytrd_batched(
            _lib.ptr(B['A']), lda, B['sA'], n, b, _lib.ptr(B['d']), _lib.ptr(B['e']),
            _lib.ptr(B['tau']), _lib.ptr(B['ws']), 1, cs), 'sytrd'), reps=1)
        print('n=%5d b=%d  dc %7.2f ms  stedc %7.2f ms  backtransform %7.2f ms  reduction %7.2f ms'
              % (n, b, t_dc, t_st, t_bt, t_red), flush=True)


if __name__ == '__main__':
    main()
