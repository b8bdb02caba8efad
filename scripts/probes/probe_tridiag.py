"""Probe: hand-written tridiagonal path vs rocSOLVER syevd per size class (ResNet-50
factor classes), ms per class solve; split into reduction / stedc+ormtr."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import _lib, eigen  # noqa: E402


def spd(n, b, dev):
    x = torch.randn(b, n, 256, device=dev)
    return x @ x.transpose(1, 2) / 256 + 1e-3 * torch.eye(n, device=dev)


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device('cuda')
    # a side stream: the reduction's hipGraph cannot be captured on the null stream
    cur = torch.cuda.Stream()
    torch.cuda.set_stream(cur)
    out = {}
    classes = [(256, 6), (512, 6), (1024, 6), (2048, 4), (2304, 6), (4608, 3)]
    if len(sys.argv) > 1:
        classes = [tuple(int(v) for v in a.split('x')) for a in sys.argv[1:]]
    L = _lib.lib()
    for n, b in classes:
        A = spd(n, b, dev)
        mats = [A[i].contiguous() for i in range(b)]
        t_syevd = timeit(lambda: eigen._syevd_class(mats, 0.0, cur))
        t_tri = timeit(lambda: eigen._tridiag_class(mats, 0.0, cur))
        B = eigen._tri_buffers(dev, n, b)
        lda = B['lda']
        red = timeit(lambda: L.kfac_sytrd_batched(_lib.ptr(B['A']), lda, B['sA'], n, b,
                                                  _lib.ptr(B['d']), _lib.ptr(B['e']),
                                                  _lib.ptr(B['tau']), _lib.ptr(B['ws']), 1,
                                                  _lib.stream()))
        # accuracy of the last solve
        (Q, d) = eigen._tridiag_class(mats[:1] if b == 1 else mats, 0.0, cur)[0]
        A64 = mats[0].double()
        resid = ((A64 @ Q.double() - Q.double() * d.double()).norm() / A64.norm()).item()
        out['%dx%d' % (n, b)] = dict(syevd_ms=t_syevd, tridiag_ms=t_tri, reduction_ms=red,
                                     resid=resid)
        print('n=%5d b=%d  syevd %8.2f ms   tridiag %8.2f ms (reduction %8.2f ms)  resid %.1e'
              % (n, b, t_syevd, t_tri, red, resid), flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
