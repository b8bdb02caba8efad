"""Probe: large symmetric eigendecomposition backends reachable from torch on
MI355X (default hipSOLVER/rocSOLVER vs MAGMA), batch 1 and 3, against our
strided-batched rocSOLVER path (ops/eigen.py).  Prints ms per call."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())


def spd(n, b, dev):
    x = torch.randn(b, n, n // 2, device=dev)
    return x @ x.transpose(1, 2) / n + 1e-3 * torch.eye(n, device=dev)


def timeit(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    from distributed_kfac_pytorch_amd.ops import eigen
    dev = torch.device('cuda')
    out = {}
    for n, b in ((1024, 1), (2304, 1), (2304, 6), (4608, 1), (4608, 3)):
        A = spd(n, b, dev)
        for lib in ('default', 'magma'):
            try:
                torch.backends.cuda.preferred_linalg_library(lib)
                ms = timeit(lambda: torch.linalg.eigh(A))
            except Exception as e:  # pragma: no cover
                ms = 'err: {}'.format(e)[:80]
            out['{}_n{}_b{}'.format(lib, n, b)] = ms
            print(lib, n, b, ms, flush=True)
        torch.backends.cuda.preferred_linalg_library('default')
        mats = [A[i].contiguous() for i in range(b)]
        ms = timeit(lambda: eigen._library_eigh(mats, 0.0, 1))
        out['kfac_syevd_n{}_b{}'.format(n, b)] = ms
        print('kfac_syevd', n, b, ms, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
