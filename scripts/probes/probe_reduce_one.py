"""Probe: one fused reduction of a given class (n x b), eager launches (no
graph), for rocprofv3 kernel traces.  argv: n b [graph]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_kfac_pytorch_amd.ops import eigen, _lib  # noqa: E402


def main():
    n, b = int(sys.argv[1]), int(sys.argv[2])
    graph = len(sys.argv) > 3 and sys.argv[3] == 'graph'
    dev = torch.device('cuda')
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    L = _lib.lib()
    g = torch.Generator(device=dev).manual_seed(n)
    B = eigen._tri_buffers(dev, n, b)
    X = torch.randn(b, n, n // 3, device=dev, generator=g)
    B['A'][:, :, :n].copy_(X @ X.transpose(1, 2) / X.shape[2])
    rr = (_lib.ReduceRecord * b)()
    for i in range(b):
        r = rr[i]
        r.A, r.lda, r.d = B['A'][i].data_ptr(), B['lda'], B['d'][i].data_ptr()
        r.e, r.tau = B['e'][i].data_ptr(), B['tau'][i].data_ptr()
        r.ws, r.n = B['rws'].data_ptr() + 4 * i * B['rwsf'], n
    cs = _lib.stream()
    stamps = torch.zeros(n * 16, dtype=torch.int64, device=dev)
    if os.environ.get('STAMPS'):
        _lib.check(L.kfac_reduce_stamps(_lib.ptr(stamps)), 'stamps')
    for it in range(int(os.environ.get('REPS', '3'))):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _lib.check(L.kfac_reduce_batched(rr, b, int(graph), cs), 'reduce')
        torch.cuda.synchronize()
        print('n=%d b=%d graph=%d run %d: %.2f ms (%.2f us/col)' % (
            n, b, graph, it, (time.perf_counter() - t) * 1e3,
            (time.perf_counter() - t) * 1e6 / n), flush=True)
    if os.environ.get('STAMPS'):
        full = stamps.view(n, 16).cpu().double()
        clk = (full[1:n - 2, 9] - full[1:n - 2, 8]) / ((full[1:n - 2, 6] - full[1:n - 2, 0]) * 10.0)
        print('fin shader clock GHz: median %.2f  min %.2f  max %.2f' % (
            clk.median().item(), clk.min().item(), clk.max().item()))
        st = full[:, :7]
        d = (st[:, 1:] - st[:, :-1]) * 10.0   # 100 MHz -> ns
        for name, rows in (('first 64 cols', slice(1, 65)), ('middle', slice(n // 2, n // 2 + 64)),
                           ('last 64', slice(n - 65, n - 1))):
            print(name, 'phase ns:', ' '.join('%7.0f' % v for v in d[rows].mean(0).tolist()),
                  ' total %.0f' % ((st[rows, 6] - st[rows, 0]) * 10).mean().item())


if __name__ == '__main__':
    main()
