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
    B['A'][:, :n, :n].copy_(X @ X.transpose(1, 2) / X.shape[2])
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
        full = stamps.view(n, 16).cpu().double() * 10.0     # 100 MHz -> ns
        # F: 0 start, 1 record loaded, 2 sums reduced, 3 scalars, 4 end;
        # S: 10/11 first tile workgroup start/end, 12/13 first row-block workgroup
        for name, rows in (('first 64 cols', slice(1, 65)), ('middle', slice(n // 2, n // 2 + 64)),
                           ('last 64', slice(n - 66, n - 2))):
            f = full[rows]
            nxt = full[rows.start + 1:rows.stop + 1]
            if (f[:, 6] > 0).all():
                # tail launch L: 0 start, 1 record, 2 loads + sums, 3 scalars,
                # 4 slot rows, 5 tile update + symv, 6 end
                ph = [(f[:, k + 1] - f[:, k]).mean().item() for k in range(6)]
                print(name, 'L phases ns: ' + ' '.join('%6.0f' % v for v in ph),
                      '| L total %6.0f | L->L %6.0f | col %6.0f' % (
                          (f[:, 6] - f[:, 0]).mean().item(), (nxt[:, 0] - f[:, 6]).mean().item(),
                          (nxt[:, 0] - f[:, 0]).mean().item()))
                continue
            ph = [(f[:, k + 1] - f[:, k]).mean().item() for k in range(4)]
            print(name, 'F phases ns: ' + ' '.join('%6.0f' % v for v in ph),
                  '| F total %6.0f | F->S gap %6.0f | S tile %6.0f (rec %5.0f load %5.0f rest %5.0f) | S part %6.0f | S->F %6.0f | col %6.0f' % (
                      (f[:, 4] - f[:, 0]).mean().item(), (f[:, 10] - f[:, 4]).mean().item(),
                      (f[:, 11] - f[:, 10]).mean().item(), (f[:, 14] - f[:, 10]).mean().item(),
                      (f[:, 15] - f[:, 14]).mean().item(), (f[:, 11] - f[:, 15]).mean().item(), (f[:, 13] - f[:, 12]).mean().item(),
                      (nxt[:, 0] - f[:, 11]).mean().item(), (nxt[:, 0] - f[:, 0]).mean().item()))

if __name__ == '__main__':
    main()
