"""Probe: where the error of a large-factor eigendecomposition comes from.
Runs the fused reduction, then compares (a) the tridiagonal T's fp64
eigenvalues with A's (reduction error), (b) the divide-and-conquer output
with T's (D&C error), (c) the full path.  argv: n"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen, _lib  # noqa: E402


def kfac_factor(n, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    A = (0.95 ** 20) * torch.eye(n, device=dev, dtype=torch.float64)
    for _ in range(3):
        X = torch.randn(n, max(1, n // 3), device=dev, dtype=torch.float64, generator=g)
        X *= torch.exp(torch.randn(n, 1, device=dev, dtype=torch.float64, generator=g))
        A += 0.05 * X @ X.t() / X.shape[1]
    return A


def main():
    n = int(sys.argv[1])
    dev = torch.device('cuda')
    A64 = kfac_factor(n, 90, dev)
    A32 = A64.float()
    ref = torch.linalg.eigvalsh(A64)
    ref32 = torch.linalg.eigvalsh(A32.double())
    an = ref.abs().max().item()
    print('n', n, 'lam range %.3e .. %.3e' % (ref.min().item(), an),
          'fp32 rounding shift %.2e' % ((ref32 - ref).abs().max().item() / an))
    L = _lib.lib()
    B = eigen._tri_buffers(dev, n, 1, slot=7)
    B['A'][0, :n, :n].copy_(A32)
    rr = (_lib.ReduceRecord * 1)()
    r = rr[0]
    r.A, r.lda, r.d = B['A'][0].data_ptr(), B['lda'], B['d'][0].data_ptr()
    r.e, r.tau = B['e'][0].data_ptr(), B['tau'][0].data_ptr()
    r.ws, r.n = B['rws'].data_ptr(), n
    _lib.check(L.kfac_reduce_batched(rr, 1, 0, _lib.stream()), 'reduce')
    torch.cuda.synchronize()
    d, e = B['d'][0].double(), B['e'][0, :n - 1].double()
    T = torch.diag(d) + torch.diag(e, 1) + torch.diag(e, -1)
    tl = torch.linalg.eigvalsh(T)
    err_red = (tl - ref32).abs() / an
    print('reduction: max |lam(T) - lam(A32)| / |A| = %.2e at index %d' % (
        err_red.max().item(), int(err_red.argmax())))
    (w, Z), = eigen.tridiag_eigh([B['d'][0].clone()], [B['e'][0].clone()])
    err_dc = (w.double() - tl).abs() / an
    print('divide and conquer: max |w - lam(T)| / |A| = %.2e at index %d of %d' % (
        err_dc.max().item(), int(err_dc.argmax()), n))
    top = torch.topk(err_dc, 8)
    print('  worst D&C indices', top.indices.tolist(), ['%.1e' % v for v in top.values.tolist()])
    Zd = Z.double()
    res = (T @ Zd.t() - Zd.t() * w.double()).norm(dim=0) / an
    print('  D&C per-vector residual max %.2e median %.2e' % (res.max().item(), res.median().item()))
    (Q, dd), = eigen.symeig_many([A32])
    err_full = (dd.double() - ref.clamp(min=0)).abs() / an
    print('full path: max eigenvalue error %.2e at %d' % (err_full.max().item(), int(err_full.argmax())))
    print('info', [int(i.item()) for i in eigen._INFOS[-2:]] if eigen._INFOS else None)


if __name__ == '__main__':
    main()
