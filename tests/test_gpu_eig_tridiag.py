"""Hand-written blocked tridiagonalisation (csrc/eig_tridiag.hip) and the large-n
eigensolver path built on it, against fp64 torch references."""
import os

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import _lib, eigen

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _spd(n, rank, seed, damping=1e-3):
    g = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.randn(n, rank, device=DEV, dtype=torch.float64, generator=g)
    return X @ X.t() / rank + damping * torch.eye(n, device=DEV, dtype=torch.float64)


def _sytrd(mats):
    n, b = mats[0].shape[0], len(mats)
    B = eigen._tri_buffers(torch.device(DEV), n, b)
    lda = B['lda']
    for i, A in enumerate(mats):
        B['A'][i, :n, :n].copy_(A)
    s = _lib.stream()
    _lib.check(_lib.lib().kfac_sytrd_batched(_lib.ptr(B['A']), lda, B['sA'], n, b,
                                             _lib.ptr(B['d']), _lib.ptr(B['e']),
                                             _lib.ptr(B['tau']), _lib.ptr(B['ws']), 0, s),
               'sytrd')
    torch.cuda.synchronize()
    return B['d'].clone(), B['e'].clone()


@pytest.mark.parametrize('n', [2, 3, 33, 128, 129, 200, 257, 400])
def test_sytrd_tridiagonal_has_the_spectrum(n):
    A64 = [_spd(n, max(1, n // 2), s) for s in (0, 1)]
    d, e = _sytrd([a.float() for a in A64])
    for i, a in enumerate(A64):
        T = torch.diag(d[i].double()) + torch.diag(e[i, :n - 1].double(), 1) + \
            torch.diag(e[i, :n - 1].double(), -1)
        got = torch.linalg.eigvalsh(T)
        want = torch.linalg.eigvalsh(a)
        err = (got - want).abs().max().item() / want.abs().max().item()
        assert err < 2e-6, (n, i, err)


@pytest.mark.parametrize('n,b', [(193, 1), (256, 3), (300, 2), (521, 2), (1000, 1), (2049, 1)])
def test_tridiag_eigensolver(n, b):
    mats64 = [_spd(n, n // 3 + 1, 10 + s) for s in range(b)]
    mats = [m.float() for m in mats64]
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()     # graph capture needs a non-default stream
    for use_graph in (False, True, True):   # eager, capture, replay
        side.wait_stream(cur)
        outs = eigen._tridiag_class(mats, 0.0, side, use_graph=use_graph)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        eigen.check_solver_status()
        for A64, (Q, d) in zip(mats64, outs):
            Q64, d64 = Q.double(), d.double()
            assert Q.is_contiguous() and Q.shape == (n, n)
            assert torch.all(d64[1:] >= d64[:-1])
            ref = torch.linalg.eigvalsh(A64).clamp(min=0)
            scale = ref.abs().max().item()
            assert (d64 - ref).abs().max().item() < 2e-6 * scale
            resid = (A64 @ Q64 - Q64 * d64).norm().item() / A64.norm().item()
            orth = (Q64.t() @ Q64 - torch.eye(n, device=DEV, dtype=torch.float64)).abs().max()
            assert resid < 2e-5, resid
            assert orth < 1e-4, orth


def test_tridiag_degenerate_columns():
    """Diagonal and block-diagonal inputs: zero Householder columns (tau = 0)."""
    n = 260
    D = torch.diag(torch.linspace(0.1, 2.0, n, device=DEV))
    Bd = D.clone()
    Bd[:130, :130] += 0.01 * torch.ones(130, 130, device=DEV)
    outs = eigen._tridiag_class([D, Bd], None, torch.cuda.current_stream())
    torch.cuda.synchronize()
    for A, (Q, d) in zip((D, Bd), outs):
        A64, Q64, d64 = A.double(), Q.double(), d.double()
        resid = (A64 @ Q64 - Q64 * d64).norm().item() / A64.norm().item()
        assert resid < 1e-5, resid
        assert torch.allclose(d64, torch.linalg.eigvalsh(A64), atol=1e-5)


@pytest.mark.parametrize('path', ['fused', 'auto'])
def test_symeig_many_routes_big_classes_to_tridiag(path, monkeypatch):
    # default: every large factor through the fused ragged path; 'auto' (opt-in)
    # routes per size class (hand-written reduction >= TRIDIAG_MIN_N)
    assert os.environ.get('KFAC_EIG_LARGE') or eigen.LARGE_PATH == 'fused'
    monkeypatch.setattr(eigen, 'LARGE_PATH', path)
    if path == 'auto':
        assert eigen._class_solver(eigen.TRIDIAG_MIN_N) is eigen._tridiag_class
        assert eigen._class_solver(eigen.TRIDIAG_MIN_N - 1) is eigen._syevd_class
    mats = [_spd(n, 50, n).float() for n in (300, 2048, 300, 2100)]
    outs = eigen.symeig_many(mats, clip=0.0)
    torch.cuda.synchronize()
    for A, (Q, d) in zip(mats, outs):
        A64 = A.double()
        resid = (A64 @ Q.double() - Q.double() * d.double()).norm() / A64.norm()
        assert resid < 2e-5
