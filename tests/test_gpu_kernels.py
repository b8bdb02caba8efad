"""Numerics of every gfx950 kernel against a plain PyTorch fp32/fp64 reference.

Run on an MI355X: `pytest tests -m gpu`.  Each test fails (never skips) when
the native library is missing on a GPU box.
"""
import pytest
import torch

from distributed_kfac_pytorch_amd.layers import utils as lutils
from distributed_kfac_pytorch_amd.ops import _lib, factors, eigen, precond, comm_pack

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _cov_patches_ref(x, k, s, p, d, bias):
    """fp64 P^T P of the explicit im2col patch matrix (columns (c, kh, kw))."""
    cols = torch.nn.functional.unfold(x.double(), k, dilation=d, padding=p, stride=s)
    P = cols.transpose(1, 2).reshape(-1, cols.shape[1])
    if bias:
        P = torch.cat([P, torch.ones(P.shape[0], 1, dtype=P.dtype, device=P.device)], 1)
    return P.t() @ P


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize('layout', ['nchw', 'nhwc'])
@pytest.mark.parametrize('geom', [
    # C, H, W, k, s, p, d, bias
    (3, 9, 11, 3, 1, 1, 1, True),
    (16, 8, 8, 1, 1, 0, 1, False),
    (7, 13, 10, 3, 2, 1, 1, False),
    (5, 12, 12, 3, 1, 2, 2, True),
    (3, 20, 20, 7, 2, 3, 1, False),
    (64, 7, 7, 3, 1, 1, 1, False),    # ncols 576 -> several 128 tiles
    # channel counts % 8 == 0: the NHWC 16-bit inputs take the vectorised
    # syrk_vec path (internal (kh, kw, c) order, permuted back by the EMA)
    (16, 9, 9, 3, 2, 1, 1, True),
    (24, 10, 12, 3, 1, 2, 2, True),
    (136, 6, 6, 3, 1, 1, 1, True),    # ncols 1225: 10 tiles, bias chunk
    (48, 14, 14, 1, 2, 0, 1, False),
])
def test_syrk_patch_matches_unfold(dtype, layout, geom):
    C, H, W, k, s, p, d, bias = geom
    torch.manual_seed(0)
    x = torch.randn(3, C, H, W, device=DEV).to(dtype)
    if layout == 'nhwc':
        x = x.contiguous(memory_format=torch.channels_last)
    ref = _cov_patches_ref(x.float(), k, s, p, d, bias)
    src = factors.FactorSource(x, factors.Geometry(k, k, s, s, p, p, d, d), bias, 1.0)
    n = src.ncols
    got = factors.compute_cov([src], torch.float32).double()
    want = ref
    assert torch.equal(got, got.t())
    tol = 1e-4 if dtype == torch.float32 else 2e-3
    err = (got - want).abs().max().item() / max(1.0, want.abs().max().item())
    assert err < tol, err


def test_grouped_syrk_matches_unfold():
    """The grouped factor-step SYRK (every factor in one launch) against fp64
    unfold covariances: padding, strides, dilation, the bias chunk, tiles
    crossing 128 and diagonal tiles."""
    torch.manual_seed(0)
    geoms = [(16, 9, 9, 3, 2, 1, 1, True), (24, 10, 12, 3, 1, 2, 2, True),
             (136, 6, 6, 3, 1, 1, 1, True), (48, 14, 14, 1, 2, 0, 1, False),
             (64, 7, 7, 3, 1, 1, 1, False), (8, 30, 30, 3, 1, 1, 1, False)]
    items, refs = [], []
    for C, H, W, k, s_, p_, d, bias in geoms:
        x = torch.randn(5, C, H, W, device=DEV).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        src = factors.FactorSource(x, factors.Geometry(k, k, s_, s_, p_, p_, d, d), bias, 1.0)
        assert factors._vec_eligible(src)
        n = src.ncols
        items.append((torch.zeros(n, n, device=DEV), [src], torch.float32))
        refs.append(_cov_patches_ref(x.float(), k, s_, p_, d, bias))
    outs = factors.update_factors_grouped(items, 0.5)
    for got, want in zip(outs, refs):
        got = 2.0 * got.double()
        err = (got - want).abs().max().item() / max(1.0, want.abs().max().item())
        assert err < 2e-3, err


def test_syrk_vec_path_is_taken():
    x = torch.randn(2, 16, 5, 5, device=DEV).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    src = factors.FactorSource(x, factors.Geometry(3, 3, 1, 1, 1, 1, 1, 1), True, 1.0)
    assert factors._vec_eligible(src)
    ws = torch.zeros(src.ncols, src.ncols, device=DEV)
    assert factors.accumulate_sources([src], ws) == (144, 16, 9)


@pytest.mark.parametrize('rows', [1, 37, 1000, 70000])
@pytest.mark.parametrize('bias', [False, True])
def test_syrk_linear(rows, bias):
    torch.manual_seed(1)
    a = torch.randn(rows, 50, device=DEV, dtype=torch.bfloat16)
    src = factors.linear_source(a, bias)
    src.scale = 1.0 / rows
    cov = factors.compute_cov([src], torch.float32)
    af = a.double()
    if bias:
        af = torch.cat([af, torch.ones(rows, 1, dtype=af.dtype, device=DEV)], 1)
    ref = af.t() @ af / rows
    assert torch.allclose(cov.double(), ref, atol=2e-3, rtol=2e-3)
    assert torch.equal(cov, cov.t())


def test_conv_layer_factor_matches_cpu_reference():
    """Full layer path (scales, EMA, identity init) vs the reference CPU math."""
    from distributed_kfac_pytorch_amd.layers import Conv2dLayer
    torch.manual_seed(2)
    conv = torch.nn.Conv2d(6, 10, 3, stride=2, padding=1, bias=True)
    lay_gpu = Conv2dLayer(conv.to(DEV))
    lay_cpu = Conv2dLayer(torch.nn.Conv2d(6, 10, 3, stride=2, padding=1, bias=True))
    xs = [torch.randn(4, 6, 9, 9) for _ in range(2)]
    gs = [torch.randn(4, 10, 5, 5) for _ in range(2)]
    for x, g in zip(xs, gs):
        lay_gpu.a_inputs = [x.to(DEV)]
        lay_gpu.g_outputs = [g.to(DEV)]
        lay_cpu.a_inputs = [x]
        lay_cpu.g_outputs = [g]
        for lay in (lay_gpu, lay_cpu):
            lay.update_A_factor(0.9)
            lay.update_G_factor(0.9)
    for key in ('A', 'G'):
        assert torch.allclose(lay_gpu.state[key].cpu(), lay_cpu.state[key], atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize('sdtype', [torch.float32, torch.bfloat16])
def test_factor_ema(sdtype):
    n = 77
    torch.manual_seed(3)
    ws = torch.randn(n, n, device=DEV)
    state = torch.randn(n, n, device=DEV)
    state = (state + state.t()).to(sdtype)
    sym = torch.triu(ws) + torch.triu(ws, 1).t()
    want = (0.95 * state.float() + 0.05 * sym)
    _lib.check(_lib.lib().kfac_factor_ema(_lib.DTYPE_CODE[sdtype], _lib.ptr(state), _lib.ptr(ws),
                                          n, n, 0.95, 0, None, _lib.stream()), 'ema')
    tol = 1e-5 if sdtype == torch.float32 else 2e-2
    assert torch.allclose(state.float(), want, atol=tol, rtol=tol)
    assert torch.equal(state, state.t())


@pytest.mark.parametrize('n', [1, 5, 64, 129, 300])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_triu_roundtrip(n, dtype):
    torch.manual_seed(4)
    a = torch.randn(n, n, device=DEV)
    a = (a + a.t()).to(dtype)
    buf = torch.empty(comm_pack.triu_numel(n), dtype=dtype, device=DEV)
    comm_pack.pack_triu(a, buf)
    assert torch.equal(buf.cpu(), lutils.get_triu(a.cpu()))
    out = torch.empty_like(a)
    comm_pack.unpack_triu(buf * 2, out, divisor=2)
    assert torch.equal(out, a)


@pytest.mark.parametrize('n', [1, 2, 3, 17, 64, 128, 147, 192])
def test_jacobi_small_eig(n):
    torch.manual_seed(5)
    X = torch.randn(n, 3 * n + 2, device=DEV, dtype=torch.float64)
    A64 = X @ X.t() / X.shape[1] + 1e-3 * torch.eye(n, device=DEV, dtype=torch.float64)
    A = A64.float()
    (Q, d), = eigen._jacobi_small([A], clip=0.0)
    Q64, d64 = Q.double(), d.double()
    ref = torch.linalg.eigvalsh(A64)
    assert torch.all(d64[1:] >= d64[:-1])
    assert torch.allclose(d64, ref, atol=1e-5 * ref.abs().max().item() + 1e-7)
    resid = (A64 @ Q64 - Q64 * d64).norm() / A64.norm()
    orth = (Q64.t() @ Q64 - torch.eye(n, device=DEV, dtype=torch.float64)).abs().max()
    # fp32 orthogonality scales like n * eps; bound by the library solver's own
    Ql = torch.linalg.eigh(A)[1].double()
    orth_lib = (Ql.t() @ Ql - torch.eye(n, device=DEV, dtype=torch.float64)).abs().max()
    assert resid < 1e-5, resid
    assert orth < max(3e-5, 4 * orth_lib.item()), orth


def test_jacobi_batch_mixed_sizes_and_clip():
    torch.manual_seed(6)
    mats = []
    for n in (64, 10, 147, 1, 33):
        X = torch.randn(n, n, device=DEV)
        mats.append(X @ X.t() - 0.5 * torch.eye(n, device=DEV))   # some negative eigenvalues
    outs = eigen.symeig_many(mats, clip=0.0)
    for A, (Q, d) in zip(mats, outs):
        ref = torch.linalg.eigvalsh(A.double()).clamp(min=0)
        assert torch.allclose(d.double(), ref, atol=1e-4 * max(1, ref.abs().max().item()))
        assert torch.all(d >= 0)


def test_symeig_large_path():
    torch.manual_seed(7)
    X = torch.randn(300, 900, device=DEV)
    A = X @ X.t() / 900
    (Q, d), = eigen.symeig_many([A])
    assert Q.is_contiguous()
    resid = (A @ Q - Q * d).norm() / A.norm()
    assert resid < 1e-4


@pytest.mark.parametrize('solver', ['auto', 'jacobi'])
def test_symeig_size_classes(solver):
    """Several factors per size class (strided batch) + several classes
    (concurrent streams); order and per-matrix results must be preserved."""
    torch.manual_seed(8)
    mats = []
    for n in (300, 256, 300, 520, 256, 300, 193):
        X = torch.randn(n, n + 7, device=DEV)
        mats.append(X @ X.t() / (n + 7) - 0.01 * torch.eye(n, device=DEV))
    outs = eigen.symeig_many(mats, clip=0.0, solver=solver)
    torch.cuda.synchronize()
    for A, (Q, d) in zip(mats, outs):
        assert Q.shape == A.shape and Q.is_contiguous()
        d_ref = torch.linalg.eigvalsh(A.double())
        assert torch.allclose(d.double(), d_ref.clamp(min=0), atol=1e-4)
        dd = torch.linalg.eigvalsh(A.double()).float()   # unclipped for the residual
        resid = (A @ Q - Q * dd).norm() / A.norm()
        assert resid < 1e-4, resid


def test_outer_recip_and_hadamard():
    torch.manual_seed(8)
    dG = torch.rand(37, device=DEV)
    dA = torch.rand(53, device=DEV)
    out = precond.outer_reciprocal(dG, dA, 0.01)
    ref = 1 / (dG[:, None] * dA[None] + 0.01)
    assert torch.allclose(out, ref, rtol=1e-6)
    v = torch.randn(37, 53, device=DEV)
    v2 = v.clone()
    _lib.check(_lib.lib().kfac_hadamard(_lib.ptr(v2), 53, None, _lib.ptr(dG), _lib.ptr(dA), 37,
                                        53, 0.01, 1, _lib.stream()), 'hadamard')
    assert torch.allclose(v2, v / (dG[:, None] * dA[None] + 0.01), rtol=1e-6)


def test_precondition_eigen_matches_cpu():
    torch.manual_seed(9)
    nG, nA = 24, 41
    QA, _ = torch.linalg.qr(torch.randn(nA, nA))
    QG, _ = torch.linalg.qr(torch.randn(nG, nG))
    dA, dG = torch.rand(nA), torch.rand(nG)
    grad = torch.randn(nG, nA)
    dGdA = 1 / (dG[:, None] * dA[None] + 0.003)
    want = QG @ ((QG.t() @ grad @ QA) * dGdA) @ QA.t()
    out = torch.empty(nG, nA, device=DEV)
    precond.precondition_eigen(grad.to(DEV), QA.to(DEV), QG.to(DEV), dGdA=dGdA.to(DEV), out=out)
    assert torch.allclose(out.cpu(), want, atol=1e-4, rtol=1e-4)
    out2 = precond.precondition_eigen(grad.to(DEV), QA.to(DEV), QG.to(DEV), dA=dA.to(DEV),
                                      dG=dG.to(DEV), damping=0.003)
    assert torch.allclose(out2.cpu(), want, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('gdtype', [torch.float32, torch.bfloat16])
def test_grouped_kl_dot_and_apply(gdtype):
    torch.manual_seed(10)
    shapes = [(16, 27), (64, 577), (10, 65), (3, 1)] * 20   # > MAXG entries -> chunked launches
    pairs = []
    for r, c in shapes:
        big = torch.randn(r, c + 3, device=DEV)
        v = big[:, 1:c + 1]             # row-strided view like the bias-split arena slices
        g = torch.randn(r, c, device=DEV).to(gdtype)
        pairs.append((v, g))
    vg = precond.kl_dot(pairs)
    want = sum((v.double() * g.double()).sum() for v, g in pairs)
    assert torch.allclose(vg, want, rtol=1e-5)
    # channels_last conv-weight gradient: K-FAC column order (c, kh, kw) vs NHWC memory
    v4 = torch.randn(8, 5 * 9, device=DEV)
    g4 = torch.randn(8, 5, 3, 3, device=DEV).to(gdtype).contiguous(memory_format=torch.channels_last)
    vg4 = precond.kl_dot([(v4, g4)])
    assert torch.allclose(vg4, (v4.double() * g4.double().reshape(8, -1)).sum(), rtol=1e-5)
    lr, kl = 0.1, 1e-3
    nu = min(1.0, (kl / abs(want.item() * lr * lr)) ** 0.5)
    precond.apply_gradients(pairs, vg, lr, kl)
    for v, g in pairs:
        tol = 1e-6 if gdtype == torch.float32 else 1e-2
        assert torch.allclose(g.float(), (nu * v).to(gdtype).float(), rtol=tol, atol=tol)
