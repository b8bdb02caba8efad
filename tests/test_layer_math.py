"""CPU layer math: reference identities and helper round trips."""
import torch
import pytest

from distributed_kfac_pytorch_amd.layers import utils as lutils
from distributed_kfac_pytorch_amd.layers import Conv2dLayer, LinearLayer, LinearMultiLayer


def test_append_bias_ones():
    x = torch.randn(4, 6)
    y = lutils.append_bias_ones(x)
    assert y.shape == (4, 7) and torch.equal(y[:, -1], torch.ones(4))


def test_get_cov_symmetric_and_scaled():
    a = torch.randn(50, 7)
    c = lutils.get_cov(a)
    assert torch.equal(c, c.t())
    assert torch.allclose(c, a.t() @ a / 50, atol=1e-6)
    b = torch.randn(50, 7)
    assert torch.allclose(lutils.get_cov(a, b, scale=5), a.t() @ b / 5, atol=1e-5)


def test_triu_roundtrip():
    x = torch.randn(9, 9)
    x = x + x.t()
    assert torch.equal(lutils.fill_triu(x.shape, lutils.get_triu(x)), x)


def test_running_avg():
    cur = torch.eye(3)
    new = torch.ones(3, 3)
    lutils.update_running_avg(new, cur, 0.9)
    assert torch.allclose(cur, 0.9 * torch.eye(3) + 0.1 * new)
    cur2 = torch.eye(3)
    lutils.update_running_avg(new, cur2, 1.0)
    assert torch.equal(cur2, torch.eye(3))


def test_eigendecomp_clip_and_contiguous():
    x = torch.randn(6, 6)
    a = x @ x.t() - torch.eye(6)
    Q, d = lutils.get_eigendecomp(a, concat=False)
    assert Q.is_contiguous() and (d >= 0).all()


def test_extract_patches_matches_unfold():
    x = torch.randn(2, 3, 7, 9)
    p = lutils.extract_patches(x, (3, 3), (2, 1), (1, 1))
    u = torch.nn.functional.unfold(x, 3, padding=1, stride=(2, 1))
    assert torch.equal(p.reshape(-1, 27), u.transpose(1, 2).reshape(-1, 27))


def test_conv_factor_identity():
    """A_1 = 0.95 I + 0.05 a^T a / (B S^3) with the ones column."""
    conv = torch.nn.Conv2d(2, 4, 3, padding=1, bias=True)
    layer = Conv2dLayer(conv)
    x = torch.randn(3, 2, 5, 5)
    layer.a_inputs = [x]
    layer.update_A_factor(0.95)
    P = lutils.append_bias_ones(lutils.extract_patches(x, (3, 3), (1, 1), (1, 1)).reshape(-1, 18))
    S = 25
    want = 0.95 * torch.eye(19) + 0.05 * P.t() @ P / (3 * S ** 3)
    assert torch.allclose(layer.state['A'], want, atol=1e-6)


def test_linear_collapses_sequence_dims():
    lin = torch.nn.Linear(5, 3)
    layer = LinearLayer(lin)
    x = torch.randn(2, 4, 5)
    layer.a_inputs = [x]
    layer.update_A_factor(0.0 + 1e-9)
    a = lutils.append_bias_ones(x.reshape(-1, 5))
    assert torch.allclose(layer.state['A'], a.t() @ a / 8, atol=1e-5)


def test_linear_multi_sums_per_call():
    lin = torch.nn.Linear(4, 2, bias=False)
    layer = LinearMultiLayer(lin)
    xs = [torch.randn(3, 4), torch.randn(5, 4)]
    A = layer._get_A_factor(xs)
    assert torch.allclose(A, xs[0].t() @ xs[0] / 3 + xs[1].t() @ xs[1] / 5, atol=1e-6)


def test_conv_rejects_grouped():
    import pytest
    with pytest.raises(ValueError):
        Conv2dLayer(torch.nn.Conv2d(4, 4, 3, groups=2))


def test_conv_dilation_factor():
    conv = torch.nn.Conv2d(2, 3, 3, padding=2, dilation=2, bias=False)
    layer = Conv2dLayer(conv)
    x = torch.randn(2, 2, 6, 6)
    u = torch.nn.functional.unfold(x, 3, dilation=2, padding=2)
    P = u.transpose(1, 2).reshape(-1, 18) / 36
    want = P.t() @ P / P.shape[0]
    assert torch.allclose(layer._get_A_factor([x]), want, atol=1e-6)


def test_inverse_many_batched_classes_match_per_matrix():
    """ops.eigen.inverse_many batches by size class; on CPU the batched LAPACK
    calls reproduce the per-matrix reference path bit for bit."""
    from distributed_kfac_pytorch_amd.ops import eigen as eigen_ops
    g = torch.Generator().manual_seed(3)
    mats = []
    for n in (5, 9, 5, 12, 9, 5):
        x = torch.randn(n, 2 * n, generator=g)
        mats.append(x @ x.t() / (2 * n))
    outs = eigen_ops.inverse_many(mats, 0.01)
    for A, out in zip(mats, outs):
        M = A + torch.diag(A.new_full((A.shape[0],), 0.01))
        ref = torch.cholesky_inverse(torch.linalg.cholesky(M))
        assert torch.equal(out, ref)


def test_inverse_many_raises_on_indefinite():
    from distributed_kfac_pytorch_amd.ops import eigen as eigen_ops
    bad = -torch.eye(4)
    with pytest.raises(torch.linalg.LinAlgError):
        eigen_ops.inverse_many([torch.eye(4), bad], 0.001)
