"""Device-side AMP unscale / non-finite filter of the G factor (layers/base.py
take_factor_job) against the CPU path (_take_g_outputs, the reference's
kfac/layers/base.py:392-417 semantics): with several accumulated sources and
one overflowed micro-batch, the factor averages over the KEPT rows only."""
import warnings

import pytest
import torch

from distributed_kfac_pytorch_amd.layers import Conv2dLayer, LinearLayer

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')


class _Scaler(object):
    def __init__(self, s):
        self.s = s

    def get_scale(self):
        return self.s


def _run(make_layer, shapes, bad):
    torch.manual_seed(5)
    lay_gpu = make_layer(DEV)
    lay_cpu = make_layer(torch.device('cpu'))
    scale = 8.0
    for lay in (lay_gpu, lay_cpu):
        lay.grad_scaler = _Scaler(scale)
    gs = [torch.randn(*s) * scale for s in shapes]
    # one clean update first, so the factor exists on both paths
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        lay_gpu.g_outputs = [(g.to(DEV), scale) for g in gs]
        lay_cpu.g_outputs = [(g, scale) for g in gs]
        for lay in (lay_gpu, lay_cpu):
            lay.update_G_factor(0.9)
    gs = [torch.randn(*s) * scale for s in shapes]
    for i in bad:
        gs[i].view(-1)[3] = float('inf')
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        lay_gpu.g_outputs = [(g.to(DEV), scale) for g in gs]
        lay_cpu.g_outputs = [(g, scale) for g in gs]
        for lay in (lay_gpu, lay_cpu):
            lay.update_G_factor(0.9)
    return lay_gpu.state['G'].cpu(), lay_cpu.state['G']


@pytest.mark.parametrize('bad', [(1,), (0, 2), ()])
def test_conv_partial_overflow_matches_cpu(bad):
    def make(dev):
        return Conv2dLayer(torch.nn.Conv2d(6, 10, 3, padding=1).to(dev))
    # micro-batches of different sizes: the kept-row count is not a fixed fraction
    g, c = _run(make, [(4, 10, 5, 5), (2, 10, 5, 5), (3, 10, 5, 5)], bad)
    assert torch.isfinite(g).all()
    assert torch.allclose(g, c, atol=1e-5, rtol=1e-4), (g - c).abs().max()


@pytest.mark.parametrize('bad', [(0,), (1, 2)])
def test_linear_partial_overflow_matches_cpu(bad):
    def make(dev):
        return LinearLayer(torch.nn.Linear(12, 9).to(dev))
    g, c = _run(make, [(5, 9), (7, 9), (3, 9)], bad)
    assert torch.isfinite(g).all()
    assert torch.allclose(g, c, atol=1e-5, rtol=1e-4), (g - c).abs().max()


def test_all_overflowed_leaves_factor():
    def make(dev):
        return LinearLayer(torch.nn.Linear(12, 9).to(dev))
    g, c = _run(make, [(5, 9), (7, 9)], (0, 1))
    assert torch.allclose(g, c)
