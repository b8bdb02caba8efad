"""Fused BatchNorm (+ add) (+ ReLU) kernels (csrc/bn.hip via ops/bn.py) against
an fp32 torch reference of the same op on the same bf16 inputs: output,
running statistics, num_batches_tracked, and every gradient."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops import bn as fbn

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _case(N, C, H, W, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(N, C, H, W, device=DEV, generator=g) * 3 + 1.5).to(torch.bfloat16)
    z = torch.randn(N, C, H, W, device=DEV, generator=g).to(torch.bfloat16)
    dy = torch.randn(N, C, H, W, device=DEV, generator=g).to(torch.bfloat16)
    cl = torch.channels_last
    return x.contiguous(memory_format=cl), z.contiguous(memory_format=cl), \
        dy.contiguous(memory_format=cl)


def _bn(C, seed):
    torch.manual_seed(seed)
    bn = nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.9, 1.1)
    return bn


def _rel(a, b):
    return ((a.float() - b.float()).norm() / max(b.float().norm().item(), 1e-30)).item()


# (8, 256, 14, 14), (32, 1024, 14, 14), (32, 2048, 7, 7): the folded small-layer
# path (M <= 6272, C % 256 == 0: finalize inside the apply pass, csrc/bn.hip)
@pytest.mark.parametrize('shape', [(4, 64, 28, 28), (8, 256, 14, 14), (32, 2048, 7, 7),
                                   (32, 1024, 14, 14), (2, 24, 5, 7), (3, 128, 9, 11)])
@pytest.mark.parametrize('relu,add', [(True, False), (True, True), (False, False)])
def test_fused_bn_matches_fp32_reference(shape, relu, add):
    N, C, H, W = shape
    x, z, dy = _case(N, C, H, W, seed=C + H)
    bn = _bn(C, seed=1)
    ref = copy.deepcopy(bn)
    assert fbn.eligible(x, bn, z if add else None)

    xr = x.float().detach().requires_grad_(True)
    zr = z.float().detach().requires_grad_(True)
    wr = ref.weight.detach().clone().requires_grad_(True)
    br = ref.bias.detach().clone().requires_grad_(True)
    yr = F.batch_norm(xr, ref.running_mean, ref.running_var, wr, br, True, ref.momentum, ref.eps)
    if add:
        yr = yr + zr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy.float())

    xf = x.detach().clone().requires_grad_(True)
    zf = z.detach().clone().requires_grad_(True)
    y = fbn.bn_act(xf, bn, relu=relu, z=zf if add else None)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    torch.cuda.synchronize()

    assert _rel(y, yr) < 4e-3, _rel(y, yr)                 # bf16 output rounding
    assert torch.allclose(bn.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(bn.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == 1
    assert _rel(xf.grad, xr.grad) < 1e-2, _rel(xf.grad, xr.grad)
    assert _rel(bn.weight.grad, wr.grad) < 1e-4, _rel(bn.weight.grad, wr.grad)
    assert _rel(bn.bias.grad, br.grad) < 1e-5, _rel(bn.bias.grad, br.grad)
    if add:
        assert _rel(zf.grad, zr.grad) < 4e-3


def test_fused_bn_deterministic_and_graph_capturable():
    x, z, dy = _case(16, 256, 14, 14, seed=5)
    outs = []
    for _ in range(2):
        bn = _bn(256, seed=2)
        xf = x.detach().clone().requires_grad_(True)
        y = fbn.bn_act(xf, bn, relu=True, z=z)
        y.backward(dy)
        outs.append((y, xf.grad, bn.weight.grad, bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # captured forward + backward == eager
    bn = _bn(256, seed=2)
    xs = x.detach().clone().requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = fbn.bn_act(xs, bn, relu=True, z=z)     # warm-up (allocations)
        y.backward(dy)
    torch.cuda.current_stream().wait_stream(s)
    bn2 = _bn(256, seed=2)
    xs2 = x.detach().clone().requires_grad_(True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y2 = fbn.bn_act(xs2, bn2, relu=True, z=z)
        y2.backward(dy)
    with torch.no_grad():
        bn2.running_mean.copy_(_bn(256, seed=2).running_mean)
        bn2.running_var.copy_(_bn(256, seed=2).running_var)
        bn2.num_batches_tracked.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y2, outs[0][0]) and torch.equal(xs2.grad, outs[0][1])
    assert torch.equal(bn2.running_var, outs[0][3])


def test_resnet_fused_bn_matches_stock_modules():
    """One training step of a Bottleneck ResNet: the bf16-autocast gradient
    with the fused BN kernels is as close to the fp32 step as the stock
    BatchNorm/ReLU modules' bf16 gradient (same yardstick: bf16 rounding
    compounds through the network at random init)."""
    from distributed_kfac_pytorch_amd.models import resnet
    torch.manual_seed(0)
    m0 = resnet.resnet_tiny(num_classes=10).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=DEV).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=DEV)
    runs = {}
    for tag, amp, fused in (('fp32', False, False), ('stock', True, False), ('fused', True, True)):
        m = copy.deepcopy(m0)
        fbn.ENABLED = fused
        try:
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
        finally:
            fbn.ENABLED = True
        runs[tag] = (torch.cat([p.grad.float().flatten() for p in m.parameters()]),
                     torch.cat([b.float().flatten() for b in m.buffers()]), loss.item())
    ref = runs['fp32']
    e_stock = _rel(runs['stock'][0], ref[0])
    e_fused = _rel(runs['fused'][0], ref[0])
    assert e_fused <= 1.5 * e_stock + 1e-2, (e_fused, e_stock)
    b_stock = _rel(runs['stock'][1], ref[1])
    b_fused = _rel(runs['fused'][1], ref[1])
    assert b_fused <= 1.5 * b_stock + 1e-3, (b_fused, b_stock)
    assert abs(runs['fused'][2] - ref[2]) <= 1.5 * abs(runs['stock'][2] - ref[2]) + 1e-2
