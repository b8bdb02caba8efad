"""bf16-stored weights with fp32 masters on the GPU (ops/mixed.BF16Weights,
csrc/mixed.hip): the grouped cast kernel equals torch's casts bit for bit, and
a graphed ResNet K-FAC + SGD run on bf16 weights follows the autocast run on
fp32 weights (same bf16 forward operands, same widened bf16 gradients)."""
import copy

import pytest
import torch
import torch.nn.functional as F

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd import graphs
from distributed_kfac_pytorch_amd.models import resnet
from distributed_kfac_pytorch_amd.ops.mixed import BF16Weights

pytestmark = pytest.mark.gpu


def test_grouped_cast_matches_torch():
    torch.manual_seed(0)
    shapes = [(64, 3, 7, 7), (1000, 2048), (1000,), (13,), (7, 5, 3, 3), (256, 64, 1, 1)]
    m = torch.nn.Module()
    mods = []
    for i, s in enumerate(shapes):
        if len(s) == 4:
            c = torch.nn.Conv2d(s[1], s[0], s[2], bias=False)
        else:
            c = torch.nn.Linear(s[-1] if len(s) == 2 else 4, s[0], bias=len(s) == 1)
        mods.append(c)
        m.add_module('m%d' % i, c)
    m = m.cuda().to(memory_format=torch.channels_last)
    ref = [p.detach().clone() for p in m.parameters()]
    w = BF16Weights(m)
    for (p, master), r in zip(w.pairs, ref):
        assert torch.equal(master.detach(), r)
        master.data.mul_(1.7).add_(0.3)
    w.master_to_model()
    for p, master in w.pairs:
        assert torch.equal(p.detach(), master.detach().to(torch.bfloat16))
        assert p.stride() == master.stride()
        p.grad = (torch.randn_like(master) * 3).to(torch.bfloat16)
    w.grads_to_master()
    torch.cuda.synchronize()
    for p, master in w.pairs:
        assert torch.equal(master.grad, p.grad.float())


def _train(bf16, steps=8):
    torch.manual_seed(0)
    model = resnet.resnet_tiny(num_classes=10).cuda().to(memory_format=torch.channels_last)
    weights = BF16Weights(model) if bf16 else None
    params = weights.parameters(model) if bf16 else model.parameters()
    opt = torch.optim.SGD(params, lr=0.05, momentum=0.9, weight_decay=5e-5)
    pre = kfac.KFAC(model, factor_update_freq=2, inv_update_freq=4, lr=0.05,
                    precond_precision='bf16x6')
    if bf16:
        pre.set_grad_params(weights.grad_params())
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = [torch.randn(8, 3, 32, 32, device='cuda', generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (8,), device='cuda', generator=g) for _ in range(steps)]
    x = torch.empty_like(xs[0]).contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(ys[0])

    def step_fn():
        model.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        if bf16:
            weights.grads_to_master()
        pre.step()
        opt.step()
        if bf16:
            weights.master_to_model()
        return loss

    step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1, enabled=True)
    losses = []
    for i in range(steps):
        x.copy_(xs[i])
        y.copy_(ys[i])
        losses.append(float(step().item()))
    torch.cuda.synchronize()
    final = [p.detach().clone() for p in (weights.parameters(model) if bf16
                                          else model.parameters())]
    return losses, final, step


def test_bf16_weights_follow_autocast_run():
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        l0, p0, _ = _train(False)
        l1, p1, s1 = _train(True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert s1.replays > 0
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (l0, l1)
    num = sum((a.double() - b.double()).norm() ** 2 for a, b in zip(p0, p1)) ** 0.5
    den = sum(a.double().norm() ** 2 for a in p0) ** 0.5
    assert float(num / den) < 1e-5, float(num / den)
