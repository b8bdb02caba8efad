"""End-to-end K-FAC on the MI355X vs the CPU (reference-numerics) path."""
import copy

import pytest
import torch
import torch.nn as nn

import distributed_kfac_pytorch_amd as kfac
from tests._oracle_common import SmallNet, build_case, run_steps

pytestmark = pytest.mark.gpu


def _run(device, steps=4, channels_last=False, **kw):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': steps})
    model = model.to(device)
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    data = [(x.to(device), y.to(device)) for x, y in data]
    if channels_last:
        data = [(x.contiguous(memory_format=torch.channels_last), y) for x, y in data]
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2, lr=0.05, damping=0.003, **kw)
    grads, factors = run_steps(model, pre, data, steps)
    return grads, factors, pre


@pytest.mark.parametrize('channels_last', [False, True])
@pytest.mark.parametrize('prediv', [True, False])
def test_gpu_matches_cpu(channels_last, prediv):
    g_cpu, f_cpu, _ = _run('cpu', precompute_outer_eigen=prediv)
    g_gpu, f_gpu, pre = _run('cuda', channels_last=channels_last, precompute_outer_eigen=prediv)
    for (a, g), (ca, cg) in zip(f_gpu, f_cpu):
        assert torch.allclose(a.cpu(), ca, rtol=1e-4, atol=1e-6)
        assert torch.allclose(g.cpu(), cg, rtol=1e-4, atol=1e-6)
    for step, (gs, cs) in enumerate(zip(g_gpu, g_cpu)):
        for x, y in zip(gs, cs):
            err = (x.cpu() - y).norm() / max(y.norm(), 1e-12)
            assert err < 2e-3, (step, err.item())


def test_gpu_inverse_path():
    """use_eigen_decomp=False: hand-written batched Cholesky inverse
    (csrc/chol.hip) and the 2-stage grouped pgemm chain G_inv Grad A_inv."""
    g_cpu, _, _ = _run('cpu', use_eigen_decomp=False)
    g_gpu, _, pre = _run('cuda', use_eigen_decomp=False)
    assert pre.fused is not None and pre.fused.inverse and len(pre.fused._stage_tables) == 2
    for gs, cs in zip(g_gpu, g_cpu):
        for x, y in zip(gs, cs):
            assert (x.cpu() - y).norm() / max(y.norm(), 1e-12) < 2e-3


def test_gpu_bf16_autocast_step_finite():
    from distributed_kfac_pytorch_amd.models import resnet_cifar
    torch.manual_seed(0)
    m = resnet_cifar.resnet20().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=2)
    x = torch.randn(32, 3, 32, 32, device='cuda').to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device='cuda')
    losses = []
    for _ in range(6):
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = nn.functional.cross_entropy(m(x), y)
        loss.backward()
        pre.step()
        opt.step()
        losses.append(loss.item())
    assert all(map(lambda v: v == v and abs(v) < 1e3, losses))
    assert losses[-1] < losses[0]
    # factors in the data dtype (bf16 under autocast), as in the reference
    assert pre.layers[1].state['A'].dtype == torch.bfloat16


def test_gpu_state_dict_roundtrip():
    # 3 steps with inv_update_freq=2: the last step recomputes the inverses
    # from the final factors, which is what load_state_dict recomputes too
    _, _, pre = _run('cuda', steps=3)
    sd = pre.state_dict(include_layer_inverses=True)
    model2 = SmallNet().cuda()
    pre2 = kfac.KFAC(model2, factor_update_freq=1, inv_update_freq=2, lr=0.05, damping=0.003)
    pre2.load_state_dict(copy.deepcopy(sd))
    for l1, l2 in zip(pre.layers, pre2.layers):
        assert torch.equal(l1.state['A'], l2.state['A'])
        assert torch.allclose(l1.state['dGdA'], l2.state['dGdA'], rtol=1e-3, atol=1e-3)


def test_gpu_inverse_many_size_classes():
    """Batched per-size-class Cholesky inverses (K9) on the GPU vs an fp64
    torch reference, ResNet-like mixed sizes."""
    from distributed_kfac_pytorch_amd.ops import eigen as eigen_ops
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(5)
    mats = []
    for n in (64, 576, 64, 1152, 576, 257):
        x = torch.randn(n, 2 * n, device=dev, generator=g)
        mats.append(x @ x.t() / (2 * n))
    outs = eigen_ops.inverse_many(mats, 0.003)
    for A, out in zip(mats, outs):
        M = A.double() + 0.003 * torch.eye(A.shape[0], device=dev, dtype=torch.float64)
        ref = torch.linalg.inv(M)
        assert (out.double() - ref).norm() / ref.norm() < 1e-4


def test_gpu_nonfinite_factor_raises_after_enqueue():
    """A NaN factor at an inverse step: no host read before the solve (the
    factor reaches the solvers as the identity, eigen.sanitize), no device
    fault, and step() still raises FloatingPointError -- after the step's work
    is enqueued (KFAC._finish_solver_check) -- naming the factor; the next
    inverse update with finite factors is clean again."""
    torch.manual_seed(0)
    model = SmallNet().cuda()
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2, lr=0.05, damping=0.003,
                    use_hip_graphs=False)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(8, 3, 8, 8, device='cuda')
    y = torch.randint(0, 10, (8,), device='cuda')

    def step():
        opt.zero_grad()
        nn.functional.cross_entropy(model(x), y).backward()
        pre.step()

    step()                                    # step 0: inverse update, finite
    step()                                    # step 1: plain
    layer = pre.layers[1]
    saved = layer.state['A'].clone()
    pre.compute_factor_in_hook = True         # keep the poisoned factor (no EMA in step())
    layer.state['A'].fill_(float('nan'))
    with pytest.raises(FloatingPointError, match='non-finite'):
        step()                                # step 2: inverse update over the NaN factor
    torch.cuda.synchronize()
    layer.state['A'].copy_(saved)
    pre.compute_factor_in_hook = False
    pre.param_groups[0]['step'] = 4
    step()                                    # step 4: inverse update, finite again
    torch.cuda.synchronize()
    for p in model.parameters():
        assert torch.isfinite(p.grad).all()
