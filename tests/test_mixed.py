"""bf16-stored weights with fp32 masters (ops/mixed.BF16Weights) reproduce the
autocast trajectory: autocast's forward operand is the RNE bf16 cast of the
fp32 weight and its fp32 weight gradient the widened bf16 gradient, so K-FAC +
SGD steps on the masters must match K-FAC + SGD on fp32 weights under autocast."""
import copy

import pytest
import torch
import torch.nn.functional as F

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.ops.mixed import BF16Weights
from tests._oracle_common import SmallNet


def _data(steps):
    g = torch.Generator().manual_seed(5)
    return [(torch.randn(6, 3, 8, 8, generator=g), torch.randint(0, 10, (6,), generator=g))
            for _ in range(steps)]


def _run(model, params, pre, data, before_step=None, after_step=None):
    opt = torch.optim.SGD(params, lr=0.05, momentum=0.9, weight_decay=1e-4)
    losses = []
    for x, y in data:
        model.zero_grad(set_to_none=True)
        with torch.autocast('cpu', dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        if before_step is not None:
            before_step()
        pre.step()
        opt.step()
        if after_step is not None:
            after_step()
        losses.append(float(loss))
    return losses


@pytest.mark.parametrize('kfac_on', [True, False])
def test_bf16_weights_match_autocast(kfac_on):
    torch.manual_seed(0)
    ref = SmallNet()
    mp = copy.deepcopy(ref)
    data = _data(5)
    kw = dict(factor_update_freq=1, inv_update_freq=2, lr=0.05, damping=0.003)
    pre_ref = kfac.KFAC(ref, **kw) if kfac_on else None
    w = BF16Weights(mp)
    pre_mp = kfac.KFAC(mp, **kw) if kfac_on else None
    if kfac_on:
        pre_mp.set_grad_params(w.grad_params())

    class _Null(object):
        def step(self):
            pass
    l_ref = _run(ref, ref.parameters(), pre_ref or _Null(), data)
    l_mp = _run(mp, w.parameters(mp), pre_mp or _Null(), data,
                before_step=w.grads_to_master, after_step=w.master_to_model)
    assert all(p.dtype == torch.bfloat16 for p, _ in w.pairs)
    assert l_ref == l_mp, (l_ref, l_mp)
    masters = {id(p): m for p, m in w.pairs}
    for pr, pm in zip(ref.parameters(), mp.parameters()):
        master = masters.get(id(pm), pm)
        assert torch.equal(pr.detach(), master.detach()), (pr - master).abs().max()
        if master is not pm:
            assert torch.equal(pm.detach(), master.detach().to(torch.bfloat16))


def test_set_grad_params_rejects_overlap():
    m = SmallNet()
    w = BF16Weights(m)
    pre = kfac.KFAC(m, overlap_precondition=True)
    with pytest.raises(ValueError):
        pre.set_grad_params(w.grad_params())
