"""K-FAC on the LSTM and Transformer language models: GPU kernels vs the CPU path."""
import pytest
import torch
import torch.nn as nn

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import LSTMModel, TransformerLM

pytestmark = pytest.mark.gpu


def _lm_grads(device, model_kind, steps=3):
    torch.manual_seed(0)
    if model_kind == 'lstm':
        m = LSTMModel(64, 32, 48, 2, dropout=0.0)
        acc = True
    else:
        m = TransformerLM(64, d_model=32, n_layers=2, n_heads=4, d_ff=64, max_len=16)
        acc = False
    m = m.to(device)
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=2, lr=0.1, damping=0.003,
                    skip_layers=['embedding'], accumulate_data=acc, batch_first=False,
                    use_hip_graphs=False)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(1)
    out = []
    for _ in range(steps):
        tokens = torch.randint(0, 64, (12, 4), generator=g).to(device)   # (T, B)
        targets = torch.randint(0, 64, (12 * 4,), generator=g).to(device)
        opt.zero_grad()
        if model_kind == 'lstm':
            logits, _ = m(tokens)
        else:
            logits = m(tokens.t().contiguous()).transpose(0, 1)
        loss = nn.functional.cross_entropy(logits.reshape(-1, 64), targets)
        loss.backward()
        pre.step()
        out.append([p.grad.detach().float().cpu().clone() for p in m.parameters()
                    if p.grad is not None])
        opt.step()
    return out


@pytest.mark.parametrize('kind', ['lstm', 'transformer'])
def test_language_models_gpu_match_cpu(kind):
    cpu = _lm_grads('cpu', kind)
    gpu = _lm_grads('cuda', kind)
    for step, (gs, cs) in enumerate(zip(gpu, cpu)):
        for a, b in zip(gs, cs):
            err = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
            assert err < 5e-3 * (10 ** step), (kind, step, err)
