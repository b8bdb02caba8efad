"""Multi-step training quality of the CPU path against the reference K-FAC's
loss curve (tests/fixtures/training_quality_resnet20.pt, written by
scripts/make_training_fixture.py from /root/reference/kfac).  The CPU path is
the reference's math op for op (tests/test_reference_oracle.py pins it
bitwise per step on a small net), so the first 50 steps of ResNet-20 --
factors every step, five inverse updates -- must give the same losses, bit for bit.  The
GPU paths are held to the same fixture in tests/test_gpu_training_quality.py.
"""
import os

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from tests import _training_task as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fixture():
    return torch.load(os.path.join(ROOT, T.FIXTURE), weights_only=True)


def test_fixture_shape_and_learning():
    fx = fixture()
    assert fx['losses'].shape == (T.STEPS,) and len(fx['grads0']) == len(list(T.model().parameters()))
    w = T.window_means(fx['losses'].tolist())
    assert w[-1] < 0.5 * w[0]          # the task is learnable: the curve means something


def test_cpu_path_reproduces_reference_curve():
    fx = fixture()
    steps = 50
    net = T.model()
    pre = kfac.KFAC(net, **T.KFAC_KW)
    opt = torch.optim.SGD(net.parameters(), **T.SGD_KW)
    losses = []
    for i, (x, y) in enumerate(T.batches()[:steps]):
        opt.zero_grad()
        loss = T.loss_fn(net(x), y)
        loss.backward()
        pre.step()
        if i == 0:
            for g, r in zip((p.grad for p in net.parameters()), fx['grads0']):
                torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-7)
        opt.step()
        losses.append(float(loss))
    ref = fx['losses'][:steps].tolist()
    err = max(abs(a - b) for a, b in zip(losses, ref))
    assert err == 0.0, (err, losses, ref)          # bitwise: same ops, same order
