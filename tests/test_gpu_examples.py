"""The examples' MI355X fast path (--graphs 1: whole-step hipGraphs) trains
like the eager reference loop: fp32, deterministic MIOpen algorithms, final
weights equal to 1e-6 (verdict r2 item 7)."""
import os

import pytest
import torch

from tests import _dist_worker  # noqa: F401  (ROOT on sys.path)

pytestmark = pytest.mark.gpu


def _final_params(tmp_path, graphs, extra=(), size=64):
    from examples import torch_imagenet_resnet as ex
    log = os.path.join(str(tmp_path), 'g{}{}'.format(graphs, '_'.join(extra)))
    argv = ['--model', 'resnet_tiny', '--synthetic-size', str(size), '--batch-size', '8',
            '--val-batch-size', '8', '--image-size', '32', '--checkpoint-freq', '1',
            '--epochs', '1', '--kfac-update-freq', '4', '--kfac-cov-update-freq', '2',
            '--no-bf16', '--deterministic', '--log-dir', log, '--graphs', str(graphs)]
    argv += list(extra)
    hist = ex.main(argv)
    sd = torch.load(os.path.join(log, 'checkpoint_1.pth.tar'), map_location='cpu',
                    weights_only=False)['model']
    return hist, sd


def test_graphed_example_matches_eager(tmp_path):
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    try:
        h1, p1 = _final_params(tmp_path, 1)
        h0, p0 = _final_params(tmp_path, 0)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    num = sum(float((p1[k].double() - p0[k].double()).norm() ** 2) for k in p0
              if p0[k].is_floating_point()) ** 0.5
    den = sum(float(p0[k].double().norm() ** 2) for k in p0 if p0[k].is_floating_point()) ** 0.5
    assert num / den <= 1e-6, (num / den, h1, h0)
    assert abs(h1[0]['train']['loss'] - h0[0]['train']['loss']) <= 1e-6 * abs(h0[0]['train']['loss'])


def _rel(p1, p0):
    num = sum(float((p1[k].double() - p0[k].double()).norm() ** 2) for k in p0
              if p0[k].is_floating_point()) ** 0.5
    den = sum(float(p0[k].double().norm() ** 2) for k in p0 if p0[k].is_floating_point()) ** 0.5
    return num / den


@pytest.mark.parametrize('extra,tol', [(('--batches-per-allreduce', '2'), 1e-6),
                                       (('--fp16',), 1e-6),
                                       (('--fp16', '--batches-per-allreduce', '2'), 1e-6)])
def test_graphed_example_modes_match_eager(tmp_path, extra, tol):
    """The reference's micro-batching (engine.py:33-65) and fp16 + GradScaler
    (engine.py:73-82) on the graphed fast path (round 3 fell back to eager
    DDP for both): same final weights as the eager loop (torch GradScaler
    API there, amp.CapturableGradScaler's device-side skip when graphed)."""
    from distributed_kfac_pytorch_amd import graphs
    replays = []
    orig = graphs.GraphedTrainStep.__call__

    def spy(self, *a, **k):
        out = orig(self, *a, **k)
        replays.append(self.replays)
        return out
    graphs.GraphedTrainStep.__call__ = spy
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    try:
        # 128 images: enough steps per epoch to warm up, capture and replay
        h1, p1 = _final_params(tmp_path, 1, extra, size=128)
        h0, p0 = _final_params(tmp_path, 0, extra, size=128)
    finally:
        graphs.GraphedTrainStep.__call__ = orig
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert replays and replays[-1] > 0, 'the graphed loop never replayed a graph'
    assert all(torch.isfinite(v).all() for v in p1.values() if v.is_floating_point())
    assert _rel(p1, p0) <= tol, (_rel(p1, p0), h1, h0)
