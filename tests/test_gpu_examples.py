"""The examples' MI355X fast path (--graphs 1: whole-step hipGraphs) trains
like the eager reference loop: fp32, deterministic MIOpen algorithms, final
weights equal to 1e-6 (verdict r2 item 7)."""
import os

import pytest
import torch

from tests import _dist_worker  # noqa: F401  (ROOT on sys.path)

pytestmark = pytest.mark.gpu


def _final_params(tmp_path, graphs):
    from examples import torch_imagenet_resnet as ex
    log = os.path.join(str(tmp_path), 'g{}'.format(graphs))
    argv = ['--model', 'resnet_tiny', '--synthetic-size', '64', '--batch-size', '8',
            '--val-batch-size', '8', '--image-size', '32', '--checkpoint-freq', '1',
            '--epochs', '1', '--kfac-update-freq', '4', '--kfac-cov-update-freq', '2',
            '--no-bf16', '--deterministic', '--log-dir', log, '--graphs', str(graphs)]
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
