"""The example applications run end to end on CPU with synthetic data."""
import json
import os

import pytest

from tests import _dist_worker  # noqa: F401  (ROOT on sys.path)


def test_cifar_example_train_resume(tmp_path, capsys):
    from examples import torch_cifar10_resnet as ex
    argv = ['--model', 'resnet20', '--synthetic-size', '48', '--batch-size', '16',
            '--val-batch-size', '24', '--kfac-update-freq', '2', '--log-dir', str(tmp_path),
            '--checkpoint-freq', '1', '--warmup-epochs', '1', '--epochs', '1']
    hist = ex.main(argv)
    assert len(hist) == 1 and hist[0]['train']['loss'] > 0
    assert os.path.exists(os.path.join(str(tmp_path), 'checkpoint_1.pth.tar'))
    argv[-1] = '2'
    hist = ex.main(argv)       # resumes from epoch 1, trains epoch 2 only
    assert [h['epoch'] for h in hist] == [2]


@pytest.mark.parametrize('extra', [[], ['--use-inv-kfac', '--batches-per-allreduce', '2'],
                                   ['--kfac-update-freq', '0'], ['--graphs', '1']])
def test_imagenet_example_variants(tmp_path, extra):
    from examples import torch_imagenet_resnet as ex
    argv = ['--model', 'resnet_tiny', '--synthetic-size', '8', '--batch-size', '2',
            '--val-batch-size', '4', '--image-size', '32', '--log-dir', str(tmp_path),
            '--checkpoint-freq', '0', '--epochs', '1', '--kfac-update-freq', '2',
            '--kfac-cov-update-freq', '1'] + extra
    hist = ex.main(argv)
    assert hist[0]['train']['loss'] > 0


@pytest.mark.parametrize('model', ['lstm', 'transformer'])
def test_language_model_example(model):
    from examples import torch_language_model as ex
    argv = ['--model', model, '--epochs', '1', '--synthetic-tokens', '2000', '--vocab', '100',
            '--emsize', '32', '--nhid', '32', '--nlayers', '2', '--nheads', '4',
            '--batch-size', '4', '--bptt', '12']
    hist = ex.main(argv)
    assert hist[0]['train_loss'] > 0 and hist[0]['val_ppl'] > 1


def test_horovod_stubs_exit_with_instructions():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, 'examples', 'horovod_cifar10_resnet.py')],
                       capture_output=True, text=True)
    assert r.returncode == 2 and 'torch.distributed.run' in r.stderr


def test_lr_schedule_and_metric():
    import torch
    from examples.utils import Metric, create_lr_schedule, LabelSmoothLoss
    f = create_lr_schedule(4, 2, [5, 8])
    assert f(0) == pytest.approx(0.25) and f(2) == 1.0 and f(5) == pytest.approx(0.1)
    assert f(9) == pytest.approx(0.01)
    m = Metric('x')
    m.update(torch.tensor(1.0))
    m.update(torch.tensor(3.0))
    assert float(m.avg) == 2.0
    out = torch.randn(4, 5)
    tgt = torch.tensor([0, 1, 2, 3])
    assert torch.allclose(LabelSmoothLoss(0.0)(out, tgt), torch.nn.functional.cross_entropy(out, tgt))
