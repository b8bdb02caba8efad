"""Probe: the CNN example with --fp16 (GradScaler) eager / graphed, fused or
plain SGD: does training stay finite?"""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.getcwd())
from examples import torch_imagenet_resnet as ex  # noqa: E402

_SGD = torch.optim.SGD


def run(graphs, fused, bf16=False, kfac=True):
    def sgd(*a, **k):
        if not fused:
            k.pop('fused', None)
        return _SGD(*a, **k)
    torch.optim.SGD = sgd
    log = tempfile.mkdtemp()
    argv = ['--model', 'resnet_tiny', '--synthetic-size', '128', '--batch-size', '8',
            '--val-batch-size', '8', '--image-size', '32', '--checkpoint-freq', '0',
            '--epochs', '1', '--kfac-update-freq', '4', '--kfac-cov-update-freq', '2',
            '--deterministic', '--log-dir', log, '--graphs', str(graphs)]
    argv += [] if bf16 else ['--no-bf16', '--fp16']
    if not kfac:
        argv[argv.index('--kfac-update-freq') + 1] = '0'
    try:
        h = ex.main(argv)
        print('graphs', graphs, 'kfac', kfac, 'fused', fused, 'bf16', bf16, 'ok', h[-1]['train'],
              flush=True)
    except Exception as e:
        print('graphs', graphs, 'kfac', kfac, 'fused', fused, 'bf16', bf16, 'FAILED', str(e)[:160],
              flush=True)
    finally:
        torch.optim.SGD = _SGD


for g, f, b, k in [(1, False, False, False), (1, False, False, True)]:
    run(g, f, b, k)
