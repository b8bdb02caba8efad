"""Bit-level parity of the CPU path with the READ-ONLY reference (/root/reference).

The reference runs in a subprocess with its one required torch-2.x shim
(symeig -> linalg.eigh(...).contiguous()); factors and the KL-clipped,
preconditioned gradients of every step must be identical.  Skipped when the
reference tree is not mounted (e.g. on the GPU box).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from tests._oracle_common import build_case, run_steps

REF = os.environ.get('KFAC_REFERENCE', '/root/reference')
HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, 'kfac')),
                                reason='reference tree not available')

CONFIGS = [
    {},
    {'precompute_outer_eigen': False},
    {'use_eigen_decomp': False},
    {'kl_clip': None},
    {'comm_method': 'MEM_OPT'},
    {'factor_update_freq': 2, 'inv_update_freq': 4},
]


@pytest.mark.parametrize('extra', CONFIGS)
def test_matches_reference(tmp_path, extra):
    kw = {'factor_update_freq': 1, 'inv_update_freq': 2, 'lr': 0.05, 'damping': 0.003}
    kw.update(extra)
    cfg = {'seed': 0, 'batch': 6, 'steps': 5, 'kfac': kw}
    cfg_path = tmp_path / 'cfg.json'
    out_path = tmp_path / 'ref.pt'
    cfg_path.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1')
    r = subprocess.run([sys.executable, os.path.join(HERE, '_ref_oracle.py'), str(cfg_path),
                        str(out_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ref = torch.load(out_path, weights_only=True)
    model, data = build_case(cfg)
    mkw = dict(kw)
    mkw['comm_method'] = getattr(kfac.CommMethod, mkw.pop('comm_method', 'COMM_OPT'))
    pre = kfac.KFAC(model, **mkw)
    grads, factors = run_steps(model, pre, data, cfg['steps'])
    for (a, g), (ra, rg) in zip(factors, ref['factors']):
        assert torch.equal(a, ra) and torch.equal(g, rg)
    for gs, rgs in zip(grads, ref['grads']):
        for x, y in zip(gs, rgs):
            assert torch.equal(x, y), (x - y).abs().max()
