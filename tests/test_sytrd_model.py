"""CPU check of the fused one-launch-per-column tridiagonalisation recurrence
that csrc/eig_reduce.hip implements (unnormalised xh, Householder scalars one
launch late; NumPy fp64 model in scripts/models/sytrd_fused_model.py):
Q T Q^T reproduces A and T keeps A's spectrum."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    spec = importlib.util.spec_from_file_location(
        'sytrd_fused_model', os.path.join(ROOT, 'scripts', 'models', 'sytrd_fused_model.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize('n,nb', [(2, 32), (5, 2), (17, 4), (64, 8), (130, 32), (200, 32)])
def test_fused_tridiagonalisation_model(n, nb):
    err, ev = _model().check(n, nb, seed=n)
    assert err < 1e-12 and ev < 1e-12
