"""CPU check of the blocked tridiagonalisation algorithm that csrc/eig_tridiag.hip
implements (NumPy model in scripts/models/sytrd_model.py, fp64)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    spec = importlib.util.spec_from_file_location(
        'sytrd_model', os.path.join(ROOT, 'scripts', 'models', 'sytrd_model.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize('n,nb', [(2, 32), (5, 2), (17, 4), (64, 8), (130, 32), (200, 32)])
def test_blocked_tridiagonalisation_model(n, nb):
    err, resid = _model().check(n, nb, seed=n)
    assert err < 1e-12 and resid < 1e-12
