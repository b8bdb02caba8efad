"""CPU checks of the two-stage eigensolver's algorithm (the fp64 model the
HIP kernels follow: scripts/models/two_stage_model.py): band reduction,
bulge chasing in the kernels' wavefront order, grouped Q2 in the pass order."""
import importlib.util
import os

import numpy as np
import pytest

_HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location(
    'two_stage_model', os.path.join(_HERE, '..', 'scripts', 'models', 'two_stage_model.py'))
model = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(model)


@pytest.mark.parametrize('n,b', [(7, 2), (40, 4), (97, 8), (130, 16), (161, 16)])
def test_two_stage_model(n, b):
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, n))
    A = X + X.T
    Bf, panels = model.sy2sb(A, b)
    assert np.abs(np.tril(Bf, -b - 1)).max() < 1e-12            # banded
    band = np.tril(np.triu(Bf, -b), b)
    d, e, refl, Bt = model.sb2st(band, b)
    d2, e2, _, _ = model.sb2st(band, b, wavefront=True)         # the kernels' tick order
    assert np.abs(np.tril(Bt, -2)).max() < 1e-10                 # tridiagonal
    assert np.allclose(d, d2, atol=1e-12) and np.allclose(e, e2, atol=1e-12)
    T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    lam, Z = np.linalg.eigh(T)
    Zt = model.apply_q2_ticks(refl, n, b, Z.copy())              # the Q2 kernels' order
    Zg = model.apply_q2(model.q2_groups(refl, n, b, b), Z.copy())
    assert np.abs(Zt - Zg).max() < 1e-12
    Q = model.apply_q1(panels, Zt)
    assert np.abs(A @ Q - Q * lam).max() < 1e-11 * np.abs(A).max() * n
    assert np.abs(Q.T @ Q - np.eye(n)).max() < 1e-12
