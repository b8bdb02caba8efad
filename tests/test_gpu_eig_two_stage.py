"""Two-stage eigensolver kernels against the fp64 model of the same
algorithm (scripts/models/two_stage_model.py) and against LAPACK eigenvalues."""
import importlib.util
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

_HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location(
    'two_stage_model', os.path.join(_HERE, '..', 'scripts', 'models', 'two_stage_model.py'))
model = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(model)


def _rand_band(n, b, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, n))
    A = np.tril(np.triu(X + X.T, -b), b)
    return A


@pytest.mark.parametrize('ns', [[40], [130], [17, 300, 64], [1100], [2100, 257]])
def test_sb2st_matches_model(ns):
    from distributed_kfac_pytorch_amd.ops import eig2s
    b = eig2s.BW
    As = [_rand_band(n, b, 7 + i) for i, n in enumerate(ns)]
    bands = [eig2s.pack_band(torch.tensor(A).cuda()) for A in As]
    outs = eig2s.sb2st(bands)
    torch.cuda.synchronize()
    for A, (d, e, v2) in zip(As, outs):
        n = A.shape[0]
        dm, em, refl, _ = model.sb2st(A, b)
        d, e, v2 = d.double().cpu().numpy(), e.double().cpu().numpy(), v2.double().cpu().numpy()
        T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
        lam = np.linalg.eigvalsh(T)
        ref = np.linalg.eigvalsh(A)
        assert np.abs(lam - ref).max() < 5e-5 * np.abs(ref).max() * max(1, n / 500)
        # d, e and the reflectors are not compared entry-wise: bulge chasing in
        # fp32 vs fp64 lands on a different (equally valid) tridiagonal form

@pytest.mark.parametrize('ns', [[64], [200], [33, 130, 515], [1152, 1024], [2304, 4608],
                                [33, 64, 147, 80] * 18])
def test_two_stage_eigh(ns):
    """Full pipeline (sy2sb, sb2st, divide and conquer, Q2, Q1) against fp64
    LAPACK: residual and orthogonality (SPD factors like K-FAC's)."""
    from distributed_kfac_pytorch_amd.ops import eig2s, eigen
    g = torch.Generator().manual_seed(3)
    mats = []
    for n in ns:
        X = torch.randn(n, max(8, n // 2), generator=g, dtype=torch.float64)
        A = X @ X.T / X.shape[1] + 1e-3 * torch.eye(n, dtype=torch.float64)
        mats.append(A)
    st = torch.cuda.current_stream()
    outs = eig2s.two_stage_group([A.float().cuda() for A in mats], None, st)
    torch.cuda.synchronize()
    eigen.check_solver_status()
    for A, (Q, D) in zip(mats, outs):
        Q, D = Q.double().cpu(), D.double().cpu()
        ref = torch.linalg.eigvalsh(A)
        nrm = torch.linalg.matrix_norm(A, 2)
        res = (A @ Q - Q * D).abs().max() / nrm
        orth = (Q.T @ Q - torch.eye(A.shape[0], dtype=torch.float64)).abs().max()
        assert (D - ref).abs().max() / nrm < 2e-5, (A.shape[0], float((D - ref).abs().max() / nrm))
        assert res < 2e-5, (A.shape[0], float(res))
        assert orth < 1e-4, (A.shape[0], float(orth))
