"""Hand-written batched damped Cholesky inverse (csrc/chol.hip)
against fp64: every size class of one call in a single ragged launch
sequence, padding (n % 64 != 0) and the non-positive-definite error."""
import pytest
import torch

from distributed_kfac_pytorch_amd.ops import eigen

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _factor(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    A = (0.95 ** 20) * torch.eye(n, device=DEV, dtype=torch.float64)
    X = torch.randn(n, max(1, n // 3), device=DEV, dtype=torch.float64, generator=g)
    return A + 0.05 * X @ X.t() / X.shape[1]


def test_chol_inverse_sizes():
    sizes = [1, 2, 17, 64, 65, 128, 147, 300, 1025, 2049, 4608]
    damping = 1e-3
    mats64 = [_factor(n, 10 + i) for i, n in enumerate(sizes)]
    for _ in range(2):                  # plan build + graph replay
        outs = eigen.inverse_many([m.float() for m in mats64], damping)
        torch.cuda.synchronize()
    for n, A, X in zip(sizes, mats64, outs):
        Ad = A + damping * torch.eye(n, device=DEV, dtype=torch.float64)
        ref = torch.linalg.inv(Ad)
        err = ((X.double() - ref).norm() / ref.norm()).item()
        res = (Ad @ X.double() - torch.eye(n, device=DEV, dtype=torch.float64)).abs().max().item()
        assert X.shape == (n, n)
        assert err <= 1e-4 and res <= 1e-3, (n, err, res)
        assert torch.allclose(X, X.t(), atol=1e-6 * X.abs().max().item())


def test_chol_inverse_not_positive_definite():
    A = torch.eye(70, device=DEV)
    A[3, 3] = -1.0
    with pytest.raises(torch.linalg.LinAlgError):
        eigen.inverse_many([A], 1e-3)


def test_chol_plan_cache_bounded_over_damping_schedule():
    """A damping schedule and fresh factor snapshots make a new plan key per
    call; the plan cache evicts (LRU, kMaxPlans = 16) and stays correct."""
    n = 200
    A64 = _factor(n, 3)
    eye = torch.eye(n, device=DEV, dtype=torch.float64)
    for k in range(40):
        damping = 1e-3 * (1.0 + 0.05 * k)
        X = eigen.inverse_many([A64.float().clone()], damping)[0]
        if k % 13 == 0 or k == 39:
            res = ((A64 + damping * eye) @ X.double() - eye).abs().max().item()
            assert res <= 1e-3, (k, res)
    torch.cuda.synchronize()
