"""Warm-started eigendecomposition refresh of slowly drifting K-FAC factors.

Between two inverse updates a factor moves by a few EMA updates
(reference: kfac/layers/base.py:381-417, update_running_avg with decay 0.95;
eigendecompositions every `inv_update_freq` steps, kfac/layers/utils.py:45-74).
The previous eigenbasis X0 then nearly diagonalises the new factor A:
S = X0^T A X0 has a dominant diagonal, and what is left is two kinds of
coupling:

  * between eigenvalues far apart in the sorted spectrum: small rotation
    angles e_ij = s_ij / (s_jj - s_ii), resolved to second order by one
    Newton step X <- X (I + E) (the Jacobi-like refinement of Ogita and
    Aishima, 2018), whose error is squared every iteration;
  * between neighbours in the sorted spectrum whose gap is comparable to
    the coupling: resolved exactly by eigendecompositions of the diagonal
    windows of S (size `window`, offset by half a window every other
    iteration so no boundary stays a boundary).

Every step is a GEMM (A X, X^T Y, X^T X, X M) or a batched small
eigenproblem, so the refresh maps onto MFMA GEMMs and the batched LDS Jacobi
kernel instead of the latency-bound column chain of a full tridiagonal
reduction.  The iteration stops when the largest off-diagonal entry of
X^T A X is below tol * |lambda|_max (a backward error on par with a full
fp32 solve); when it does not get there within max_iter the caller falls
back to the full solver.

This module holds the torch reference of the algorithm (any dtype/device;
the oracle of the GPU path's tests).
"""
import torch

__all__ = ['refine_reference', 'window_bounds']


def window_bounds(n, window, it):
    """Half-open [a, b) diagonal windows of iteration `it`: size `window`,
    shifted by window // 2 on odd iterations."""
    off = (it % 2) * (window // 2)
    cuts = [0] + list(range(off if off > 0 else window, n, window)) + [n]
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def _window_rotation(S, bounds):
    """Block-diagonal orthogonal W whose blocks diagonalise S's windows."""
    n = S.shape[0]
    W = torch.zeros_like(S)
    sizes = {}
    for a, b in bounds:
        sizes.setdefault(b - a, []).append(a)
    for m, starts in sizes.items():
        blk = torch.stack([S[a:a + m, a:a + m] for a in starts])
        blk = 0.5 * (blk + blk.transpose(1, 2))
        _, V = torch.linalg.eigh(blk)
        for k, a in enumerate(starts):
            W[a:a + m, a:a + m] = V[k]
    return W


def refine_reference(A, X0, window=128, max_iter=8, tol=1e-7, theta=0.1):
    """Refine approximate eigenvectors X0 (columns) of the symmetric A.

    Returns (X, d, hist): X with orthonormal columns sorted by ascending
    Rayleigh quotient d, and hist = the relative off-diagonal max of
    X^T A X at the start of every iteration (hist[-1] <= tol on success).
    """
    n = A.shape[0]
    dt = A.dtype
    eye = torch.eye(n, dtype=dt, device=A.device)
    X = X0.to(dt).clone()
    hist = []
    d = None
    for it in range(max_iter + 1):
        # orthonormalise (Cholesky QR: X^T X = L L^T, X <- X L^-T)
        L = torch.linalg.cholesky(X.t() @ X)
        X = torch.linalg.solve_triangular(L, X.t(), upper=False).t()
        S = X.t() @ (A @ X)
        S = 0.5 * (S + S.t())
        d = S.diagonal()
        perm = torch.argsort(d)
        X = X[:, perm]
        S = S[perm][:, perm]
        d = S.diagonal().clone()
        scale = float(d.abs().max().clamp_min(torch.finfo(dt).tiny))
        off = S - torch.diag(d)
        hist.append(float(off.abs().max()) / scale)
        if hist[-1] <= tol or it == max_iter:
            break
        bounds = window_bounds(n, window, it)
        W = _window_rotation(S, bounds)
        S = W.t() @ S @ W
        X = X @ W
        mu = S.diagonal()
        bid = torch.empty(n, dtype=torch.long, device=A.device)
        for k, (a, b) in enumerate(bounds):
            bid[a:b] = k
        den = mu[None, :] - mu[:, None]
        same = bid[:, None] == bid[None, :]
        tiny = den.abs() <= torch.finfo(dt).tiny * 1e3
        E = S / torch.where(same | tiny, torch.ones_like(den), den)
        E = torch.where(same | tiny | (E.abs() > theta), torch.zeros_like(E), E)
        X = X + X @ E
    return X, d, hist
