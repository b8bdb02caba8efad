"""NumPy model of the reduction's single-launch tail (csrc/eig_reduce.hip,
`red_tail_kernel`): the blocked F / U / S columns up to a panel start j0, then
ONE launch L(k) per column with the trailing matrix updated in place (rank 2,
unblocked) by the same launch that runs the symv.

L(k) uses only what the previous launch (S(j0) or L(k-1)) left behind:

  scalars  beta, tau, s of column k-1 from the global sums |xh|^2, xh.a, xh.yh
  row work v = e_k + s xh, w = tau (a + s yh) + alpha2 v           (rows >= k)
           x_k = a - w - w[k] v       (row k of A^(k): the next pivot row)
           a_k = A[k+1] - v[k+1] w - w[k+1] v                     (row k+1 of A^(k))
  tiles    A[r][c] -= v[r] w[c] + w[r] v[c] for r >= k+2 (stored), row k+1
           taken from a_k (it is read by every workgroup, so nobody stores it
           in that launch), then yh = A^(k)_22 xh_k

Invariant entering L(k): storage rows >= k+1 hold A^(k-1), `a` (slot AV) holds
row k of A^(k-1).  The blocked part is scripts/models/sytrd_fused_model.py.
"""
import numpy as np

from sytrd_fused_model import householder_scalars


def sytrd_hybrid(A, nb=32, j0=0):
    assert j0 % nb == 0
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(n)
    tau = np.zeros(n)
    V = np.zeros((n, nb))
    W = np.zeros((n, nb))
    prev = None
    for j in range(min(j0, n - 1) + 1):             # ---- blocked columns 0 .. j0
        c = j % nb
        snap_j, snap_j1 = A[j].copy(), (A[j + 1].copy() if j + 1 < n else None)
        if prev is not None:
            pc = prev['c']
            beta, t, s = householder_scalars(prev['alpha'], prev['sig2'])
            s1 = W[j, :pc] + s * prev['Wx']
            s2 = V[j, :pc] + s * prev['Vx']
            vy = prev['a'][j] + 2.0 * s * prev['xa'] + s * s * prev['xy']
            alpha2 = -0.5 * t * t * (vy - 2.0 * np.dot(s1, s2))
            v = np.zeros(n)
            v[j] = 1.0
            v[j + 1:] = s * prev['xh'][j + 1:]
            y = prev['a'] + s * prev['yh']
            w = t * (y - V[:, :pc] @ s1 - W[:, :pc] @ s2) + alpha2 * v
            w[:j] = 0.0
            W[:, pc] = w
            V[:, pc] = v
            d[j - 1], e[j - 1], tau[j - 1] = prev['d'], beta, t
            A[j - 1, j] = beta
            A[j - 1, j + 1:] = v[j + 1:]
        if c == 0 and j > 0:
            U = V @ W.T + W @ V.T
            m = np.zeros((n, n), dtype=bool)
            m[j:, j:] = True
            m &= np.triu(np.ones((n, n), dtype=bool))
            A[m] -= U[m]
            snap_j = snap_j - (V @ W[j] + W @ V[j])
            if snap_j1 is not None:
                snap_j1 = snap_j1 - (V @ W[j + 1] + W @ V[j + 1])
            V[:] = 0.0
            W[:] = 0.0
        x = snap_j - V[:, :c] @ W[j, :c] - W[:, :c] @ V[j, :c]
        if j == n - 1:
            d[j] = x[j]
            return d, e, tau, A
        xh = np.zeros(n)
        xh[j + 2:] = x[j + 2:]
        a = np.zeros(n)
        a[j + 1:] = snap_j1[j + 1:]
        B = np.triu(A)
        B = B + np.triu(B, 1).T
        A22 = np.zeros((n, n))
        A22[j + 1:, j + 1:] = B[j + 1:, j + 1:]
        yh = A22 @ xh
        prev = dict(alpha=x[j + 1], sig2=float(xh @ xh), Wx=W[:, :c].T @ xh, Vx=V[:, :c].T @ xh,
                    xa=float(xh @ a), xy=float(xh @ yh), xh=xh, yh=yh, a=a, c=c, d=x[j])
    # at j0 the panel was flushed (c == 0): the tail needs no V / W
    assert prev['c'] == 0
    for k in range(j0 + 1, n):                       # ---- tail launches L(k)
        beta, t, s = householder_scalars(prev['alpha'], prev['sig2'])
        a = prev['a']
        vy = a[k] + 2.0 * s * prev['xa'] + s * s * prev['xy']
        alpha2 = -0.5 * t * t * vy
        v = np.zeros(n)
        v[k] = 1.0
        v[k + 1:] = s * prev['xh'][k + 1:]
        w = t * (a + s * prev['yh']) + alpha2 * v
        w[:k] = 0.0
        d[k - 1], e[k - 1], tau[k - 1] = prev['d'], beta, t
        A[k - 1, k] = beta
        A[k - 1, k + 1:] = v[k + 1:]
        x = a - w - w[k] * v
        if k == n - 1:
            d[k] = x[k]
            break
        xh = np.zeros(n)
        xh[k + 2:] = x[k + 2:]
        an = np.zeros(n)
        an[k + 1:] = A[k + 1, k + 1:] - v[k + 1] * w[k + 1:] - w[k + 1] * v[k + 1:]
        for r in range(k + 2, n):                   # stored rows only
            A[r, r:] -= v[r] * w[r:] + w[r] * v[r:]
        B = np.triu(A)
        B = B + np.triu(B, 1).T
        A22 = np.zeros((n, n))
        A22[k + 1:, k + 1:] = B[k + 1:, k + 1:]
        A22[k + 1, k + 1:] = an[k + 1:]
        A22[k + 1:, k + 1] = an[k + 1:]
        yh = A22 @ xh
        prev = dict(alpha=x[k + 1], sig2=float(xh @ xh), xa=float(xh @ an),
                    xy=float(xh @ yh), xh=xh, yh=yh, a=an, d=x[k])
    return d, e, tau, A


def check(n, nb=32, j0=0, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, max(1, n // 2)))
    A = X @ X.T / X.shape[1] + 1e-3 * np.eye(n)
    d, e, tau, R = sytrd_hybrid(A, nb, j0)
    Q = np.eye(n)
    for j in range(n - 2, -1, -1):
        v = np.zeros(n)
        v[j + 1] = 1.0
        v[j + 2:] = R[j, j + 2:]
        Q = Q - tau[j] * np.outer(v, v @ Q)
    T = np.diag(d) + np.diag(e[:n - 1], 1) + np.diag(e[:n - 1], -1)
    err = np.abs(Q @ T @ Q.T - A).max() / np.abs(A).max()
    ev = np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A)).max() / np.abs(A).max()
    return err, ev


if __name__ == '__main__':
    for n, nb, j0 in [(2, 4, 0), (3, 4, 0), (5, 2, 2), (17, 4, 0), (17, 4, 8), (40, 8, 16),
                      (70, 32, 32), (130, 32, 64), (130, 32, 128), (129, 32, 96)]:
        print(n, nb, j0, check(n, nb, j0, seed=n))
