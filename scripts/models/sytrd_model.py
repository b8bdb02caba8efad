"""NumPy model of the blocked Householder tridiagonalisation in csrc/eig_tridiag.hip.

Mirrors the kernels phase by phase (same buffers, same index conventions) so the
algorithm can be checked on the CPU:

  storage   row-major, UPPER triangle maintained (== LAPACK lower, column-major);
            row j of the working matrix is "column j"
  X         the current column's updated row: X[r] = A_upd[j, r], r >= j
  V, W      panel reflectors / LATRD w-vectors, n x nb
  phase A   v from X (Householder), symv y = A22 v on the stale panel-start matrix
            (upper tiles only), dot partials W^T v, V^T v
  phase B   w' = tau (y - V (W^T v) - W (V^T v)), partial w'^T v
  phase C   W[:, c] = w' + alpha2 v; next column's X with the panel corrections
  trailing  A[q:, q:] -= V W^T + W V^T (upper triangle), then prep X for column q
Output: d, e, tau and the reflectors in A[j, j+1:] (e_j at j+1, v[1:] after), the
layout rocSOLVER's ormtr (lower, column-major) reads.
"""
import numpy as np


def sytrd_upper(A, nb=32):
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(n)
    tau = np.zeros(n)
    X = A[0].copy()                      # prep(q=0)
    p = 0
    while p < n - 1:
        w = min(nb, n - 1 - p)           # columns p .. p+w-1 get reflectors
        V = np.zeros((n, nb))
        W = np.zeros((n, nb))
        S = A.copy()                     # the stale panel-start matrix (kernels read A itself)
        for c in range(w):
            j = p + c
            # ---- phase A: Householder of x = X[j+1:]
            alpha = X[j + 1]
            sigma2 = float(np.sum(X[j + 2:] ** 2))
            if sigma2 == 0.0:
                t, beta, scale = 0.0, alpha, 0.0
            else:
                beta = -np.copysign(np.sqrt(alpha * alpha + sigma2), alpha)
                t = (beta - alpha) / beta
                scale = 1.0 / (alpha - beta)
            v = np.zeros(n)
            v[j + 1] = 1.0
            v[j + 2:] = X[j + 2:] * scale
            tau[j], e[j], d[j] = t, beta, X[j]
            V[:, c] = v
            A[j, j + 1] = beta
            A[j, j + 2:] = v[j + 2:]
            # symv on the stale trailing matrix, upper storage of rows/cols > j
            U = np.triu(S)
            y = U @ v + np.triu(S, 1).T @ v
            y[:j + 1] = 0.0
            s1 = W[:, :c].T @ v
            s2 = V[:, :c].T @ v
            # ---- phase B
            wp = t * (y - V[:, :c] @ s1 - W[:, :c] @ s2)
            wp[:j + 1] = 0.0
            # ---- phase C
            alpha2 = -0.5 * t * float(wp @ v)
            W[:, c] = wp + alpha2 * v
            if c + 1 < w:
                jn = j + 1
                x = S[jn].copy()
                x -= V[:, :c + 1] @ W[jn, :c + 1] + W[:, :c + 1] @ V[jn, :c + 1]
                X = np.zeros(n)
                X[jn:] = x[jn:]
        # ---- trailing update + prep for the next panel
        q = p + w
        upd = V @ W.T + W @ V.T
        for r in range(q, n):
            A[r, r:] -= upd[r, r:]
        # keep the (unused) lower part consistent for the next panel's stale reads
        for r in range(q, n):
            A[r:, r] = A[r, r:]
        if q <= n - 1:
            X = np.zeros(n)
            X[q:] = A[q, q:]
        p = q
    d[n - 1] = X[n - 1]
    return d, e, tau, A


def check(n, nb, seed=0):
    rng = np.random.default_rng(seed)
    M = rng.standard_normal((n, n // 2))
    A0 = M @ M.T / n + 1e-3 * np.eye(n)
    d, e, tau, A = sytrd_upper(A0, nb)
    T = np.diag(d) + np.diag(e[:n - 1], 1) + np.diag(e[:n - 1], -1)
    ev_t = np.linalg.eigvalsh(T)
    ev = np.linalg.eigvalsh(A0)
    err = np.abs(ev_t - ev).max() / np.abs(ev).max()
    # Q from the reflectors: Q = H0 H1 ... ; check Q^T A0 Q == T
    Q = np.eye(n)
    for j in range(n - 1):
        v = np.zeros(n)
        v[j + 1] = 1.0
        v[j + 2:] = A[j, j + 2:]
        Q = Q @ (np.eye(n) - tau[j] * np.outer(v, v))
    resid = np.abs(Q.T @ A0 @ Q - T).max() / np.abs(A0).max()
    print('n=%d nb=%d  eigenvalue rel err %.2e   ||Q^T A Q - T|| %.2e' % (n, nb, err, resid))
    return err, resid


if __name__ == '__main__':
    for n, nb in ((5, 2), (17, 4), (64, 8), (100, 32), (130, 32), (257, 32)):
        check(n, nb)
