"""NumPy model of the fused one-launch-per-column tridiagonalisation in
csrc/eig_reduce.hip (the F / U / S launches of one column).

Launch K(j), j = 0 .. n-1, does in ONE kernel what LAPACK latrd spreads over a
chain of BLAS-2 calls, using only data the previous launch left behind:

  step 1  scalars of column j-1 (beta, tau, scale s) from the previous launch's
          partial sums: |xh|^2, W^T xh, V^T xh, xh.a, xh^T yh
  step 2  w_{j-1} = tau (a + s yh - V s1 - W s2) + alpha2 v   (rows >= j)
          -> W[:, c-1], V[:, c-1], reflector row j-1, d/e/tau of column j-1
  panel   at a panel start (c == 0, j > 0): A_base -= V W^T + W V^T (upper)
  step 3  x_j = base row j - V W[j]^T - W V[j]^T (rows > j), d[j]; xh = x_j
          past j+1 (UNNORMALISED: the Householder scale needs a global norm,
          so the symv runs on xh and the scale is applied by K(j+1));
          partial sums |xh|^2, W^T xh, V^T xh, xh.a_j with a_j = base row j+1
  step 4  yh = A22_base xh (symv over upper tiles), tile partials xh^T yh

with y_{j} = A22 v_j = a_j + s_j yh_j because v_j = e_{j+1} + s_j xh_j.
Base rows j, j+1 come from a snapshot the previous launch took (at a panel
start the tiles are rewritten by the same launch).  Output layout = LAPACK
sytrd lower / column-major: d, e, tau, reflector j in row j (beta at j+1,
v[2:] after).
"""
import numpy as np


def householder_scalars(alpha, sig2):
    if sig2 == 0.0:
        return alpha, 0.0, 0.0          # beta, tau, scale
    beta = -np.copysign(np.sqrt(alpha * alpha + sig2), alpha)
    return beta, (beta - alpha) / beta, 1.0 / (alpha - beta)


def sytrd_fused(A, nb=32):
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    d = np.zeros(n)
    e = np.zeros(n)
    tau = np.zeros(n)
    V = np.zeros((n, nb))
    W = np.zeros((n, nb))
    prev = None     # what K(j-1) left: dict(alpha, sig2, Wx, Vx, xa, xy, xh, yh, a, c)
    for j in range(n):
        c = j % nb
        snap_j, snap_j1 = A[j].copy(), (A[j + 1].copy() if j + 1 < n else None)
        # ---- steps 1-2: finish column j-1 (panel position pc)
        if prev is not None:
            pc = prev['c']
            beta, t, s = householder_scalars(prev['alpha'], prev['sig2'])
            s1 = W[j, :pc] + s * prev['Wx']          # W^T v over rows >= j
            s2 = V[j, :pc] + s * prev['Vx']
            vy = prev['a'][j] + 2.0 * s * prev['xa'] + s * s * prev['xy']
            alpha2 = -0.5 * t * t * (vy - 2.0 * np.dot(s1, s2))
            v = np.zeros(n)
            v[j] = 1.0
            v[j + 1:] = s * prev['xh'][j + 1:]
            y = prev['a'] + s * prev['yh']           # rows >= j
            w = t * (y - V[:, :pc] @ s1 - W[:, :pc] @ s2) + alpha2 * v
            w[:j] = 0.0
            W[:, pc] = w
            V[:, pc] = v
            d[j - 1] = prev['d']
            e[j - 1] = beta
            tau[j - 1] = t
            A[j - 1, j] = beta
            A[j - 1, j + 1:] = v[j + 1:]
        # ---- panel start: trailing update of the base (upper triangle)
        if c == 0 and j > 0:
            U = V @ W.T + W @ V.T
            iu = np.triu_indices(n)
            mask = np.zeros((n, n), dtype=bool)
            mask[j:, j:] = True
            m2 = np.zeros((n, n), dtype=bool)
            m2[iu] = True
            A[mask & m2] -= U[mask & m2]
            # the launch computed x_j from the OLD snapshot minus the full
            # panel: identical to the updated row
            snap_j = snap_j - (V @ W[j] + W @ V[j])
            if snap_j1 is not None:
                snap_j1 = snap_j1 - (V @ W[j + 1] + W @ V[j + 1])
            V[:] = 0.0
            W[:] = 0.0
        # ---- step 3: x_j and its partial sums
        x = snap_j - V[:, :c] @ W[j, :c] - W[:, :c] @ V[j, :c]
        dj = x[j]
        if j == n - 1:
            d[j] = dj
            break
        alpha = x[j + 1]
        xh = np.zeros(n)
        xh[j + 2:] = x[j + 2:]
        a = np.zeros(n)
        a[j + 1:] = snap_j1[j + 1:]                  # column j+1 of A22 (base)
        # ---- step 4: symv on the base (upper triangle mirrored)
        B = np.triu(A)
        B = B + np.triu(B, 1).T
        A22 = np.zeros((n, n))
        A22[j + 1:, j + 1:] = B[j + 1:, j + 1:]
        yh = A22 @ xh
        prev = dict(alpha=alpha, sig2=float(xh @ xh), Wx=W[:, :c].T @ xh, Vx=V[:, :c].T @ xh,
                    xa=float(xh @ a), xy=float(xh @ yh), xh=xh, yh=yh, a=a, c=c, d=dj)
    return d, e, tau, A


def check(n, nb=32, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, max(1, n // 2)))
    A = X @ X.T / X.shape[1] + 1e-3 * np.eye(n)
    d, e, tau, R = sytrd_fused(A, nb)
    # Q = H_0 ... H_{n-2}, H_j = I - tau_j v_j v_j^T, v_j = e_{j+1} + R[j, j+2:]
    Q = np.eye(n)
    for j in range(n - 2, -1, -1):
        v = np.zeros(n)
        if j + 1 < n:
            v[j + 1] = 1.0
            v[j + 2:] = R[j, j + 2:]
        Q = Q - tau[j] * np.outer(v, v @ Q)
    T = np.diag(d) + np.diag(e[:n - 1], 1) + np.diag(e[:n - 1], -1)
    err = np.abs(Q @ T @ Q.T - A).max() / np.abs(A).max()
    ev = np.abs(np.linalg.eigvalsh(T) - np.linalg.eigvalsh(A)).max() / np.abs(A).max()
    return err, ev


if __name__ == '__main__':
    for n, nb in [(2, 4), (3, 4), (5, 2), (17, 4), (40, 8), (70, 32), (130, 32)]:
        print(n, nb, check(n, nb, seed=n))
