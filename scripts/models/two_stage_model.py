"""fp64 model of the two-stage symmetric eigensolver in the exact data layouts
and operation order of csrc/eig_sy2sb.hip (stage 1), csrc/eig_sb2st.hip
(stage 2) and csrc/eig_q2.hip (stage-2 back-transformation); stage 3 is the
tridiagonal divide and conquer (csrc/eig_dc.hip), the stage-1
back-transformation the compact-WY kernel of csrc/eig_backtransform.hip with
shift = B.

Reference semantics: kfac/layers/utils.py:45-74 (eigenvalues ascending,
eigenvectors of a symmetric factor).

Layouts (row-major, the views the kernels use):
  stage 1  A full symmetric (lda >= n).  Panel p = rows j0 .. j0+B-1; its
           columns j0+B .. n-1 are QR-factorised as B row vectors (the
           transpose of LAPACK's column panel).  Reflector j = j0 + c is left
           in row j: beta at column j+B, v[1:] after it (the layout of the
           compact-WY back-transformation with shift B); tau1[j].
           Trailing update: X = A22 V T, N = T^T V^T X, Zm = X - V N / 2,
           A22 -= Zm V^T + V Zm^T.
  band     Bs[r][c - r + 2B - 1] = B[r][c] for r - 2B < c <= r (lower band,
           2B diagonals: the band plus room for the bulge).
  stage 2  task (s, j): c = s (j = 0) or s + 1 + (j-1) B; rows r0 = s+1+j B ..
           r1 = min(s + (j+1) B, n-1); reflector from B[r0..r1, c]; two-sided
           on the stored lower band.  (s+1, j) depends on (s, j+2).
           V2[s][j B + 0] = tau, V2[s][j B + i] = v[i] (v[0] = 1 implicit).
  stage 2  back-transformation on the row view of Z (row k = eigenvector k):
           for s descending, every step j of sweep s (disjoint components).
"""
import numpy as np


def house(x):
    """LAPACK larfg: (I - tau v v^T) x = beta e1, v[0] = 1."""
    alpha = x[0]
    sig = float(np.dot(x[1:], x[1:]))
    v = np.zeros_like(x)
    v[0] = 1.0
    if sig == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.sqrt(alpha * alpha + sig), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def larft(Vr, tau):
    """Forward columnwise T for H_0 H_1 .. = I - V T V^T, V given as rows Vr[c]."""
    k = Vr.shape[0]
    T = np.zeros((k, k))
    G = Vr @ Vr.T
    for i in range(k):
        T[i, i] = tau[i]
        if i:
            T[:i, i] = -tau[i] * (T[:i, :i] @ G[:i, i])
    return T


def sy2sb(A, B):
    """Stage 1 -> (A with reflectors in rows, tau1, band Bs)."""
    A = A.copy()
    n = A.shape[0]
    tau1 = np.zeros(n)
    for j0 in range(0, n, B):
        m = n - j0 - B
        if m < 1:
            break
        kb = min(B, m)          # reflectors of this panel (the last one may be short)
        nr = min(B, n - j0)     # panel rows: every one is transformed
        P = A[j0:j0 + nr, j0 + B:].copy()           # nr x m
        Vr = np.zeros((kb, m))
        tau = np.zeros(kb)
        for c in range(kb):
            v, t, beta = house(P[c, c:].copy())
            Vr[c, c:] = v
            tau[c] = t
            if c + 1 < nr:
                w = P[c + 1:, c:] @ v
                P[c + 1:, c:] -= t * np.outer(w, v)
            P[c, c] = beta
            P[c, c + 1:] = v[1:]
        A[j0:j0 + nr, j0 + B:] = P
        tau1[j0:j0 + kb] = tau
        T = larft(Vr, tau)
        A22 = A[j0 + B:, j0 + B:]
        V = Vr.T                                    # m x kb
        X = A22 @ V @ T
        N = T.T @ (V.T @ X)
        Zm = X - 0.5 * V @ N
        A22 -= Zm @ V.T + V @ Zm.T
    # band: B[r][c] = A[c][r] for c <= r, r - c <= B (upper storage of row c)
    Bs = np.zeros((n, 2 * B))
    for r in range(n):
        for c in range(max(0, r - B), r + 1):
            if r - c <= B and (r - c < B or True):
                # entry (c, r) of the upper band: diagonal block or the panel's R
                Bs[r, c - r + 2 * B - 1] = A[c, r] if c == r else _band_entry(A, c, r, B)
    return A, tau1, Bs


def _band_entry(A, c, r, B):
    """Upper band entry (c, r), 0 < r - c <= B, after stage 1: inside row c's
    panel diagonal block or in its reduced (R) part.  Row c's reflector
    occupies columns >= c + B, its beta at c + B."""
    return A[c, r]


def sb2st(Bs, n, B):
    """Stage 2 on the lower band storage -> (d, e, V2)."""
    W = 2 * B
    Bs = Bs.copy()

    def g(r, c):
        return Bs[r, c - r + W - 1]

    def s_(r, c, val):
        Bs[r, c - r + W - 1] = val

    J = (n + B - 1) // B + 1
    V2 = np.zeros((max(n - 1, 1), J * B))
    for s in range(n - 1):
        j = 0
        while True:
            c = s if j == 0 else s + 1 + (j - 1) * B
            r0 = s + 1 + j * B
            r1 = min(s + (j + 1) * B, n - 1)
            if r0 > n - 1 or r1 - r0 < 1:
                break
            L = r1 - r0 + 1
            x = np.array([g(r0 + i, c) for i in range(L)])
            v, t, beta = house(x)
            V2[s, j * B] = t
            V2[s, j * B + 1:j * B + L] = v[1:]
            s_(r0, c, beta)
            for i in range(1, L):
                s_(r0 + i, c, 0.0)
            if t != 0.0:
                # left: rows R x columns c+1 .. r0-1 (the bulge block)
                for k in range(c + 1, r0):
                    col = np.array([g(r0 + i, k) for i in range(L)])
                    col -= t * v * (v @ col)
                    for i in range(L):
                        s_(r0 + i, k, col[i])
                # both sides: diagonal block R x R (lower stored)
                D = np.zeros((L, L))
                for i in range(L):
                    for k in range(i + 1):
                        D[i, k] = D[k, i] = g(r0 + i, r0 + k)
                p = t * (D @ v)
                K = 0.5 * t * (v @ p)
                w = p - K * v
                D -= np.outer(v, w) + np.outer(w, v)
                for i in range(L):
                    for k in range(i + 1):
                        s_(r0 + i, r0 + k, D[i, k])
                # right: rows r1+1 .. min(r1+B, n-1) x columns R (the next bulge)
                for r in range(r1 + 1, min(r1 + B, n - 1) + 1):
                    row = np.array([g(r, r0 + k) for k in range(L)])
                    row -= t * (row @ v) * v
                    for k in range(L):
                        s_(r, r0 + k, row[k])
            j += 1
    d = np.array([g(r, r) for r in range(n)])
    e = np.array([g(r + 1, r) for r in range(n - 1)])
    return d, e, V2


def apply_q2(V2, n, B, Zr):
    """Zr (rows = eigenvectors, components along axis 1) <- (Q2 Z^T)^T."""
    Zr = Zr.copy()
    for s in reversed(range(n - 1)):
        j = 0
        while True:
            r0 = s + 1 + j * B
            r1 = min(s + (j + 1) * B, n - 1)
            if r0 > n - 1 or r1 - r0 < 1:
                break
            L = r1 - r0 + 1
            t = V2[s, j * B]
            v = np.concatenate([[1.0], V2[s, j * B + 1:j * B + L]])
            seg = Zr[:, r0:r1 + 1]
            seg -= t * np.outer(seg @ v, v)
            j += 1
    return Zr


def apply_q1(A, tau1, n, B, Zr):
    """Compact-WY stage-1 back-transformation on the row view (reflector j in
    row j of A: implicit 1 at column j+B, v after), Q1 = H_0 H_1 .."""
    Zr = Zr.copy()
    for j in reversed(range(n)):
        if tau1[j] == 0.0 or j + B >= n:
            continue
        v = np.concatenate([[1.0], A[j, j + B + 1:]])
        seg = Zr[:, j + B:]
        seg -= tau1[j] * np.outer(seg @ v, v)
    return Zr


def eigh_two_stage(A, B=16):
    n = A.shape[0]
    Ar, tau1, Bs = sy2sb(A, B)
    d, e, V2 = sb2st(Bs, n, B)
    T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    lam, Z = np.linalg.eigh(T)
    Zr = Z.T.copy()
    Zr = apply_q2(V2, n, B, Zr)
    Zr = apply_q1(Ar, tau1, n, B, Zr)
    return lam, Zr.T


if __name__ == '__main__':
    rng = np.random.default_rng(0)
    for n, B in [(5, 2), (19, 4), (40, 4), (97, 8), (130, 16), (200, 16), (33, 16), (17, 16)]:
        X = rng.standard_normal((n, n))
        A = X + X.T
        lam, Q = eigh_two_stage(A, B)
        res = np.abs(A @ Q - Q * lam).max() / np.abs(A).max()
        orth = np.abs(Q.T @ Q - np.eye(n)).max()
        ref = np.linalg.eigvalsh(A)
        print('n=%d B=%d  resid %.1e orth %.1e eig err %.1e' % (n, B, res, orth,
                                                               np.abs(lam - ref).max()))
        assert res < 1e-12 and orth < 1e-12 and np.abs(lam - ref).max() < 1e-10
