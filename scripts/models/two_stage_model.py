"""fp64 model of the two-stage symmetric eigensolver (csrc/eig_sy2sb.hip,
csrc/eig_sb2st.hip): the exact operation order the kernels use.

  stage 1  sy2sb: dense -> band (half-bandwidth b) by panels of b columns:
           Householder QR of the panel below the band, T factor (larft),
           X = A22 V T, W = X - V (T^T V^T X) / 2, A22 -= V W^T + W V^T.
  stage 2  sb2st: band -> tridiagonal by bulge chasing; sweep s annihilates
           column s, step j >= 1 the first column of the bulge its step j-1
           created.  Reflector (s, j) acts on rows s+1+j b .. s+(j+1) b.
  back     eigenvectors of A = Q1 Q2 Z.  Q2 Z in groups: sweeps
           [s0, s0+nb) at one step j form G = H(s0,j) ... H(s0+nb-1,j) =
           I - V T V^T (V staggered by one row); Q2 = prod_{s0 asc}
           prod_{j desc} G(s0, j), so Q2 Z applies blocks s0 descending and,
           inside a block, j ascending (reflectors of one sweep commute,
           sweeps s < s' at steps j < j' have disjoint supports).

Dependencies of stage 2 (used by the persistent kernel's progress counters):
task (s, j) touches rows s+1+(j-1) b .. s+(j+2) b; (s+1, j) may start once
(s, j+2) is done -- checked here by running the sweeps in that wavefront
order and comparing with the sweep-by-sweep result.
"""
import numpy as np


def house(x):
    """LAPACK larfg: H x = beta e1, H = I - tau v v^T, v[0] = 1."""
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


def larft(V, tau):
    """Forward, columnwise: H1 H2 ... Hk = I - V T V^T, T upper triangular."""
    k = V.shape[1]
    T = np.zeros((k, k))
    for i in range(k):
        T[i, i] = tau[i]
        if i:
            T[:i, i] = -tau[i] * (T[:i, :i] @ (V[:, :i].T @ V[:, i]))
    return T


def sy2sb(A, b):
    A = A.copy()
    n = A.shape[0]
    panels = []
    for k in range(0, n, b):
        m = n - k - b
        if m < 2:
            break
        kb = min(b, n - k)
        P = A[k + b:, k:k + kb].copy()
        nr = min(m, kb)
        V = np.zeros((m, nr))
        tau = np.zeros(nr)
        for i in range(nr):
            v, t, beta = house(P[i:, i])
            V[i:, i] = v
            tau[i] = t
            P[i:, i:] -= t * np.outer(v, v @ P[i:, i:])
            P[i, i] = beta
            P[i + 1:, i] = 0.0
        T = larft(V, tau)
        A[k + b:, k:k + kb] = P
        A[k:k + kb, k + b:] = P.T
        A22 = A[k + b:, k + b:]
        X = A22 @ V @ T
        W = X - 0.5 * V @ (T.T @ (V.T @ X))
        A22 -= V @ W.T + W @ V.T
        panels.append((k + b, V, T))
    return A, panels


def apply_q1(panels, Y):
    for r0, V, T in reversed(panels):
        Y[r0:] -= V @ (T @ (V.T @ Y[r0:]))
    return Y


def _task(B, n, b, s, j, refl):
    """One bulge-chasing step; returns False once the sweep has run off the end."""
    c = s if j == 0 else s + 1 + (j - 1) * b
    r0 = s + 1 + j * b
    r1 = min(s + (j + 1) * b, n - 1)
    if r0 > n - 1 or r1 - r0 < 1:
        return False
    v, t, beta = house(B[r0:r1 + 1, c].copy())
    lo, hi = max(0, r0 - 2 * b), min(n, r1 + 2 * b + 1)   # nonzeros of rows r0..r1
    B[r0:r1 + 1, lo:hi] -= t * np.outer(v, v @ B[r0:r1 + 1, lo:hi])
    B[lo:hi, r0:r1 + 1] -= t * np.outer(B[lo:hi, r0:r1 + 1] @ v, v)
    B[r0 + 1:r1 + 1, c] = 0.0
    B[c, r0 + 1:r1 + 1] = 0.0
    refl[(s, j)] = (r0, v, t)
    return True


def sb2st(Bband, b, wavefront=False):
    B = Bband.copy()
    n = B.shape[0]
    refl = {}
    if not wavefront:
        for s in range(n - 1):
            j = 0
            while _task(B, n, b, s, j, refl):
                j += 1
    else:
        # (s, j) at tick 3 s + j: (s+1, j) runs two ticks after (s, j+2)... i.e.
        # every task of a tick has disjoint support; order within a tick reversed
        # to show it does not matter
        done = {s: False for s in range(n - 1)}
        t = 0
        while not all(done.values()):
            for s in reversed(range(n - 1)):
                j = t - 3 * s
                if j < 0 or done[s]:
                    continue
                if not _task(B, n, b, s, j, refl):
                    done[s] = True
            t += 1
    d = np.diag(B).copy()
    e = np.diag(B, -1).copy()
    return d, e, refl, B


def q2_groups(refl, n, b, nb):
    """[(row0, V (rows x k), T)] in application order for Q2 Z."""
    sweeps = sorted({s for s, _ in refl})
    out = []
    for s0 in reversed(range(0, n - 1, nb)):
        j = 0
        while True:
            mem = [(s, refl[(s, j)]) for s in range(s0, min(s0 + nb, n - 1)) if (s, j) in refl]
            if not mem:
                if not any((s, jj) in refl for s in range(s0, min(s0 + nb, n - 1))
                           for jj in range(j, j + 2)):
                    break
                j += 1
                continue
            row0 = mem[0][1][0]
            rowe = max(r0 + len(v) for _, (r0, v, _) in mem)
            V = np.zeros((rowe - row0, len(mem)))
            tau = np.zeros(len(mem))
            for i, (s, (r0, v, t)) in enumerate(mem):
                V[r0 - row0:r0 - row0 + len(v), i] = v
                tau[i] = t
            out.append((row0, V, larft(V, tau)))
            j += 1
    del sweeps
    return out


def apply_q2(groups, Z):
    for row0, V, T in groups:
        r = slice(row0, row0 + V.shape[0])
        Z[r] -= V @ (T @ (V.T @ Z[r]))
    return Z


def apply_q2_ticks(refl, n, b, Z):
    """Q2 Z in the kernel's launch order: group (g, j) (sweeps b g .. b g+b-1
    at step j, nb = b) at tick (G-1-g) + j; groups of one tick touch
    disjoint row windows (asserted), so their order inside a tick is free."""
    G = (n - 1 + b - 1) // b
    groups = {}
    for (s, j), (r0, v, t) in refl.items():
        groups.setdefault((s // b, j), []).append((s, r0, v, t))
    ticks = {}
    for (g, j), mem in groups.items():
        ticks.setdefault(G - 1 - g + j, []).append((g, j, sorted(mem)))
    for t in sorted(ticks):
        seen = set()
        for g, j, mem in reversed(ticks[t]):
            row0 = b * g + 1 + b * j
            V = np.zeros((2 * b - 1, b))
            tau = np.zeros(b)
            for s, r0, v, tt in mem:
                i = s - b * g
                V[r0 - row0:r0 - row0 + len(v), i] = v
                tau[i] = tt
            rows = set(range(row0, min(row0 + 2 * b - 1, n)))
            assert not rows & seen
            seen |= rows
            T = larft(V, tau)
            w = min(2 * b - 1, n - row0)
            Z[row0:row0 + w] -= V[:w] @ (T @ (V[:w].T @ Z[row0:row0 + w]))
    return Z


def eigh_two_stage(A, b=16, nb=16):
    n = A.shape[0]
    Bfull, panels = sy2sb(A, b)
    band = np.tril(np.triu(Bfull, -b), b)
    d, e, refl, _ = sb2st(band, b)
    T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    lam, Z = np.linalg.eigh(T)
    Z = apply_q2(q2_groups(refl, n, b, nb), Z)
    Z = apply_q1(panels, Z)
    return lam, Z, Bfull


if __name__ == '__main__':
    rng = np.random.default_rng(0)
    for n, b, nb in [(7, 2, 2), (40, 4, 3), (97, 8, 8), (130, 16, 16), (200, 16, 5), (64, 16, 32)]:
        X = rng.standard_normal((n, n))
        A = X + X.T
        Bf, panels = sy2sb(A, b)
        assert np.abs(np.tril(Bf, -b - 1)).max() < 1e-12
        band = np.tril(np.triu(Bf, -b), b)
        d, e, refl, Bt = sb2st(band, b)
        d2, e2, refl2, _ = sb2st(band, b, wavefront=True)
        assert np.abs(np.tril(Bt, -2)).max() < 1e-10
        assert np.allclose(d, d2, atol=1e-12) and np.allclose(e, e2, atol=1e-12)
        lam, Z, _ = eigh_two_stage(A, b, nb)
        res = np.abs(A @ Z - Z * lam).max() / np.abs(A).max()
        orth = np.abs(Z.T @ Z - np.eye(n)).max()
        ref = np.linalg.eigvalsh(A)
        print('n=%d b=%d nb=%d  resid %.1e orth %.1e eig err %.1e  steps %d' %
              (n, b, nb, res, orth, np.abs(lam - ref).max(), len(refl)))
        assert res < 1e-12 and orth < 1e-12
        if nb == b:
            Z2 = apply_q2_ticks(refl, n, b, np.eye(n))
            Z1 = apply_q2(q2_groups(refl, n, b, nb), np.eye(n))
            assert np.abs(Z2 - Z1).max() < 1e-12, np.abs(Z2 - Z1).max()
