"""NumPy model of the batched tridiagonal divide-and-conquer eigensolver in
csrc/eig_dc.hip (replaces rocSOLVER's stedc).

Mirrors the kernels step by step, with the same buffers and index conventions,
so the algorithm can be checked on the CPU:

  tree      recursive halving of [0, n) down to leaves of <= LEAF rows (Cuppen's
            tearing: T = diag(T1', T2') + |b| w w^T, w = e_{mid-1} + sgn(b) e_mid,
            the diagonal at each tear reduced by |b|)
  leaf      dense eigensolver of the torn leaf block (GPU: LDS Jacobi), ascending
  storage   Z (n x n, fp32, row-major): ROW i of a node's block is eigenvector i
            of that node's matrix in the node's own columns [lo, hi); every node
            output is TWO ascending runs of eigenvalues (dval, fp64): the
            non-deflated roots [lo, lo+k) and the deflated values [lo+k, hi)
  prep      z from the children's boundary columns; 4-run merge by rank; LAPACK
            dlaed2 deflation scan (small rho*z, and Givens rotations for close
            poles with the deflated run kept sorted by insertion); the surviving
            poles grouped into types (1 = left-only rows, 2 = mixed by a
            rotation, 3 = right-only) so the eigenvector GEMMs skip the
            structural zeros
  rotate    the recorded Givens rotations applied to the node's rows, in order
  gather    ZpT[c][j] = Z[src_j][c] (type order), deflated rows -> scratch
  secular   one root per wave in fp64: Li's "middle way" two-pole model with a
            bracket safeguard (geometric bisection near a pole); eigenvector
            u_j = w_j / (d_j - lambda) normalised, into U (type order).  fp64
            roots of the fp32 rank-one problem give eigenvectors orthogonal to
            fp32 precision without the Gu-Eisenstat z recomputation
  gemm      Z[:, left cols]  = U[:, type 1+2] ZpT[left, type 1+2]^T
            Z[:, right cols] = U[:, type 2+3] ZpT[right, type 2+3]^T  (f32 MFMA)
  final     the root's two runs merged into ascending order (rows permuted)
"""
import numpy as np

EPS32 = float(np.finfo(np.float32).eps) / 2   # LAPACK slamch('E')
EPS64 = float(np.finfo(np.float64).eps) / 2
LEAF = 64
MAX_IT = 64


def build_tree(n, leaf=LEAF):
    """Nodes (lo, mid, hi, height); children before parents."""
    nodes = []

    def rec(lo, hi):
        if hi - lo <= leaf:
            nodes.append((lo, None, hi, 0))
            return 0
        mid = lo + (hi - lo) // 2
        h = 1 + max(rec(lo, mid), rec(mid, hi))
        nodes.append((lo, mid, hi, h))
        return h

    rec(0, n)
    return nodes


def _runs_merge(vals, runs):
    """Merge ascending runs [(start, end)] of `vals` (local) by rank: rank of an
    element = its index in its run + #elements of every other run that sort
    before it (ties: earlier run first) -> perm[p] = local index."""
    m = sum(e - s for s, e in runs)
    perm = np.empty(m, dtype=np.int64)
    for r, (s, e) in enumerate(runs):
        for i in range(s, e):
            v = vals[i]
            rank = i - s
            for r2, (s2, e2) in enumerate(runs):
                if r2 == r:
                    continue
                seg = vals[s2:e2]
                rank += int(np.searchsorted(seg, v, side='right' if r2 < r else 'left'))
            perm[rank] = i
    return perm


def deflate(ds, zs, src, typ, rho):
    """LAPACK dlaed2-style scan in ascending pole order.  Returns the
    non-deflated poles (d, z, src row, type), the deflated run (d, src row;
    ascending) and the rotation list (row p, row q, c, s)."""
    m = len(ds)
    ds = ds.copy()
    zs = zs.copy()
    typ = typ.copy()
    tol = 8.0 * EPS32 * max(float(np.max(np.abs(ds))), rho * float(np.max(np.abs(zs))))
    nd, defl, rots = [], [], []

    def push_defl(d, s):
        defl.append((d, s))
        i = len(defl) - 1           # insertion: keep the deflated run ascending
        while i > 0 and defl[i - 1][0] > defl[i][0]:
            defl[i - 1], defl[i] = defl[i], defl[i - 1]
            i -= 1

    pj = -1
    for p in range(m):
        if rho * abs(zs[p]) <= tol:
            push_defl(ds[p], src[p])
            continue
        if pj < 0:
            pj = p
            continue
        s = zs[pj]
        c = zs[p]
        tau = float(np.hypot(c, s))
        t = ds[p] - ds[pj]
        c /= tau
        s = -s / tau
        if abs(t * c * s) <= tol:
            zs[p] = tau
            zs[pj] = 0.0
            rots.append((src[pj], src[p], c, s))
            tmp = ds[pj] * c * c + ds[p] * s * s
            ds[p] = ds[pj] * s * s + ds[p] * c * c
            ds[pj] = tmp
            if typ[p] != typ[pj]:
                typ[p] = 2
            push_defl(ds[pj], src[pj])
        else:
            nd.append((ds[pj], zs[pj], src[pj], typ[pj]))
        pj = p
    if pj >= 0:
        nd.append((ds[pj], zs[pj], src[pj], typ[pj]))
    return nd, defl, rots


def _quad_root(qa, qb, qc, tl, th):
    """The root of qa t^2 + qb t + qc in (tl, th) (NaN if none), by the
    cancellation-free pair of formulas."""
    if qa == 0.0:
        return -qc / qb if qb != 0.0 else np.nan
    disc = qb * qb - 4.0 * qa * qc
    if disc < 0.0:
        disc = 0.0
    sq = np.sqrt(disc)
    q = -0.5 * (qb + (sq if qb >= 0.0 else -sq))
    r1 = q / qa
    r2 = qc / q if q != 0.0 else np.nan
    if tl < r1 < th:
        return r1
    return r2


def secular_root(i, dl, w, rho):
    """Root i of 1 + rho sum w_j^2 / (dl_j - x) = 0 -> (origin index, tau)
    with lambda = dl[origin] + tau, in fp64 (the kernel's algorithm)."""
    k = len(dl)
    w2 = rho * w * w
    if i < k - 1:
        gap = dl[i + 1] - dl[i]
        mid = 0.5 * gap
        fm = 1.0 + np.sum(w2 / ((dl - dl[i]) - mid))
        if fm >= 0.0:
            o, lo, hi = i, 0.0, mid
        else:
            o, lo, hi = i + 1, -mid, 0.0
    else:
        o, lo, hi = k - 1, 0.0, float(np.sum(w2))
    delta = dl - dl[o]
    left = o if o == i else o - 1          # pole index at the interval's left end
    right = left + 1 if left + 1 < k else -1
    # start: midpoint of the bracket, or its geometric split near the pole
    x = 0.5 * (lo + hi)
    for _ in range(MAX_IT):
        den = delta - x
        terms = w2 / den
        f = 1.0 + np.sum(terms)
        # f is zero to rounding: |f| within a few ulps of its summed magnitude
        if abs(f) <= 16.0 * EPS64 * (1.0 + np.sum(np.abs(terms))):
            break
        if f < 0.0:
            lo = x
        else:
            hi = x
        if hi - lo <= 4.0 * EPS64 * max(abs(lo), abs(hi)):
            break
        # middle way: psi (poles <= left) and phi (poles >= right) each by one
        # pole matched in value and derivative at x
        dterms = terms / den
        psi = np.sum(terms[:left + 1])
        dpsi = np.sum(dterms[:left + 1])
        a = delta[left]
        B = dpsi * (a - x) ** 2
        A = psi - B / (a - x)
        if right >= 0:
            phi = np.sum(terms[right:])
            dphi = np.sum(dterms[right:])
            b = delta[right]
            E = dphi * (b - x) ** 2
            C = phi - E / (b - x)
            K = 1.0 + A + C
            # K (a-y)(b-y) + B (b-y) + E (a-y) = 0 for the root y in (a, b),
            # solved for the offset from the ORIGIN pole (a = 0 or b = 0):
            # no cancellation when the root hugs that pole
            g = b - a
            if o == left:      # y = t, t in (0, g): K t^2 - (K g + B + E) t + B g = 0
                qa, qb, qc = K, -(K * g + B + E), B * g
                tl, th = 0.0, g
            else:              # y = t, t in (-g, 0): K t^2 + (K g - B - E) t - E g = 0
                qa, qb, qc = K, K * g - B - E, -E * g
                tl, th = -g, 0.0
            y = _quad_root(qa, qb, qc, tl, th)
        else:
            K = 1.0 + A
            y = a + B / K if K > 0.0 else np.nan
        if np.isfinite(y) and abs(y - x) <= 4.0 * EPS64 * abs(x):
            x = y            # converged (the model step is at rounding level)
            break
        if not (lo < y < hi) or not np.isfinite(y):
            # bracket safeguard: geometric split when the bracket touches the
            # pole (0) or spans orders of magnitude on one side of it
            if lo == 0.0:
                y = hi * 0.0625 if hi > 0.0 else 0.5 * (lo + hi)
            elif hi == 0.0:
                y = lo * 0.0625
            elif lo > 0.0 and hi > 8.0 * lo:
                y = np.sqrt(lo * hi)
            elif hi < 0.0 and lo < 8.0 * hi:
                y = -np.sqrt(lo * hi)
            else:
                y = 0.5 * (lo + hi)
        x = y
    return o, x


def merge(Z, dval, kk, lo, mid, hi, e):
    n1, m = mid - lo, hi - lo
    beta = float(e[mid - 1])
    rho = abs(beta)
    sgn = 1.0 if beta >= 0.0 else -1.0
    loc = np.arange(m)
    z = np.where(loc < n1, Z[lo + loc, mid - 1].astype(np.float64),
                 sgn * Z[lo + loc, mid].astype(np.float64))
    d = dval[lo:hi].copy()
    kl, kr = kk[lo], kk[mid]
    runs = [(0, kl), (kl, n1), (n1, n1 + kr), (n1 + kr, m)]
    perm = _runs_merge(d, runs)
    nz2 = float(np.sum(z * z))
    z /= np.sqrt(nz2)
    rho *= nz2
    nd, defl, rots = deflate(d[perm], z[perm], perm, np.where(perm < n1, 1, 3), rho)
    k = len(nd)
    dl = np.array([x[0] for x in nd])
    w = np.array([x[1] for x in nd])
    assert np.all(np.diff(dl) > 0), 'poles not strictly ascending'
    typ = np.array([x[3] for x in nd], dtype=np.int64)
    order = np.concatenate([np.nonzero(typ == t)[0] for t in (1, 2, 3)]).astype(np.int64)
    typepos = np.empty(k, dtype=np.int64)
    typepos[order] = np.arange(k)
    k1, k2 = int(np.sum(typ == 1)), int(np.sum(typ == 2))
    gsrc = np.array([nd[p][2] for p in order], dtype=np.int64)
    # rotate (node rows, all m columns), in order
    blk = Z[lo:hi, lo:hi]
    for pr, qr, c, s in rots:
        x = blk[pr].astype(np.float64)
        y = blk[qr].astype(np.float64)
        blk[pr] = (c * x + s * y).astype(np.float32)
        blk[qr] = (c * y - s * x).astype(np.float32)
    ZpT = blk[gsrc].T.copy() if k else np.zeros((m, 0), np.float32)   # [c][j]
    Dbuf = blk[[s for _, s in defl]].copy()
    # secular equation, eigenvectors in type order
    U = np.zeros((k, k), dtype=np.float32)
    lam = np.zeros(k)
    for i in range(k):
        o, tau = secular_root(i, dl, w, rho)
        lam[i] = dl[o] + tau
        u = w / ((dl - dl[o]) - tau)
        u /= np.linalg.norm(u)
        U[i, typepos] = u.astype(np.float32)
    out = np.zeros((m, m), dtype=np.float32)
    if k:
        jl = k1 + k2
        out[:k, :n1] = U[:, :jl] @ ZpT[:n1, :jl].T
        out[:k, n1:] = U[:, k1:] @ ZpT[n1:, k1:].T
    out[k:] = Dbuf
    Z[lo:hi, lo:hi] = out
    dval[lo:lo + k] = lam
    dval[lo + k:hi] = [v for v, _ in defl]
    kk[lo] = k
    return k, len(rots)


def dc_eigh(d, e, leaf=LEAF, stats=None):
    """Eigen-decomposition of the symmetric tridiagonal (d, e[:n-1]) -> (lam
    ascending, Z rows = eigenvectors), fp32 storage as on the GPU."""
    n = len(d)
    d = np.asarray(d, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    Z = np.zeros((n, n), dtype=np.float32)
    dval = np.zeros(n)
    kk = np.zeros(n, dtype=np.int64)          # node -> k (indexed by node lo)
    nodes = build_tree(n, leaf)
    dt = d.copy()
    for lo, mid, hi, h in nodes:              # tears
        if mid is not None:
            dt[mid - 1] -= abs(e[mid - 1])
            dt[mid] -= abs(e[mid - 1])
    for lo, mid, hi, h in sorted(nodes, key=lambda x: x[3]):
        if mid is None:
            T = np.diag(dt[lo:hi]) + np.diag(e[lo:hi - 1], 1) + np.diag(e[lo:hi - 1], -1)
            lam, V = np.linalg.eigh(T)
            Z[lo:hi, lo:hi] = V.T.astype(np.float32)
            dval[lo:hi] = lam
            kk[lo] = hi - lo
        else:
            k, nr = merge(Z, dval, kk, lo, mid, hi, e)
            if stats is not None:
                stats.append((hi - lo, k, nr))
    k = kk[0]
    perm = _runs_merge(dval, [(0, k), (k, n)])
    return dval[perm], Z[perm]


def kfac_like(n, rank, seed=0):
    """A K-FAC-shaped SPD factor: EMA of low-rank covariances plus a decayed
    identity (many tiny, clustered eigenvalues)."""
    rng = np.random.default_rng(seed)
    A = 0.95 ** 20 * np.eye(n)
    for _ in range(4):
        X = rng.standard_normal((rank, n)) * np.exp(rng.standard_normal(n))
        A += 0.05 * X.T @ X / rank
    return A


def check(n, leaf=LEAF, seed=0, kind='kfac'):
    from scipy.linalg import eigh_tridiagonal, hessenberg
    if kind == 'kfac':
        A = kfac_like(n, max(8, n // 3), seed)
        H = hessenberg(A)
        d = np.diag(H).astype(np.float32).astype(np.float64)
        e = np.diag(H, 1).astype(np.float32).astype(np.float64)
    else:
        rng = np.random.default_rng(seed)
        d = rng.standard_normal(n).astype(np.float32).astype(np.float64)
        e = rng.standard_normal(n - 1).astype(np.float32).astype(np.float64)
        if kind == 'glued':     # repeated blocks -> heavy deflation
            d[:] = np.tile(d[:7], n // 7 + 1)[:n]
            e[:] = 1e-3
    stats = []
    lam, Z = dc_eigh(d, np.append(e, 0.0), leaf, stats)
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    Zd = Z.astype(np.float64)
    tn = np.linalg.norm(T, 2)
    resid = np.linalg.norm(T @ Zd.T - Zd.T * lam) / (tn * np.sqrt(n))
    orth = np.abs(Zd @ Zd.T - np.eye(n)).max()
    ref = eigh_tridiagonal(d, e, eigvals_only=True)
    lam_err = np.abs(lam - ref).max() / tn
    return resid, orth, lam_err, stats


if __name__ == '__main__':
    import sys
    for n in [int(a) for a in sys.argv[1:]] or [5, 64, 65, 130, 300, 577]:
        for kind in ('kfac', 'rand', 'glued'):
            r, o, l, st = check(n, kind=kind)
            print('n=%5d %-6s resid %.2e orth %.2e lam %.2e  merges(m,k,rot) %s' % (
                n, kind, r, o, l, st[-3:]))
