"""Two-stage symmetric eigensolver glue (reference:
kfac/layers/utils.py:45-74, torch.symeig per factor).

    dense A --sy2sb (csrc/eig_sy2sb.hip)--> band (half-bandwidth 16) + Q1
            --sb2st (csrc/eig_sb2st.hip)--> tridiagonal d, e + Q2 reflectors
            --divide and conquer (csrc/eig_dc.hip)--> Z
    eigenvectors = Q1 Q2 Z (csrc/eig_q2.hip, then the compact-WY
    back-transformation of csrc/eig_library.hip with the band offset).

The one-stage reduction (csrc/eig_reduce.hip) streams the whole trailing
matrix through a mat-vec for every column (~(2/3) n^3 bytes per factor);
stage 1 here reads it once per 16 columns through MFMA-friendly panel
updates and stage 2 works on a band that fits in LDS.
"""
import torch

from . import _lib

__all__ = ['BW', 'sb2st', 'pack_band']

BW = 16
ND = 2 * BW


def pack_band(A, b=BW):
    """Lower band of a dense symmetric matrix as the stage-2 input layout:
    (n, 2 BW) column-major band, band[c, d] = A[c + d, c] for d <= b."""
    n = A.shape[0]
    out = torch.zeros(n, ND, dtype=torch.float32, device=A.device)
    for d in range(b + 1):
        out[:n - d, d] = torch.diagonal(A, -d).to(torch.float32)
    return out


def sb2st(bands):
    """Band -> tridiagonal for a list of (n_i, 2 BW) float32 band tensors
    (modified in place).  Returns [(d, e, V2)] per matrix: V2 row s holds
    sweep s's reflectors (step j at [16 j, 16 j + 16): tau, v[1:])."""
    L = _lib.lib()
    assert int(L.kfac_sb2st_bw()) == BW
    dev = bands[0].device
    recs = (_lib.SbRecord * len(bands))()
    outs = []
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    for i, band in enumerate(bands):
        n = band.shape[0]
        assert band.dtype == torch.float32 and band.is_contiguous() and band.shape[1] == ND
        ldv2 = int(L.kfac_sb2st_ldv2(n))
        v2 = torch.zeros(n, ldv2, dtype=torch.float32, device=dev)
        d = torch.empty(n, dtype=torch.float32, device=dev)
        e = torch.empty(n, dtype=torch.float32, device=dev)
        prog = torch.empty(int(L.kfac_sb2st_nwg(n)) + 1, dtype=torch.int32, device=dev)
        r = recs[i]
        r.band, r.v2, r.d, r.e, r.prog = (band.data_ptr(), v2.data_ptr(), d.data_ptr(),
                                          e.data_ptr(), prog.data_ptr())
        r.n, r.ldv2 = n, ldv2
        outs.append((d, e, v2, prog))
    _lib.check(L.kfac_sb2st_batched(recs, len(bands), err.data_ptr(), _lib.stream(dev)),
               'kfac_sb2st_batched')
    if int(err.item()) != 0:
        raise RuntimeError('kfac_sb2st_batched: a pipeline wait timed out (err=%d)' % int(err.item()))
    return [(d, e[:-1], v2) for d, e, v2, _ in outs]


_BUFS = {}


def _extra_buffers(dev, n, b, slot):
    key = (str(dev), n, b, slot)
    X = _BUFS.get(key)
    if X is None:
        L = _lib.lib()
        f32 = dict(dtype=torch.float32, device=dev)
        ldv2 = int(L.kfac_sb2st_ldv2(n))
        X = dict(ldv2=ldv2, band=torch.zeros(b, n, ND, **f32),
                 v2=torch.zeros(b, n, ldv2, **f32),
                 prog=torch.zeros(b, int(L.kfac_sb2st_nwg(n)) + 1, dtype=torch.int32, device=dev),
                 s1ws=torch.zeros(b, int(L.kfac_sy2sb_ws_floats(n)) + 64, **f32),
                 tq2=torch.zeros(b, int(L.kfac_q2_t_floats(n)), **f32),
                 zc=torch.zeros(b, n, (n + 63) // 64 * 64, **f32),
                 err=torch.zeros(1, dtype=torch.int32, device=dev))
        _BUFS[key] = X
    return X


def two_stage_group(mats, clip, stream, use_graph=True, slot=0):
    """Eigen-decompose a ragged batch of symmetric fp32 matrices on `stream`
    through the two-stage path; [(Q, D)] like ops.eigen._fused_group."""
    from . import eigen
    L = _lib.lib()
    dev = mats[0].device
    classes = {}
    for i, A in enumerate(mats):
        classes.setdefault(A.shape[0], []).append(i)
    order = sorted(classes.items(), key=lambda kv: -kv[0])
    total = len(mats)
    outs = [None] * total
    with torch.cuda.stream(stream):
        cs = _lib.c_vp(stream.cuda_stream)
        s1 = (_lib.S1Record * total)()
        sb = (_lib.SbRecord * total)()
        dc = (_lib.DcRecord * total)()
        q2 = (_lib.Q2Record * total)()
        bufs = []
        k = 0
        err = None
        for n, idx in order:
            b = len(idx)
            B = eigen._tri_buffers(dev, n, b, slot)
            X = _extra_buffers(dev, n, b, slot)
            err = X['err'] if err is None else err
            bufs.append((n, idx, B, X))
            lda = B['lda']
            for i, m in enumerate(idx):
                B['A'][i, :n, :n].copy_(mats[m])
            dcr = eigen._dc_records(B, n, b)
            for i in range(b):
                r = s1[k]
                r.A, r.lda, r.tau = B['A'][i].data_ptr(), lda, B['tau'][i].data_ptr()
                r.ws = (X['s1ws'][i].data_ptr() + 255) // 256 * 256
                r.band, r.n = X['band'][i].data_ptr(), n
                r = sb[k]
                r.band, r.v2 = X['band'][i].data_ptr(), X['v2'][i].data_ptr()
                r.d, r.e, r.prog = B['d'][i].data_ptr(), B['e'][i].data_ptr(), X['prog'][i].data_ptr()
                r.n, r.ldv2 = n, X['ldv2']
                dc[k] = dcr[i]
                r = q2[k]
                r.v2, r.ldv2 = X['v2'][i].data_ptr(), X['ldv2']
                r.Z, r.ldz, r.T, r.n = X['zc'][i].data_ptr(), lda, X['tq2'][i].data_ptr(), n
                k += 1
        err.zero_()
        _lib.check(L.kfac_sy2sb_batched(s1, total, int(use_graph), cs), 'kfac_sy2sb_batched')
        _lib.check(L.kfac_sb2st_batched(sb, total, err.data_ptr(), cs), 'kfac_sb2st_batched')
        _lib.check(L.kfac_dc_batched(dc, total, int(use_graph), cs), 'kfac_dc_batched')
        for n, idx, B, X in bufs:     # eigenvector rows -> component rows (coalesced Q2)
            X['zc'][:, :, :n].copy_(B['Z'][:, :, :n].transpose(1, 2))
        _lib.check(L.kfac_q2_batched(q2, total, int(use_graph), cs), 'kfac_q2_batched')
        for n, idx, B, X in bufs:
            B['Z'][:, :, :n].copy_(X['zc'][:, :, :n].transpose(1, 2))
        for n, idx, B, X in bufs:
            b = len(idx)
            _lib.check(L.kfac_backtransform_shift(*eigen._bt_args(B, n, b), BW, int(use_graph), cs),
                       'kfac_backtransform_shift')
            eigen._INFOS.append(eigen._dc_info(B, n, b))
            Q = B['Z'][:, :, :n].transpose(1, 2).contiguous()
            D = B['w'].clone()
            if clip is not None:
                D.clamp_(min=clip)
            for i, m in enumerate(idx):
                outs[m] = (Q[i], D[i])
        eigen._INFOS.append(err.clone())
    return outs
