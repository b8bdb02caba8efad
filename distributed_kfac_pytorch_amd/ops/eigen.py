"""Symmetric eigendecomposition / damped inverse of Kronecker factors (K6, K9).

GPU path (MI355X), hand-written end to end (no vendor solver is linked):
every factor of the step (any size from 2 up to FUSED_MAX_N) goes through
ONE ragged launch sequence per stage -- the fused tridiagonal reduction
(csrc/eig_reduce.hip), the batched divide and conquer (csrc/eig_dc.hip) and
the compact-WY back-transformation (csrc/eig_backtransform.hip) -- split
over two streams by size (_fused_groups).  1x1 factors, and the opt-in
solver='jacobi' for n <= SMALL_N, use the batched LDS Jacobi kernel
(csrc/eig_jacobi.hip).  Factors above FUSED_MAX_N (a 16384^2 fp32 factor is
1 GiB; e.g. the 33k-vocabulary decoder of the wikitext-2 language model) fall
back to torch.linalg.eigh on the device, with a one-time warning.
CPU path: torch.linalg.eigh (the reference semantics, kfac/layers/utils.py:45-74).

Results: ascending eigenvalues clipped at `clip` (reference default 0.0),
Q row-major contiguous with eigenvector k in column k.
"""
import os

import torch

from . import _lib

__all__ = ['symeig_many', 'inverse_many', 'SMALL_N']

SMALL_N = 192
FUSED_MAX_N = 16384   # csrc/eig_reduce.hip NMAX
BT = 256   # back-transformation block (csrc/eig_backtransform.hip kfac_backtransform_block)
_streams = {}
# debug / probes: a list -> _fused_group appends (group slot, stage, event)
# after each stage it enqueues (scripts/probes/probe_eig_stream_ends.py).
# KFAC_EIG_STAGE_LOG=1: every native symeig_many call records them, and the
# next check_solver_status() prints the stage times to stderr.
STAGE_EVENTS = None
STAGE_LOG = os.environ.get('KFAC_EIG_STAGE_LOG') == '1'


def _mark(slot, stage, stream):
    if STAGE_EVENTS is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        STAGE_EVENTS.append((slot, stage, e))


def _side_streams(device, k):
    pool = _streams.setdefault(str(device), [])
    while len(pool) < k:     # grow only: a stream in the pool may still run work
        pool.append(torch.cuda.Stream(device=device))
    return pool[:k]


def side_streams(device):
    """Every worker stream the eigensolver has used on `device` (a caller
    that needs the device quiet joins these instead of a full device sync)."""
    return list(_streams.get(str(device), []))


def _jacobi_small(mats, clip, max_sweeps=30, tol=1e-7):
    dev = mats[0].device
    outs = []
    recs = (_lib.EigRecord * len(mats))()
    scratch = []
    for i, A in enumerate(mats):
        n = A.shape[0]
        A = A.contiguous()
        Q = torch.empty(n, n, dtype=torch.float32, device=dev)
        d = torch.empty(n, dtype=torch.float32, device=dev)
        Vt = torch.empty(n, n, dtype=torch.float32, device=dev)
        scratch.append((A, Vt))
        recs[i].A = A.data_ptr(); recs[i].Q = Q.data_ptr(); recs[i].d = d.data_ptr()
        recs[i].Vt = Vt.data_ptr(); recs[i].n = n
        outs.append((Q, d))
    _lib.check(_lib.lib().kfac_eig_jacobi_small(recs, len(mats), max_sweeps, tol,
                                                 int(clip is not None),
                                                 float(clip if clip is not None else 0.0),
                                                 _lib.stream(dev)), 'kfac_eig_jacobi_small')
    # keep inputs / scratch alive until the kernel has consumed them
    cur = torch.cuda.current_stream(dev)
    for A, Vt in scratch:
        A.record_stream(cur)
        Vt.record_stream(cur)
    return outs


_INFOS = []
_TRI_BUFS = {}


def _tri_buffers(dev, n, b, slot=0):
    """Persistent per-(device, n, batch, slot) buffers of the hand-written
    path: the captured reduction graph addresses them, so they live (and are
    reused) for the whole run.  Concurrent jobs of one (n, b) use distinct
    slots."""
    key = (str(dev), n, b, slot)
    bufs = _TRI_BUFS.get(key)
    if bufs is None:
        L = _lib.lib()
        if int(L.kfac_backtransform_block()) != BT:
            raise RuntimeError('back-transformation block: library {} vs eigen.BT {}'.format(
                int(L.kfac_backtransform_block()), BT))
        # A: lda x lda per matrix, lda = n rounded up to the reduction's 128-row
        # tiles, zero past n (its symv tiles read whole tiles unmasked; the
        # MFMA GEMMs of the back-transformation step k by 64)
        lda = (n + 127) // 128 * 128
        f32 = dict(dtype=torch.float32, device=dev)
        nblk = (n + BT - 1) // BT
        wsb = int(L.kfac_dc_ws_bytes(n))
        rwsf = int(L.kfac_reduce_ws_floats(n))
        bufs = dict(lda=lda, sA=lda * lda, A=torch.zeros(b, lda, lda, **f32), Z=torch.zeros(b, n, lda, **f32),
                    d=torch.zeros(b, n, **f32), e=torch.zeros(b, n, **f32),
                    w=torch.zeros(b, n, **f32), wsb=wsb,
                    dcws=torch.zeros(b * wsb, dtype=torch.uint8, device=dev),
                    rwsf=rwsf, rws=torch.zeros(b * rwsf, **f32),
                    tau=torch.zeros(b, n, **f32),
                    info=torch.zeros(b, dtype=torch.int32, device=dev),
                    T=torch.zeros(2 * b * nblk * BT * BT, **f32),
                    W1=torch.zeros(b * int(L.kfac_backtransform_slabs(lda)) * BT * n, **f32),
                    W2=torch.zeros(b * BT * n, **f32),
                    Vt=torch.zeros(b * BT * lda, **f32))
        _TRI_BUFS[key] = bufs
    return bufs


def _dc_records(B, n, b):
    recs = (_lib.DcRecord * b)()
    lda, wsb = B['lda'], B['wsb']
    for i in range(b):
        r = recs[i]
        r.d = B['d'][i].data_ptr()
        r.e = B['e'][i].data_ptr()
        r.dout = B['w'][i].data_ptr()
        r.Zout = B['Z'][i].data_ptr()
        r.ldz = lda
        r.ws = B['dcws'].data_ptr() + i * wsb
        r.n = n
    return recs


def _dc_info(B, n, b):
    """Per matrix: secular roots of the divide and conquer that hit the
    iteration cap (device int in the workspace), as a (b,) int32 tensor."""
    off = int(_lib.lib().kfac_dc_info_offset(n))
    return B['dcws'].view(b, B['wsb'])[:, off:off + 4].contiguous().view(torch.int32).reshape(b)


def tridiag_eigh(ds, es, use_graph=False):
    """Eigen-decompose symmetric tridiagonal matrices (fp32 CUDA vectors d of
    length n, e of length >= n-1) with ONE batched divide-and-conquer launch
    sequence (csrc/eig_dc.hip; sizes may differ) -> [(w ascending, Z rows =
    eigenvectors)]."""
    L = _lib.lib()
    dev = ds[0].device
    recs = (_lib.DcRecord * len(ds))()
    keep, outs = [], []
    for i, (d, e) in enumerate(zip(ds, es)):
        n = d.shape[0]
        lda = (n + 63) // 64 * 64
        dd = d.contiguous().float()
        ee = torch.zeros(n, dtype=torch.float32, device=dev)
        ee[:n - 1] = e[:n - 1]
        w = torch.empty(n, dtype=torch.float32, device=dev)
        Z = torch.empty(n, lda, dtype=torch.float32, device=dev)
        ws = torch.empty(int(L.kfac_dc_ws_bytes(n)), dtype=torch.uint8, device=dev)
        r = recs[i]
        r.d, r.e, r.dout, r.Zout = dd.data_ptr(), ee.data_ptr(), w.data_ptr(), Z.data_ptr()
        r.ldz, r.ws, r.n = lda, ws.data_ptr(), n
        keep += [dd, ee, ws]
        outs.append((w, Z, ws, n))
    _lib.check(L.kfac_dc_batched(recs, len(ds), int(use_graph), _lib.stream(dev)),
               'kfac_dc_batched')
    infos = [ws[int(L.kfac_dc_info_offset(n)):][:4].view(torch.int32) for _, _, ws, n in outs]
    res = [(w, Z[:, :n]) for w, Z, _, n in outs]
    torch.cuda.current_stream(dev).synchronize()
    del keep
    bad = [int(i.item()) for i in infos]
    if any(bad):
        raise RuntimeError('divide and conquer: secular roots not converged {}'.format(bad))
    return res


def _bt_args(B, n, b):
    lda = B['lda']
    return (_lib.ptr(B['A']), lda, B['sA'], _lib.ptr(B['tau']), _lib.ptr(B['Z']), lda, n * lda,
            n, b, _lib.ptr(B['T']), _lib.ptr(B['W1']), _lib.ptr(B['W2']), _lib.ptr(B['Vt']))


def _fused_groups(mats):
    """Split the batch over concurrent streams.  The reduction is a chain of
    n columns per matrix, latency bound with few workgroups: the largest
    factors (n above half the largest n) stay ONE batched chain (separate
    chains per big factor were slower, 213 vs 160 ms on ResNet-50: every
    extra concurrent launch chain lengthens each chain's per-launch latency),
    and the smaller factors' whole solve (reduction, divide and conquer,
    back-transformation) runs on FUSED_STREAMS - 1 more streams under the big
    chain, split again at half the next size.  One group when splitting is
    off or pointless."""
    idx = list(range(len(mats)))
    if not FUSED_SPLIT:
        return [idx]
    groups = []
    while idx and len(groups) < FUSED_STREAMS - 1:
        nmax = max(mats[i].shape[0] for i in idx)
        groups.append([i for i in idx if 2 * mats[i].shape[0] > nmax])
        idx = [i for i in idx if 2 * mats[i].shape[0] <= nmax]
    if idx:
        groups.append(idx)
    return groups


FUSED_STREAMS = int(os.environ.get('KFAC_EIG_FUSED_STREAMS', '2'))
# tail threshold (csrc/eig_reduce.hip KFAC_REDUCE_TAIL, 768) of the groups after
# the leading one (-1 = the same): their single-launch tail columns redo F's row
# work over every tile, traffic that slows the leading chain beside them.
# ResNet-50's 108 factors, same box (profiles/r6_reduce_tail_rest_sweep.log):
# 768 103.7-103.8 ms; 256 / 384 / 512 102.2-102.7; 0 104.9; 1536 110.2; 2304 122
TAIL_REST = int(os.environ.get('KFAC_REDUCE_TAIL_REST', '384'))
FUSED_SPLIT = bool(int(os.environ.get('KFAC_EIG_FUSED_SPLIT', '1')))


def leading_group(sizes):
    """Indices of the group _fused_groups puts on the caller's stream first
    (the critical chain: every n above half the largest), or None when the
    solve is not split over streams."""
    if not sizes or not FUSED_SPLIT or FUSED_STREAMS < 2:
        return None
    nmax = max(sizes)
    return [i for i, n in enumerate(sizes) if 2 * n > nmax]


def early_stream(device):
    """The worker stream of symeig_group (the first of the side-stream pool:
    the stream _large_fused's second group uses, so the early chain and the
    caller's stream sit on two hardware queues as in a split solve)."""
    return _side_streams(device, 1)[0]


def symeig_group(mats, clip, stream, finite=None):
    """Enqueue the fused solve of `mats` as ONE group on `stream` (staging,
    reduction, divide and conquer, back-transformation; slot 0 buffers, as the
    leading group of a split solve) and return [(Q, d)] without joining:
    the caller orders its stream after `stream` before reading them.  KFAC's
    early inverse update runs the leading group this way while the rest of
    the step's factors are still being computed."""
    if not mats:
        return []
    if any(A.shape[0] <= 1 or A.shape[0] > FUSED_MAX_N for A in mats):
        raise ValueError('symeig_group: sizes 2 .. {} only'.format(FUSED_MAX_N))
    _lib.check_pgemm_extent(max(A.shape[0] for A in mats))
    outs = _fused_group(mats, clip, stream, True, 0, finite)
    for A in mats:
        A.record_stream(stream)
    del _INFOS[:-256]
    return outs


def _large_fused(mats, clip, stream, use_graph=True, finite=None, split=True):
    """Every factor of the inverse update in ragged launch sequences: per
    group (_fused_groups) the fused one-launch-per-column reduction over all
    its matrices (csrc/eig_reduce.hip), the batched divide and conquer over
    all its matrices (csrc/eig_dc.hip), then the compact-WY back-
    transformation per size class (csrc/eig_backtransform.hip); every further group
    on a side stream.  No library solver, no host round trip; each stage is
    a cached hipGraph.

    Measured and dropped (profiles/r2_eig_streams.log, r4_eig_groups.log):
    enqueueing the side groups from worker threads (157 vs 156 ms) and the
    largest factors' chain on a high-priority stream (162 vs 157 ms; 277 ms
    in round 4)."""
    dev = mats[0].device
    groups = _fused_groups(mats) if split else [list(range(len(mats)))]
    outs = [None] * len(mats)
    caller = stream
    streams = [stream] + _side_streams(dev, len(groups) - 1)
    for s in streams[1:]:
        s.wait_stream(caller)
    for slot, (g, st) in enumerate(zip(groups, streams)):
        fl = None if finite is None else [finite[i] for i in g]
        for i, r in zip(g, _fused_group([mats[i] for i in g], clip, st, use_graph, slot, fl)):
            outs[i] = r
    del _INFOS[:-256]
    for g, st in zip(groups[1:], streams[1:]):
        caller.wait_stream(st)
        for i in g:
            mats[i].record_stream(st)
            outs[i][0].record_stream(caller)
            outs[i][1].record_stream(caller)
    return outs


def _fused_group(mats, clip, stream, use_graph, slot=0, finite=None):
    dev = mats[0].device
    L = _lib.lib()
    classes = {}
    for i, A in enumerate(mats):
        classes.setdefault(A.shape[0], []).append(i)
    order = sorted(classes.items(), key=lambda kv: -kv[0])
    total = len(mats)
    outs = [None] * total
    with torch.cuda.stream(stream):
        cs = _lib.c_vp(stream.cuda_stream)
        rr = (_lib.ReduceRecord * total)()
        dr = (_lib.DcRecord * total)()
        k = 0
        bufs = []
        for n, idx in order:
            b = len(idx)
            B = _tri_buffers(dev, n, b, slot)     # per group: concurrent groups never share
            bufs.append((n, idx, B))
            for i, m in enumerate(idx):
                if finite is None:
                    B['A'][i, :n, :n].copy_(mats[m])
                else:
                    sanitize(mats[m], finite[m], out=B['A'][i, :n, :n])
            dcr = _dc_records(B, n, b)
            for i in range(b):
                r = rr[k]
                r.A = B['A'][i].data_ptr()
                r.lda = B['lda']
                r.d = B['d'][i].data_ptr()
                r.e = B['e'][i].data_ptr()
                r.tau = B['tau'][i].data_ptr()
                r.ws = B['rws'].data_ptr() + 4 * i * B['rwsf']
                r.n = n
                dr[k] = dcr[i]
                k += 1
        _mark(slot, 'staged', stream)
        prev = L.kfac_reduce_set_tail(TAIL_REST) if slot > 0 and TAIL_REST >= 0 else None
        try:
            _lib.check(L.kfac_reduce_batched(rr, total, int(use_graph), cs),
                       'kfac_reduce_batched')
        finally:
            if prev is not None:
                L.kfac_reduce_set_tail(prev)
        _mark(slot, 'reduce', stream)
        _lib.check(L.kfac_dc_batched(dr, total, int(use_graph), cs), 'kfac_dc_batched')
        _mark(slot, 'dc', stream)
        for n, idx, B in bufs:
            b = len(idx)
            _lib.check(L.kfac_tridiag_backtransform(*_bt_args(B, n, b), int(use_graph), cs),
                       'kfac_tridiag_backtransform')
            _mark(slot, 'bt%d' % n, stream)
            _INFOS.append(_dc_info(B, n, b))
            Q = B['Z'][:, :, :n].transpose(1, 2).contiguous()
            D = B['w'].clone()
            if clip is not None:
                D.clamp_(min=clip)
            for i, m in enumerate(idx):
                outs[m] = (Q[i], D[i])
    return outs


# Two-stage path (csrc/eig_sy2sb.hip -> eig_sb2st.hip -> eig_dc.hip ->
# eig_q2.hip -> eig_backtransform.hip with shift 16): dense -> band in 16-wide
# panels (16x fewer passes over the trailing matrix than the one-stage
# column chain), bulge chasing with every hand-off inside one CU, then the
# two back-transformations.  Factors with TWO_STAGE_MIN <= n <= TWO_STAGE_MAX
# take it when KFAC_EIG_TWO_STAGE=1; the rest stay on the one-stage path, on
# the other streams.
TWO_STAGE = bool(int(os.environ.get('KFAC_EIG_TWO_STAGE', '0')))
TWO_STAGE_MIN = int(os.environ.get('KFAC_EIG_TWO_STAGE_MIN', '1024'))
# largest size csrc/eig_sy2sb.hip (NMAX2) and csrc/eig_q2.hip (16 x QT) take;
# KFAC_EIG_TWO_STAGE_MAX lowers the eligible range (e.g. a middle size class)
TWO_STAGE_MAX = min(5120, int(os.environ.get('KFAC_EIG_TWO_STAGE_MAX', '5120')))
# at most this many eligible factors (largest first) take the two-stage path
# (0 = all): the two paths run concurrently on two streams, so moving only
# part of the largest size class shortens the one-stage critical path
TWO_STAGE_COUNT = int(os.environ.get('KFAC_EIG_TWO_STAGE_COUNT', '0'))
SB2 = 16                 # band half-bandwidth
_TS_BUFS = {}


def _ts_buffers(dev, n, b, slot=0):
    key = (str(dev), n, b, slot)
    bufs = _TS_BUFS.get(key)
    if bufs is None:
        L = _lib.lib()
        lda = (n + 127) // 128 * 128
        ldv2 = (n + 15) // 16 * 16 + 16
        f32 = dict(dtype=torch.float32, device=dev)
        nblk = (n + BT - 1) // BT
        wsb = int(L.kfac_dc_ws_bytes(n))
        # stage 1's Y launch reads whole 16-row blocks of A22, up to 15 rows
        # past n (n == lda for 4608): 16 spare zero rows after the last matrix
        a_full = torch.zeros(b * lda * lda + 16 * lda, **f32)
        bufs = dict(lda=lda, ldv2=ldv2, sA=lda * lda,
                    A=a_full[:b * lda * lda].view(b, lda, lda), A_full=a_full,
                    tau=torch.zeros(b, n, **f32),  # larft: stride n
                    band=torch.zeros(b, (n + 2 * SB2) * 2 * SB2, **f32),
                    syws=torch.zeros(b, int(L.kfac_sy2sb_ws_floats(lda)), **f32),
                    v2=torch.zeros(b, max(n - 1, 1), ldv2, **f32),
                    d=torch.zeros(b, n, **f32), e=torch.zeros(b, n, **f32),
                    w=torch.zeros(b, n, **f32), Z=torch.zeros(b, n, lda, **f32),
                    sbstat=torch.zeros(b, dtype=torch.int32, device=dev),
                    wsb=wsb, dcws=torch.zeros(b * wsb, dtype=torch.uint8, device=dev),
                    T=torch.zeros(2 * b * nblk * BT * BT, **f32),
                    W1=torch.zeros(b * int(L.kfac_backtransform_slabs(lda)) * BT * n, **f32),
                    W2=torch.zeros(b * BT * n, **f32),
                    Vt=torch.zeros(b * BT * lda, **f32))
        _TS_BUFS[key] = bufs
    return bufs


def _two_stage_group(mats, clip, stream, use_graph=True, slot=0):
    """Every matrix of `mats` (TWO_STAGE_MIN..TWO_STAGE_MAX) through the
    two-stage solver on `stream`: one batched launch sequence per stage."""
    dev = mats[0].device
    L = _lib.lib()
    if not _lib.has('kfac_sy2sb_batched'):
        raise RuntimeError('the two-stage eigensolver is not in this build: rebuild with '
                           'KFAC_BUILD_TWO_STAGE=1 python csrc/build.py')
    classes = {}
    for i, A in enumerate(mats):
        classes.setdefault(A.shape[0], []).append(i)
    order = sorted(classes.items(), key=lambda kv: -kv[0])
    total = len(mats)
    outs = [None] * total
    with torch.cuda.stream(stream):
        cs = _lib.c_vp(stream.cuda_stream)
        r1 = (_lib.Sy2sbRecord * total)()
        r2 = (_lib.Sb2stRecord * total)()
        r3 = (_lib.DcRecord * total)()
        r4 = (_lib.Q2Record * total)()
        k = 0
        bufs = []
        for n, idx in order:
            b = len(idx)
            B = _ts_buffers(dev, n, b, slot)
            bufs.append((n, idx, B))
            dcr = _dc_records(B, n, b)
            for i, m in enumerate(idx):
                B['A'][i, :n, :n].copy_(mats[m])
                r = r1[k]
                r.A, r.lda, r.tau = B['A'][i].data_ptr(), B['lda'], B['tau'][i].data_ptr()
                r.band, r.ws, r.n = B['band'][i].data_ptr(), B['syws'][i].data_ptr(), n
                q = r2[k]
                q.band_in = q.band = B['band'][i].data_ptr()
                q.v2, q.d, q.e = B['v2'][i].data_ptr(), B['d'][i].data_ptr(), B['e'][i].data_ptr()
                q.ldv2, q.n = B['ldv2'], n
                q.status = B['sbstat'][i].data_ptr()    # timed-out bulge-chasing waits
                r3[k] = dcr[i]
                z = r4[k]
                z.Z, z.v2, z.ldz, z.ldv2, z.n = (B['Z'][i].data_ptr(), B['v2'][i].data_ptr(),
                                                 B['lda'], B['ldv2'], n)
                k += 1
        _lib.check(L.kfac_sy2sb_batched(r1, total, int(use_graph), cs), 'kfac_sy2sb_batched')
        _lib.check(L.kfac_sb2st_batched(r2, total, int(use_graph), cs), 'kfac_sb2st_batched')
        # a bounded wait that timed out leaves garbage d / e / v2: the count
        # joins the solver status that check_solver_status() raises on
        for _, _, B in bufs:
            _INFOS.append(B['sbstat'].clone())
        _lib.check(L.kfac_dc_batched(r3, total, int(use_graph), cs), 'kfac_dc_batched')
        _lib.check(L.kfac_q2_batched(r4, total, int(use_graph), cs), 'kfac_q2_batched')
        for n, idx, B in bufs:
            b = len(idx)
            lda = B['lda']
            _lib.check(L.kfac_band_backtransform(
                _lib.ptr(B['A']), lda, B['sA'], _lib.ptr(B['tau']), _lib.ptr(B['Z']), lda,
                n * lda, n, b, _lib.ptr(B['T']), _lib.ptr(B['W1']), _lib.ptr(B['W2']),
                _lib.ptr(B['Vt']), SB2, int(use_graph), cs), 'kfac_band_backtransform')
            _INFOS.append(_dc_info(B, n, b))
            Q = B['Z'][:, :, :n].transpose(1, 2).contiguous()
            D = B['w'].clone()
            if clip is not None:
                D.clamp_(min=clip)
            for i, m in enumerate(idx):
                outs[m] = (Q[i], D[i])
    return outs


def two_stage_eigh(mats, clip=0.0, use_graph=True):
    """The two-stage solver on the current stream (tests, probes)."""
    cur = torch.cuda.current_stream(mats[0].device)
    return _two_stage_group([A.float().contiguous() for A in mats], clip, cur, use_graph)


def check_solver_status():
    """Host-side check of every divide-and-conquer call issued since the last
    check (info != 0 -> the solver did not converge) and of every bulge-chasing
    launch of the two-stage path (nonzero = bounded waits that timed out, the
    band reduction's output is garbage).  Syncs; call once per inverse step,
    not in the hot path."""
    global _INFOS, STAGE_EVENTS
    if STAGE_LOG and STAGE_EVENTS:
        evs, STAGE_EVENTS = STAGE_EVENTS, None
        evs[-1][2].synchronize()
        t0 = evs[0][2]
        import sys
        print('[kfac-eig] ' + ', '.join('%s%s %.2f' % ('' if slot < 0 else 'g%d ' % slot, stage,
                                                         t0.elapsed_time(e))
                                        for slot, stage, e in evs[1:]), file=sys.stderr)
    infos, _INFOS = _INFOS, []
    if not infos:
        return
    flat = torch.cat([i.reshape(-1).to(torch.int64) for i in infos])
    if not bool((flat != 0).any()):      # one host read for every call
        return
    bad = [int(i.abs().max().item()) for i in infos if (i != 0).any().item()]
    if bad:
        raise RuntimeError('symmetric eigensolver failed to converge (info={})'.format(bad))


_EYES = {}


def _eye(n, device):
    key = (n, str(device))
    e = _EYES.get(key)
    if e is None:
        e = _EYES[key] = torch.eye(n, dtype=torch.float32, device=device)
    return e


def sanitize(A, ok, out=None):
    """A where the device flag `ok` holds, else the identity (a non-finite
    factor must not reach the solvers' data-dependent loops, which are not
    NaN-safe) -- no host read; the caller raises on `ok` later."""
    return torch.where(ok, A, _eye(A.shape[0], A.device), out=out)


def symeig_many(mats, clip=0.0, solver='auto', finite=None, split=True):
    """Eigendecompose a list of symmetric fp32 matrices -> list of (Q, d).

    finite: None, or a device bool tensor (one flag per matrix): a matrix
    whose flag is False is decomposed as the identity instead (see
    sanitize); the caller checks the flags after enqueueing its work.
    split=False: the fused path runs every factor as one group on the
    caller's stream (the leading group already runs elsewhere: symeig_group)."""
    global STAGE_EVENTS
    if len(mats) == 0:
        return []
    if finite is not None and not _lib.use_native(mats[0]):
        mats = [sanitize(A, finite[i]) for i, A in enumerate(mats)]
        finite = None
    if not _lib.use_native(mats[0]):
        outs = []
        for A in mats:
            d, Q = torch.linalg.eigh(A)
            Q = Q.contiguous()
            if clip is not None:
                d = torch.clamp(d, min=clip)
            outs.append((Q, d))
        return outs
    if solver not in ('auto', 'jacobi'):
        raise ValueError("solver must be 'auto' or 'jacobi', got {!r}".format(solver))
    if finite is not None:
        # paths other than the fused one-stage group take sanitised copies
        def _clean(idx):
            for i in idx:
                mats[i] = sanitize(mats[i], finite[i])
        mats = list(mats)
    huge = [i for i, A in enumerate(mats) if A.shape[0] > FUSED_MAX_N]
    if huge:
        if finite is not None:
            _clean(range(len(mats)))
        return _with_huge(mats, huge, clip, solver)
    nmax = max(A.shape[0] for A in mats)
    _lib.check_pgemm_extent(nmax)
    # EVERY factor rides the fused ragged launch sequence (a small factor's
    # reduction columns run alongside the big ones', its divide and conquer is
    # one or two levels); the batched LDS Jacobi takes 1x1 factors, and every
    # n <= SMALL_N with solver='jacobi' (its latency is the slowest matrix's:
    # ~40 ms for ResNet-50's 64..192 factors, profiles/r2_eig_kernel_stats.txt)
    lim = SMALL_N if solver == 'jacobi' else 1
    small = [i for i, A in enumerate(mats) if A.shape[0] <= lim]
    large = [i for i, A in enumerate(mats) if A.shape[0] > lim]
    if finite is not None:
        _clean(small)
    outs = [None] * len(mats)
    if small:
        for i, r in zip(small, _jacobi_small([mats[i] for i in small], clip)):
            outs[i] = r
    ts = []
    if TWO_STAGE:
        ts = [i for i in large if TWO_STAGE_MIN <= mats[i].shape[0] <= TWO_STAGE_MAX]
        if TWO_STAGE_COUNT > 0:
            ts = sorted(ts, key=lambda i: -mats[i].shape[0])[:TWO_STAGE_COUNT]
        large = [i for i in large if i not in set(ts)]
        if finite is not None:
            _clean(ts)
    cur = torch.cuda.current_stream(mats[0].device)
    if STAGE_LOG and not STAGE_EVENTS:
        STAGE_EVENTS = []
        _mark(-1, 'start', cur)
    _mark(-1, 'symeig', cur)
    side = None
    if ts:
        # the two-stage group on its own stream, under the one-stage chains
        side = _side_streams(mats[0].device, FUSED_STREAMS + 1)[-1]
        side.wait_stream(cur)
        sub = [mats[i] for i in ts]
        res = _two_stage_group(sub, clip, side)
        for A in sub:
            A.record_stream(side)
        for i, r in zip(ts, res):
            outs[i] = r
    if large:
        sub = [mats[i] for i in large]
        res = _large_fused(sub, clip, cur,
                           finite=None if finite is None else [finite[i] for i in large],
                           split=split)
        for A in sub:
            A.record_stream(cur)
        for i, r in zip(large, res):
            outs[i] = r
    if side is not None:
        cur.wait_stream(side)
        for i in ts:
            outs[i][0].record_stream(cur)
            outs[i][1].record_stream(cur)
    _mark(-1, 'end', cur)
    return outs


_HUGE_WARNED = []


def _with_huge(mats, huge, clip, solver):
    """Factors above FUSED_MAX_N: torch.linalg.eigh on the device (the
    reference's solver, kfac/layers/utils.py:45-74); the rest as usual."""
    if not _HUGE_WARNED:
        _HUGE_WARNED.append(1)
        import warnings
        warnings.warn('K-FAC: factor(s) of size {} exceed the native eigensolver limit {} '
                      '(csrc/eig_reduce.hip NMAX); using torch.linalg.eigh for them (slow: '
                      'consider skip_layers for that layer)'.format(
                          sorted({mats[i].shape[0] for i in huge}), FUSED_MAX_N))
    hs = set(huge)
    rest = [i for i in range(len(mats)) if i not in hs]
    outs = [None] * len(mats)
    for i, r in zip(rest, symeig_many([mats[i] for i in rest], clip, solver)):
        outs[i] = r
    for i in huge:
        d, Q = torch.linalg.eigh(mats[i].float())
        if clip is not None:
            d = torch.clamp(d, min=clip)
        outs[i] = (Q.contiguous(), d)
    return outs


_CHOL_BUFS = {}


def _chol_buffers(dev, n, b):
    key = (str(dev), n, b)
    bufs = _CHOL_BUFS.get(key)
    if bufs is None:
        wsb = int(_lib.lib().kfac_chol_ws_bytes(n))
        bufs = dict(out=torch.empty(b, n, n, dtype=torch.float32, device=dev), wsb=wsb,
                    ws=torch.zeros(b * wsb, dtype=torch.uint8, device=dev),
                    info_off=int(_lib.lib().kfac_chol_info_offset(n)))
        _CHOL_BUFS[key] = bufs
    return bufs


def inverse_many(mats, damping, check=True):
    """(F + damping I)^-1 for symmetric positive definite F (Cholesky), the
    reference's inverse path (kfac/layers/utils.py:76-96).

    GPU: every factor in ONE ragged launch sequence of the hand-written
    batched Cholesky / triangular inverse / X^T X product (csrc/chol.hip,
    damping fused into the first copy, a cached hipGraph); the factorisation
    status of all factors is checked with ONE host read at the end.  Results
    are views of persistent per-size-class buffers (callers copy them).
    CPU: torch.linalg.cholesky_ex + cholesky_inverse per size class."""
    outs = [None] * len(mats)
    if mats and _lib.use_native(mats[0]):
        _lib.check_pgemm_extent(max(A.shape[0] for A in mats))
        dev = mats[0].device
        classes = {}
        for i, A in enumerate(mats):
            classes.setdefault(A.shape[0], []).append(i)
        recs = (_lib.CholRecord * len(mats))()
        infos = []
        k = 0
        keep = []
        for n, idx in sorted(classes.items(), key=lambda kv: -kv[0]):
            B = _chol_buffers(dev, n, len(idx))
            for j, i in enumerate(idx):
                F = mats[i].float().contiguous()
                keep.append(F)
                r = recs[k]
                r.F, r.ldf = F.data_ptr(), F.stride(0)
                r.out, r.ldo = B['out'][j].data_ptr(), n
                r.ws, r.n = B['ws'].data_ptr() + j * B['wsb'], n
                outs[i] = B['out'][j]
                k += 1
            infos.append(B['ws'].view(len(idx), B['wsb'])[:, B['info_off']:B['info_off'] + 4])
        stream = _lib.stream(dev)
        _lib.check(_lib.lib().kfac_chol_inverse_batched(recs, len(mats), float(damping), 1,
                                                         stream), 'kfac_chol_inverse_batched')
        cur = torch.cuda.current_stream(dev)
        for F in keep:
            F.record_stream(cur)
        if check:
            bad = torch.cat([i.contiguous().view(torch.int32).reshape(-1) for i in infos]).ne(0)
            if bool(bad.any()):
                raise torch.linalg.LinAlgError(
                    'Cholesky of a damped factor failed (not positive definite)')
        return outs
    groups = {}
    for i, A in enumerate(mats):
        groups.setdefault((A.shape[0], A.dtype, A.device), []).append(i)
    infos = []
    for idx in groups.values():
        M = torch.stack([mats[i] for i in idx])
        M.diagonal(dim1=-2, dim2=-1).add_(damping)
        L, info = torch.linalg.cholesky_ex(M)
        inv = torch.cholesky_inverse(L)
        infos.append((idx, info))
        for k, i in enumerate(idx):
            outs[i] = inv[k]
    if check and infos:
        bad = torch.cat([info.reshape(-1) for _, info in infos]).ne(0)
        if bool(bad.any()):
            flat = [i for idx, _ in infos for i in idx]
            which = [flat[k] for k in bad.nonzero().reshape(-1).tolist()]
            raise torch.linalg.LinAlgError(
                'Cholesky of the damped factor(s) {} failed (not positive definite)'.format(which))
    return outs
