"""Kronecker-factor computation on MI355X: implicit-im2col SYRK + fused EMA.

`FactorSource` describes one hook tensor as an implicit patch matrix P
(rows = samples x output positions, cols = C*kh*kw [+1 bias]) and the scale
its P^T P contributes with; `update_factor()` accumulates every source into
an f32 workspace with `kfac_syrk_patch` (MFMA, upper tiles only) and folds
the running average + symmetrisation + dtype cast into `kfac_factor_ema`.
Two launches per factor update, no im2col materialisation, no host sync.

Reference math being reproduced: kfac/layers/conv.py:24-70,
kfac/layers/linear.py:12-59, kfac/layers/utils.py:13-43,164-178.
"""
import collections
import ctypes
import os

import torch

from . import _lib

__all__ = ['FactorSource', 'conv_input_source', 'conv_grad_source', 'linear_source',
           'update_factor', 'accumulate_sources']

# kh, kw, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w
Geometry = collections.namedtuple('Geometry', 'kh kw sh sw ph pw dh dw')
POINTWISE = Geometry(1, 1, 1, 1, 0, 0, 1, 1)


class FactorSource(object):
    """A (B, C, H, W)-strided tensor viewed as an implicit patch matrix."""
    __slots__ = ('x', 'geom', 'has_bias', 'scale', 'ncols', 'dscale')

    def __init__(self, x4d, geom, has_bias, scale, dscale=None):
        self.x, self.geom, self.has_bias, self.scale = x4d, geom, has_bias, float(scale)
        # optional device f32 scalar multiplying `scale` (AMP: finite(g) / s^2,
        # 0 drops the source; no host read)
        self.dscale = dscale
        self.ncols = x4d.shape[1] * geom.kh * geom.kw + (1 if has_bias else 0)

    @property
    def rows(self):
        B, _, H, W = self.x.shape
        g = self.geom
        oh = (H + 2 * g.ph - g.dh * (g.kh - 1) - 1) // g.sh + 1
        ow = (W + 2 * g.pw - g.dw * (g.kw - 1) - 1) // g.sw + 1
        return B * oh * ow, oh * ow


def conv_input_source(x, module_geom, has_bias):
    """Conv2d input (B, C, H, W); scale set later by the caller."""
    return FactorSource(x, Geometry(*module_geom), has_bias, 1.0)


def conv_grad_source(g):
    """Conv2d grad_output (B, Cout, OH, OW) as a pointwise patch matrix."""
    return FactorSource(g, POINTWISE, False, 1.0)


def linear_source(a2d, has_bias):
    """Linear input / grad_output flattened to (rows, features)."""
    if a2d.stride(-1) != 1:
        a2d = a2d.contiguous()
    x4 = a2d.as_strided((a2d.shape[0], a2d.shape[1], 1, 1),
                        (a2d.stride(0), a2d.stride(1), 1, 1))
    return FactorSource(x4, POINTWISE, has_bias, 1.0)


def _vec_eligible(s):
    """Mirror of kfac_syrk_vec's checks (channel-contiguous 16-bit data)."""
    x = s.x
    if x.dtype not in (torch.bfloat16, torch.float16):
        return False
    sb, sc, sh, sw = x.stride()
    _, C, H, W = x.shape
    return (sc == 1 and C % 8 == 0 and sb % 8 == 0 and (H == 1 or sh % 8 == 0) and
            (W == 1 or sw % 8 == 0) and x.data_ptr() % 16 == 0)


# fp32 inputs with at most 4 channels (ResNet's conv1 images) take the
# channels-contiguous grouped path as fp16 hi / lo planes (kfac_split_f16:
# 22 significand bits, the factor is the four plane-pair blocks' sum):
# KFAC_FACTOR_SPLIT=0 keeps them on the generic fp32 SYRK
SPLIT_F32 = os.environ.get('KFAC_FACTOR_SPLIT', '1') != '0'
split_launches = 0


def _split_eligible(sources):
    if not SPLIT_F32 or len(sources) != 1:
        return False
    s = sources[0]
    x = s.x
    return (x.is_cuda and x.dtype == torch.float32 and 1 <= x.shape[1] <= 4 and not s.has_bias
            and s.dscale is None and x.dim() == 4)


def _split_source(s):
    """The fp16 hi / lo plane image of an fp32 source (8 channels, NHWC) as
    a channels-contiguous source whose device dscale is 1 / s^2."""
    x = s.x
    B, C, H, W = x.shape
    dev = x.device
    out = torch.empty(B, H, W, 8, dtype=torch.float16, device=dev)
    part = torch.empty(int(_lib.lib().kfac_split_blocks()), dtype=torch.float32, device=dev)
    dscale = torch.empty(1, dtype=torch.float32, device=dev)
    sb, sc, sh, sw = x.stride()
    global split_launches
    split_launches += 1
    _lib.check(_lib.lib().kfac_split_f16(_lib.ptr(x), B, C, H, W, sb, sc, sh, sw, _lib.ptr(out),
                                         _lib.ptr(part), _lib.ptr(dscale), _lib.stream(dev)),
               'kfac_split_f16')
    return FactorSource(out.permute(0, 3, 1, 2), s.geom, False, s.scale, dscale=dscale), C


TILE = 128    # csrc/factors.hip output tile
# grouped SYRK: factors with at least KFAC_SYRK_WIDE_MIN columns use 256-wide
# output tiles (8 waves): each tile streams its two column panels for 4x the
# products, half the operand bytes per product.  Opt-in (0 = off): the
# ResNet-50 factor step measured 3.25-3.36 ms with wide tiles from n >= 256 /
# 512 / 1024 against 3.26-3.30 ms without (profiles/r6_syrk_wide*.log) --
# the grouped SYRK kernel (1.70 of the 3.3 ms) is not bound by its operand
# bytes; the EMA (0.74 ms), the fp32 conv1 path (0.51) and the tile
# reduction (0.36) are the rest (profiles/r6_factor_step_kernels.csv)
WIDE_MIN = int(os.environ.get('KFAC_SYRK_WIDE_MIN', '0'))


def _tile_width(n):
    return 256 if WIDE_MIN > 0 and n >= WIDE_MIN else TILE


def _tile_pairs(n, tw=TILE):
    t = (n + tw - 1) // tw
    return t * (t + 1) // 2


class RedJob(ctypes.Structure):
    """Mirror of csrc/factors.hip RedJob (size checked on first use)."""
    _fields_ = [('ws', ctypes.c_void_p), ('ldw', ctypes.c_int), ('ncols', ctypes.c_int),
                ('ntiles', ctypes.c_int), ('ncontrib', ctypes.c_int),
                ('part', ctypes.c_void_p * 8), ('splits', ctypes.c_int * 8),
                ('block_begin', ctypes.c_int), ('accum', ctypes.c_int),
                ('bt', ctypes.c_int), ('mirror', ctypes.c_int)]


def _red_jobs(ws_ptr, ldw, n, contribs, tw=TILE, mirror=False):
    """contribs: [(part pointer, splits)] in the fixed summation order ->
    one RedJob per chunk of MAX_CONTRIB contributions: chunk 0 stores, the
    later chunks add (launched in order by _tile_reduce: deterministic).
    mirror: store the strict lower triangle too (the grouped EMA's row reads)."""
    jobs = []
    for c0 in range(0, max(len(contribs), 1), MAX_CONTRIB):
        J = RedJob()
        J.ws, J.ldw, J.ncols, J.ntiles = ws_ptr, ldw, n, (n + tw - 1) // tw
        J.bt = tw
        J.mirror = int(mirror)
        chunk = contribs[c0:c0 + MAX_CONTRIB]
        J.ncontrib = len(chunk)
        J.accum = int(c0 > 0)
        for c, (ptr, sp) in enumerate(chunk):
            J.part[c] = ptr
            J.splits[c] = sp
        jobs.append(J)
    return jobs


def _check_red_layout():
    L = _lib.lib()
    if L.kfac_red_job_size() != ctypes.sizeof(RedJob) or L.kfac_red_max_contrib() != 8:
        raise RuntimeError('RedJob layout mismatch with the native library')
    if L.kfac_ema_job_size() != ctypes.sizeof(EmaJob):
        raise RuntimeError('EmaJob layout mismatch with the native library')


def accumulate_sources(sources, ws, allow_vec=True):
    """ws (n x n f32) = sum_s scale_s * P_s^T P_s  (upper triangle only).

    Deterministic: every (source, row split, tile pair) of the SYRK stores its
    partial tile and tile_reduce adds them in a fixed order (source, split)
    -- one launch per MAX_CONTRIB sources, chained -- bitwise-reproducible
    factors for any number of sources, no f32 atomics.
    Returns None when ws is in the reference column order (c, kh, kw), or
    (kcols, C, kh*kw) when the channels-contiguous fast path filled it in the
    internal order (kh, kw, c) -- `kfac_factor_ema_perm` maps it back."""
    L = _lib.lib()
    stream = _lib.stream(ws.device)
    n = ws.shape[0]
    det = True
    _check_red_layout()
    vec = allow_vec and all(_vec_eligible(s) for s in sources)
    parts, contribs = [], []
    if det:
        sizes = []
        for s in sources:
            sp = int(L.kfac_syrk_splits(int(vec), s.rows[0], n, 0))
            sizes.append(sp)
        total = sum(sp * _tile_pairs(n) for sp in sizes) * TILE * TILE
        arena = _lib.workspace(ws.device, max(total, 1), tag='syrk_parts')
        off = 0
        for sp in sizes:
            ptr = arena.data_ptr() + 4 * off
            parts.append(_lib.c_vp(ptr))
            contribs.append((ptr, sp))
            off += sp * _tile_pairs(n) * TILE * TILE
    else:
        parts = [None] * len(sources)
    if vec:
        order = None
        for s, part in zip(sources, parts):
            x = s.x
            B, C, H, W = x.shape
            sb, sc, sh, sw = x.stride()
            g = s.geom
            if s.ncols != n:
                raise ValueError('factor source has {} columns, workspace {}'.format(s.ncols, n))
            r = L.kfac_syrk_vec(_lib.DTYPE_CODE[x.dtype], _lib.ptr(x), sb, sc, sh, sw, B, C, H, W,
                                g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.dh, g.dw, int(s.has_bias),
                                s.scale, _lib.ptr(ws), ws.stride(0), 0, part,
                                _dptr(s.dscale), stream)
            if r != 1:
                raise RuntimeError('kfac_syrk_vec failed ({})'.format(r))
            kk = g.kh * g.kw
            o = (C * kk, C, kk)
            if order is not None and order != o:
                raise ValueError('factor sources disagree on the patch geometry')
            order = o
        _tile_reduce([_red_jobs(ws.data_ptr(), ws.stride(0), n, contribs)], stream)
        return None if order[2] == 1 else order
    for s, part in zip(sources, parts):
        x = s.x
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
            x = x.float()
        if s.ncols != n:
            raise ValueError('factor source has {} columns, workspace {}'.format(s.ncols, n))
        B, C, H, W = x.shape
        sb, sc, sh, sw = x.stride()
        g = s.geom
        if x.numel() >= 2 ** 31 - 1:
            raise ValueError('activation too large for 32-bit column offsets')
        _lib.check(L.kfac_syrk_patch(
            _lib.DTYPE_CODE[x.dtype], _lib.ptr(x), sb, sc, sh, sw, B, C, H, W,
            g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.dh, g.dw, int(s.has_bias), s.scale,
            _lib.ptr(ws), ws.stride(0), 0, part, _dptr(s.dscale), stream), 'kfac_syrk_patch')
    _tile_reduce([_red_jobs(ws.data_ptr(), ws.stride(0), n, contribs)], stream)
    return None


MAX_CONTRIB = 8    # csrc/factors.hip: sources per tile-reduction job


def _tile_reduce(job_chains, stream):
    """job_chains: per factor, its chunk jobs (_red_jobs).  Level l launches
    chunk l of every factor that has one, in order."""
    depth = max(len(c) for c in job_chains)
    for lvl in range(depth):
        jobs = [c[lvl] for c in job_chains if len(c) > lvl]
        arr = (RedJob * len(jobs))(*jobs)
        _lib.check(_lib.lib().kfac_tile_reduce(arr, len(jobs), stream), 'kfac_tile_reduce')


def _dptr(t):
    return None if t is None else _lib.ptr(t)


def _ema(state, ws, n, alpha, mode, order, keep=None):
    """keep: None or a device f32 flag; 0 leaves the factor untouched (AMP:
    no finite source this step, the reference skips the update)."""
    L = _lib.lib()
    dev = ws.device
    if order is None:
        _lib.check(L.kfac_factor_ema(_lib.DTYPE_CODE[state.dtype], _lib.ptr(state), _lib.ptr(ws),
                                     n, n, float(alpha), mode, _dptr(keep), _lib.stream(dev)),
                   'kfac_factor_ema')
    else:
        kcols, C, kk = order
        _lib.check(L.kfac_factor_ema_perm(_lib.DTYPE_CODE[state.dtype], _lib.ptr(state),
                                          _lib.ptr(ws), n, n, float(alpha), mode, kcols, C, kk,
                                          _dptr(keep), _lib.stream(dev)), 'kfac_factor_ema_perm')


def update_factor(state, sources, alpha, out_dtype, keep=None):
    """Running-average factor update on the GPU.

    state: existing factor (n x n, any of f32/bf16/f16) or None (-> identity).
    Returns the (possibly new) state tensor, updated in place:
        state = alpha * state + (1 - alpha) * sum_s scale_s P_s^T P_s
    alpha == 1 leaves the state untouched (reference semantics).
    """
    n = sources[0].ncols
    dev = sources[0].x.device
    if state is None:
        state = torch.eye(n, dtype=out_dtype, device=dev)
    if alpha == 1:
        return state
    ws = _lib.workspace(dev, n * n).view(n, n)
    order = accumulate_sources(sources, ws)
    _ema(state, ws, n, alpha, 0, order, keep)
    return state


def compute_cov(sources, out_dtype=torch.float32):
    """sum_s scale_s P_s^T P_s as a fresh symmetric matrix (no running average)."""
    n = sources[0].ncols
    dev = sources[0].x.device
    ws = _lib.workspace(dev, n * n).view(n, n)
    order = accumulate_sources(sources, ws)
    out = torch.empty(n, n, dtype=out_dtype, device=dev)
    _ema(out, ws, n, 0.0, 1, order)
    return out


# ---------------------------------------------------------------- grouped
class EmaJob(ctypes.Structure):
    _fields_ = [('state', ctypes.c_void_p), ('ws', ctypes.c_void_p),
                ('n', ctypes.c_int), ('ldw', ctypes.c_int), ('kcols', ctypes.c_int),
                ('C', ctypes.c_int), ('kk', ctypes.c_int), ('sdtype', ctypes.c_int),
                ('row_begin', ctypes.c_int), ('full', ctypes.c_int),
                ('a1', ctypes.c_float), ('a2', ctypes.c_float),
                ('mode', ctypes.c_int), ('cint', ctypes.c_int), ('lo', ctypes.c_int),
                ('pad3', ctypes.c_int), ('keep', ctypes.c_void_p)]


SPLIT_ROWS = 2048   # patch rows per block of the grouped SYRK


def update_factors_grouped(items, alpha, tag=''):
    """Running-average update of MANY factors in a fixed number of launches.

    items: list of (state_or_None, sources, out_dtype[, keep]) -- keep: None or
    a device f32 flag (0: leave the factor as it is).  Returns the list of
    updated states (new identity-initialised tensors where state was None).
    Every factor whose sources all qualify for the channels-contiguous path
    goes through ONE grouped SYRK launch per input dtype plus ONE grouped EMA
    launch; the rest fall back to the per-factor path.  One memset zeroes the
    shared f32 workspace arena.  `tag` names the workspaces: calls that may
    run concurrently on different streams (KFAC(early_factors=True)) use
    different tags.
    """
    if not items:
        return []
    L = _lib.lib()
    dev = items[0][1][0].x.device
    stream = _lib.stream(dev)
    out = [None] * len(items)
    grouped, rest = [], []
    items = [tuple(it) + (None,) * (4 - len(it)) for it in items]
    split = {}        # k -> reference channel count of a split (fp16 hi / lo) factor
    for k, (state, sources, out_dtype, keep) in enumerate(items):
        if alpha != 1 and all(_vec_eligible(s) for s in sources) and \
                len({(s.x.dtype, s.x.shape[1], s.geom.kh * s.geom.kw) for s in sources}) == 1:
            grouped.append(k)
        elif alpha != 1 and _split_eligible(sources):
            src, split[k] = _split_source(sources[0])
            items[k] = (state, [src], out_dtype, keep)
            grouped.append(k)
        else:
            rest.append(k)
    for k in rest:
        state, sources, out_dtype, keep = items[k]
        out[k] = update_factor(state, sources, alpha, out_dtype, keep)
    if not grouped:
        return out
    _check_red_layout()
    sizes = [items[k][1][0].ncols for k in grouped]
    total = sum(n * n for n in sizes)
    # no memset: tile_reduce writes every upper-triangle element the EMA reads
    arena = _lib.workspace(dev, total, tag='syrk_grouped' + tag)
    psize = L.kfac_syrk_problem_size()
    by_dtype = {}
    ws_of = {}
    off = 0
    for k, n in zip(grouped, sizes):
        ws_of[k] = (off, n)
        off += n * n
        for s in items[k][1]:
            by_dtype.setdefault(s.x.dtype, []).append((k, s))
    contribs = {k: [] for k in grouped}
    launches = []
    for dtype, probs in by_dtype.items():
        raw = ctypes.create_string_buffer(psize * len(probs))
        blocks = 0
        nbs = []
        for i, (k, s) in enumerate(probs):
            x = s.x
            B, C, H, W = x.shape
            sb, sc, sh, sw = x.stride()
            g = s.geom
            woff, n = ws_of[k]
            ws_ptr = arena.data_ptr() + 4 * woff
            nb = L.kfac_syrk_problem_init(
                ctypes.byref(raw, i * psize), blocks, _lib.DTYPE_CODE[dtype], _lib.ptr(x),
                sb, sc, sh, sw, B, C, H, W, g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.dh, g.dw,
                int(s.has_bias), s.scale, _lib.c_vp(ws_ptr), n, SPLIT_ROWS, _tile_width(n))
            if nb <= 0:
                raise RuntimeError('grouped SYRK rejected an eligible source')
            nbs.append(nb)
            blocks += nb
        launches.append((dtype, probs, raw, nbs))
    # partial tiles of every (problem, split, tile pair): one arena, then the
    # fixed-order tile reduction per factor (sources in order, splits in order)
    tot_parts = sum(nb * _tile_width(ws_of[k][1]) ** 2
                    for _, probs, _, nbs in launches for (k, _), nb in zip(probs, nbs))
    parts = _lib.workspace(dev, tot_parts, tag='syrk_parts_grouped' + tag)
    poff = 0
    for dtype, probs, raw, nbs in launches:
        for i, ((k, s), nb) in enumerate(zip(probs, nbs)):
            ptr = parts.data_ptr() + 4 * poff
            L.kfac_syrk_problem_set_part(ctypes.byref(raw, i * psize), _lib.c_vp(ptr))
            L.kfac_syrk_problem_set_dscale(ctypes.byref(raw, i * psize), _dptr(s.dscale))
            tw = _tile_width(ws_of[k][1])
            contribs[k].append((ptr, nb // _tile_pairs(ws_of[k][1], tw)))
            poff += nb * tw * tw
        _lib.check(L.kfac_syrk_grouped(raw, len(probs), _lib.DTYPE_CODE[dtype], stream),
                   'kfac_syrk_grouped')
    # both triangles: the EMA below reads whole rows of the workspace (its
    # column walks over the upper triangle were most of its time)
    _tile_reduce([_red_jobs(arena.data_ptr() + 4 * ws_of[k][0], ws_of[k][1], ws_of[k][1],
                            contribs[k], _tile_width(ws_of[k][1]), mirror=True)
                  for k in grouped], stream)
    jobs = (EmaJob * len(grouped))()
    a1, a2 = alpha / (1.0 - alpha), 1.0 - alpha
    for j, k in enumerate(grouped):
        state, sources, out_dtype, keep = items[k]
        n = ldw = sizes[j]
        s0 = sources[0]
        kk = s0.geom.kh * s0.geom.kw
        C = cint = s0.x.shape[1]
        lo = 0
        if k in split:      # internal 8-channel planes -> the reference C x kh x kw factor
            C = lo = split[k]
            n = C * kk
        if state is None:
            state = torch.eye(n, dtype=out_dtype, device=dev)
        out[k] = state
        woff, _ = ws_of[k]
        J = jobs[j]
        J.state, J.ws = state.data_ptr(), arena.data_ptr() + 4 * woff
        J.n, J.ldw, J.kcols, J.C, J.kk = n, ldw, C * kk, C, kk
        J.cint, J.lo = cint, lo
        J.sdtype = _lib.DTYPE_CODE[state.dtype]
        J.a1, J.a2, J.mode = a1, a2, 0
        J.full = 1
        J.keep = None if keep is None else keep.data_ptr()
    _lib.check(L.kfac_ema_grouped(jobs, len(grouped), stream), 'kfac_ema_grouped')
    return out
