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

import torch

from . import _lib

__all__ = ['FactorSource', 'conv_input_source', 'conv_grad_source', 'linear_source',
           'update_factor', 'accumulate_sources']

# kh, kw, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w
Geometry = collections.namedtuple('Geometry', 'kh kw sh sw ph pw dh dw')
POINTWISE = Geometry(1, 1, 1, 1, 0, 0, 1, 1)


class FactorSource(object):
    """A (B, C, H, W)-strided tensor viewed as an implicit patch matrix."""
    __slots__ = ('x', 'geom', 'has_bias', 'scale', 'ncols')

    def __init__(self, x4d, geom, has_bias, scale):
        self.x, self.geom, self.has_bias, self.scale = x4d, geom, has_bias, float(scale)
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


def accumulate_sources(sources, ws):
    """ws (n x n f32, zeroed) += sum_s scale_s * P_s^T P_s  (upper triangle only)."""
    L = _lib.lib()
    stream = _lib.stream(ws.device)
    n = ws.shape[0]
    for s in sources:
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
            _lib.ptr(ws), ws.stride(0), 0, stream), 'kfac_syrk_patch')


def update_factor(state, sources, alpha, out_dtype):
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
    ws.zero_()
    accumulate_sources(sources, ws)
    L = _lib.lib()
    _lib.check(L.kfac_factor_ema(_lib.DTYPE_CODE[state.dtype], _lib.ptr(state), _lib.ptr(ws), n,
                                 n, float(alpha), 0, _lib.stream(dev)), 'kfac_factor_ema')
    return state


def compute_cov(sources, out_dtype=torch.float32):
    """sum_s scale_s P_s^T P_s as a fresh symmetric matrix (no running average)."""
    n = sources[0].ncols
    dev = sources[0].x.device
    ws = _lib.workspace(dev, n * n).view(n, n)
    ws.zero_()
    accumulate_sources(sources, ws)
    out = torch.empty(n, n, dtype=out_dtype, device=dev)
    _lib.check(_lib.lib().kfac_factor_ema(_lib.DTYPE_CODE[out_dtype], _lib.ptr(out), _lib.ptr(ws),
                                          n, n, 0.0, 1, _lib.stream(dev)), 'kfac_factor_ema')
    return out
