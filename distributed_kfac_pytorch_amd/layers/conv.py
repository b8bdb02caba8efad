"""K-FAC layer for nn.Conv2d (reference: kfac/layers/conv.py:10-70).

KFC approximation with the reference's exact scaling:
  A = P^T P / (B * S^3)   P = im2col patches [+ ones column], S = OH*OW
  G = g^T g / (B * S^3)   g = grad_output as (B*S, Cout)
On the GPU the patches are never materialised: `_a_sources` hands the raw
(B, C, H, W) activation (NCHW or channels_last strides) plus the conv
geometry to the implicit-im2col SYRK kernel.  Dilation is supported on both
paths (the reference silently ignored it: defect #14); grouped convolutions
and non-zero padding modes are rejected.
"""
import torch

from . import utils as lutils
from .base import KFACLayer
from ..ops import factors as factor_ops

__all__ = ['Conv2dLayer']


class Conv2dLayer(KFACLayer):
    def __init__(self, *args, **kwargs):
        super(Conv2dLayer, self).__init__(*args, **kwargs)
        m = self.module
        self.has_bias = m.bias is not None
        if not self.batch_first:
            raise ValueError('Conv2D layer must use batch_first=True')
        if m.groups != 1:
            raise ValueError('K-FAC Conv2dLayer does not support grouped convolutions '
                             '(groups={})'.format(m.groups))
        if getattr(m, 'padding_mode', 'zeros') != 'zeros':
            raise ValueError('K-FAC Conv2dLayer only supports zero padding')
        padding = m.padding
        if isinstance(padding, str):
            if padding == 'valid':
                padding = (0, 0)
            else:  # 'same': symmetric for odd kernels
                rp = m._reversed_padding_repeated_twice
                if rp[0] != rp[1] or rp[2] != rp[3]:
                    raise ValueError('asymmetric "same" padding is not supported')
                padding = (rp[2], rp[0])
        self.padding = tuple(padding)
        self.geometry = (m.kernel_size[0], m.kernel_size[1], m.stride[0], m.stride[1],
                         self.padding[0], self.padding[1], m.dilation[0], m.dilation[1])

    def weight_grad_2d(self):
        g = self._get_weight_grad()
        return g.reshape(g.size(0), -1)

    def _patches(self, x):
        m = self.module
        if tuple(m.dilation) == (1, 1):
            return lutils.extract_patches(x, m.kernel_size, m.stride, self.padding)
        cols = torch.nn.functional.unfold(x, m.kernel_size, dilation=m.dilation,
                                          padding=self.padding, stride=m.stride)
        B = x.shape[0]
        kh, kw, sh, sw, ph, pw, dh, dw = self.geometry
        oh = (x.shape[2] + 2 * ph - dh * (kh - 1) - 1) // sh + 1
        ow = (x.shape[3] + 2 * pw - dw * (kw - 1) - 1) // sw + 1
        return cols.transpose(1, 2).reshape(B, oh, ow, -1)

    def _get_A_factor(self, a_inputs):
        parts = []
        for x in a_inputs:
            p = self._patches(x)
            spatial = p.size(1) * p.size(2)
            p = p.reshape(-1, p.size(-1))
            if self.has_bias:
                p = lutils.append_bias_ones(p)
            parts.append(p / spatial)
        a = lutils.reshape_data(parts, batch_first=self.batch_first)
        return lutils.get_cov(a)

    def _get_G_factor(self, g_outputs):
        parts = []
        for g in g_outputs:
            spatial = g.size(2) * g.size(3)
            g2 = g.permute(0, 2, 3, 1).contiguous().view(-1, g.size(1))
            parts.append(g2 / spatial)
        g = lutils.reshape_data(parts, batch_first=self.batch_first)
        return lutils.get_cov(g)

    def _a_sources(self, a_inputs):
        srcs = [factor_ops.conv_input_source(x, self.geometry, self.has_bias) for x in a_inputs]
        rows = [s.rows for s in srcs]
        total = sum(r for r, _ in rows)
        for s, (r, spatial) in zip(srcs, rows):
            s.scale = 1.0 / (float(spatial) ** 2 * total)
        return srcs

    def _g_sources(self, g_outputs):
        srcs = [factor_ops.conv_grad_source(g) for g in g_outputs]
        total = sum(g.shape[0] * g.shape[2] * g.shape[3] for g in g_outputs)
        for s, g in zip(srcs, g_outputs):
            spatial = g.shape[2] * g.shape[3]
            s.scale = 1.0 / (float(spatial) ** 2 * total)
        return srcs

    def _g_rows(self, g):
        return g.shape[0] * g.shape[2] * g.shape[3]
