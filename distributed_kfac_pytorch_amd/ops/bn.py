"""Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels_last
bf16 activations (csrc/bn.hip) -- the normalisation layers of the ResNet-50
benchmark model (models/resnet.py).

`bn_act(x, bn, relu=True, z=None)` computes ``relu(bn(x) + z)`` (each part
optional) with the semantics of `nn.BatchNorm2d` in training mode: batch
statistics (biased variance) normalise, the running statistics move by
`momentum` with the unbiased variance, `num_batches_tracked` counts the call.
On a GPU, for a bf16 channels_last input with C % 8 == 0, it is three
kernels forward and three backward (hipGraph-capturable, deterministic);
anything else (CPU, eval mode, fp32, other layouts, momentum=None) takes the
stock `bn(x)` path.  `KFAC_FUSED_BN=0` disables the fused kernels.

The K-FAC layers hook Conv2d / Linear only; BatchNorm is not preconditioned
(reference: kfac/layers/__init__.py registers Linear and Conv2d), so this
changes the model's kernels, not the optimiser's math.
"""
import os

import torch
import torch.nn.functional as F

from . import _lib

__all__ = ['bn_act', 'eligible', 'ENABLED']

ENABLED = os.environ.get('KFAC_FUSED_BN', '1') != '0'


def _nhwc(t):
    return (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)
            and t.data_ptr() % 16 == 0)


def eligible(x, bn, z=None):
    if not (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and bn.training):
        return False
    if not (bn.affine and bn.track_running_stats and bn.momentum is not None
            and bn.running_mean is not None):
        return False
    if x.shape[1] % 8 or not _nhwc(x) or x.numel() == 0:
        return False
    if z is not None and (z.dtype != x.dtype or z.shape != x.shape or not _nhwc(z)):
        return False
    return True


def _ptr(t):
    return None if t is None else t.data_ptr()


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, z, bn, relu):
        L = _lib.lib()
        N, C, H, W = x.shape
        M = N * H * W
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(L.kfac_bn_ws_floats(M, C)), dtype=torch.float32, device=x.device)
        nbt = bn.num_batches_tracked
        _lib.check(L.kfac_bn_forward(x.data_ptr(), _ptr(z), weight.data_ptr(), bias.data_ptr(),
                                     bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                     _ptr(nbt), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                     ws.data_ptr(), M, C, float(bn.eps), float(bn.momentum),
                                     int(relu), _lib.stream(x.device)), 'kfac_bn_forward')
        ctx.save_for_backward(x, y, weight, mean, invstd)
        ctx.relu, ctx.has_z = bool(relu), z is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, y, weight, mean, invstd = ctx.saved_tensors
        N, C, H, W = x.shape
        M = N * H * W
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dz = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_z else None
        dw = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(L.kfac_bn_ws_floats(M, C)), dtype=torch.float32, device=x.device)
        _lib.check(L.kfac_bn_backward(dy.data_ptr(), y.data_ptr() if ctx.relu else None,
                                      x.data_ptr(), weight.data_ptr(), mean.data_ptr(),
                                      invstd.data_ptr(), dx.data_ptr(), _ptr(dz), dw.data_ptr(),
                                      db.data_ptr(), ws.data_ptr(), M, C, int(ctx.relu),
                                      _lib.stream(x.device)), 'kfac_bn_backward')
        return dx, dw.to(weight.dtype), db.to(weight.dtype), dz, None, None


def bn_act(x, bn, relu=True, z=None):
    """relu(bn(x) [+ z]) -- fused on eligible GPU inputs, stock ops otherwise."""
    if eligible(x, bn, z):
        return _BNAct.apply(x, bn.weight, bn.bias, z, bn, relu)
    y = bn(x)
    if z is not None:
        y = y + z
    return F.relu(y) if relu else y
