"""Gradient preconditioning on MI355X (K7, K8, K10, K11).

`precondition_eigen` computes, per layer,
    out = QG @ ((QG^T @ grad @ QA) * dGdA) @ QA^T          (prediv)
    out = QG @ ((QG^T @ grad @ QA) / (dG dA^T + damping)) @ QA^T
with the four GEMMs on hipBLASLt/rocBLAS (plain library GEMMs) writing
straight into the preconditioned-gradient arena, and the Hadamard step as
a HIP kernel.  `kl_dot` and `apply_gradients` then process ALL layers in
one launch each, with the KL-clip scale living on the device (no host
sync; the reference does >= 54 .item() per step).

Reference: kfac/layers/base.py:321-362,459-483, kfac/preconditioner.py:661-682.
"""
import math

import torch

from . import _lib

__all__ = ['outer_reciprocal', 'precondition_eigen', 'precondition_inverse', 'kl_dot',
           'kl_scale_reference',
           'apply_gradients']


def outer_reciprocal(dG, dA, damping, out=None):
    """1 / (dG[:, None] * dA[None, :] + damping) (written into `out`, a
    contiguous fp32 nG x nA tensor, when given)."""
    if _lib.use_native(dG) and dG.dtype == torch.float32 and dA.dtype == torch.float32:
        if out is None or out.dtype != torch.float32 or not out.is_contiguous() or \
                out.shape != (dG.shape[0], dA.shape[0]):
            out = torch.empty(dG.shape[0], dA.shape[0], dtype=torch.float32, device=dG.device)
        _lib.check(_lib.lib().kfac_outer_recip(_lib.ptr(dG), _lib.ptr(dA), _lib.ptr(out),
                                               dG.shape[0], dA.shape[0], float(damping),
                                               _lib.stream(dG.device)), 'kfac_outer_recip')
        return out
    return 1 / (dG.unsqueeze(1) * dA.unsqueeze(0) + damping)


def precondition_eigen(grad, QA, QG, dGdA=None, dA=None, dG=None, damping=0.0, out=None):
    """Eigenbasis preconditioning; result in float32 (written into `out` if given)."""
    native = _lib.use_native(grad) and grad.dtype == torch.float32
    v1 = torch.matmul(torch.matmul(QG.t(), grad), QA)
    if native:
        nG, nA = v1.shape
        L = _lib.lib()
        if dGdA is not None:
            _lib.check(L.kfac_hadamard(_lib.ptr(v1), nA, _lib.ptr(dGdA), None, None, nG, nA, 0.0,
                                       0, _lib.stream(grad.device)), 'kfac_hadamard')
        else:
            _lib.check(L.kfac_hadamard(_lib.ptr(v1), nA, None, _lib.ptr(dG), _lib.ptr(dA), nG, nA,
                                       float(damping), 1, _lib.stream(grad.device)),
                       'kfac_hadamard')
        v2 = v1
    else:
        if dGdA is not None:
            v2 = v1 * dGdA
        else:
            v2 = v1 / (dG.unsqueeze(1) * dA.unsqueeze(0) + damping)
    tmp = torch.matmul(QG, v2)
    if out is not None and out.dtype == tmp.dtype:
        torch.matmul(tmp, QA.t(), out=out)
        return out
    res = torch.matmul(tmp, QA.t()).to(torch.float32)
    if out is not None:
        out.copy_(res)
        return out
    return res


def precondition_inverse(grad, A_inv, G_inv, out=None):
    res = torch.matmul(torch.matmul(G_inv, grad), A_inv)
    if out is not None:
        out.copy_(res)
        return out
    return res.to(torch.float32)


def _records(pairs):
    """pairs: (v, g) with v a row-strided (rows x cols) f32 view of the
    preconditioned gradient and g the parameter's .grad in any layout whose
    logical shape flattens to (rows, cols) in K-FAC column order (c, kh, kw)."""
    recs = (_lib.MatRecord * len(pairs))()
    for i, (v, g) in enumerate(pairs):
        if v.dim() != 2 or v.stride(1) != 1:
            raise ValueError('kl/apply expects a row-strided 2-D v')
        r = recs[i]
        r.v = v.data_ptr()
        r.g = g.data_ptr()
        r.ldv = v.stride(0)
        r.rows, r.cols = v.shape
        r.gdtype = _lib.DTYPE_CODE[g.dtype]
        st = g.stride()
        if g.dim() == 4:
            r.gs0, r.gs1, r.gs2, r.gs3 = st
            r.kk, r.kw = g.shape[2] * g.shape[3], g.shape[3]
        elif g.dim() == 2:
            r.gs0, r.gs1, r.gs2, r.gs3 = st[0], st[1], 0, 0
            r.kk, r.kw = 1, 1
        elif g.dim() == 1:
            r.gs0, r.gs1, r.gs2, r.gs3 = st[0], 0, 0, 0
            r.kk, r.kw = 1, 1
        else:
            raise ValueError('unsupported gradient rank {}'.format(g.dim()))
        if g.numel() != v.numel():
            raise ValueError('gradient / preconditioned gradient size mismatch')
    return recs


def kl_dot(pairs):
    """sum over (v, g) pairs of <v, g> as a device float64 scalar.

    v: 2-D row-strided float32 view of a preconditioned gradient;
    g: the matching .grad (any memory layout, e.g. channels_last conv weights).
    """
    v0 = pairs[0][0]
    if _lib.use_native(v0):
        # result + one partial slot per workgroup (summed in a fixed order on
        # the device: bit-identical on every rank)
        L = _lib.lib()
        per = int(L.kfac_kl_elems_per_block())
        slots = sum((v.numel() + per - 1) // per for v, _ in pairs)
        buf = torch.empty(1 + slots, dtype=torch.float64, device=v0.device)
        _lib.check(L.kfac_grouped_kl_dot(_records(pairs), len(pairs), _lib.ptr(buf),
                                         _lib.stream(v0.device)), 'kfac_grouped_kl_dot')
        return buf[0]
    vg = torch.zeros((), dtype=torch.float64)
    for v, g in pairs:
        vg += (v.reshape(g.shape) * g).sum().double()
    return vg


def kl_scale(vg, lr, kl_clip):
    """Host-side KL-clip scale (CPU path): None when vg == 0."""
    s = float(vg) * lr ** 2
    if s == 0.0:
        return None
    return min(1.0, math.sqrt(kl_clip / abs(s)))


def kl_scale_reference(pairs, lr, kl_clip):
    """KL-clip scale of the host path with the reference's rounding
    (/root/reference/kfac/preconditioner.py:660-682): one float32 sum of
    v * g * lr^2 per tensor, accumulated as a Python float; None when 0."""
    s = 0.0
    for v, g in pairs:
        s += (v.reshape(g.shape) * g * lr ** 2).sum().item()
    if s == 0.0:
        return None
    return min(1.0, math.sqrt(kl_clip / abs(s)))


def apply_gradients(pairs, vg=None, lr=0.0, kl_clip=None):
    """g <- nu * v for every pair; nu from the device-side KL sum (or 1)."""
    v0 = pairs[0][0]
    use_clip = vg is not None and kl_clip is not None
    if _lib.use_native(v0):
        vgp = _lib.ptr(vg) if use_clip else None
        _lib.check(_lib.lib().kfac_grouped_apply(_records(pairs), len(pairs), vgp,
                                                 float(lr) ** 2, float(kl_clip or 0.0),
                                                 int(use_clip), _lib.stream(v0.device)),
                   'kfac_grouped_apply')
        return
    nu = kl_scale(vg, lr, kl_clip) if use_clip else None
    for v, g in pairs:
        v = v.reshape(g.shape)
        g.copy_(v if nu is None else nu * v)
