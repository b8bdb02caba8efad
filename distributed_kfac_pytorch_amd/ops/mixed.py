"""bf16 model weights with fp32 master copies, cast in ONE launch per direction.

`torch.autocast(dtype=torch.bfloat16)` re-casts every fp32 Conv/Linear weight
to bf16 in each forward and widens every bf16 weight gradient back to fp32 in
each backward: one small elementwise launch per tensor and direction (~110 per
ResNet-50 step, ~1.4 ms; profiles/r3_s2_bench_window_breakdown.txt).
`BF16Weights(model)` stores those weights in bf16 (autocast then has nothing
to cast) and keeps fp32 masters for the optimizer and K-FAC:

    forward / backward        bf16 weights, bf16 weight gradients (the values
                              autocast produces before widening them)
    grads_to_master()         master.grad = fp32(weight.grad), one launch
    K-FAC step                reads and writes the fp32 master gradients
                              (KFAC.set_grad_params)
    optimizer.step()          on the fp32 masters
    master_to_model()         weight = bf16_rne(master), one launch

The numerics are those of autocast: its forward operand is the same RNE bf16
cast of the fp32 weight, its fp32 gradient the same widened bf16 gradient.
Casts: csrc/mixed.hip (kfac_cast_grouped); CPU tensors use torch copies.
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib

__all__ = ['BF16Weights']


class _CastRec(ctypes.Structure):
    _fields_ = [('src', ctypes.c_void_p), ('dst', ctypes.c_void_p), ('n', ctypes.c_longlong)]


class BF16Weights(object):
    """Args:
      model: the module tree; every Conv/Linear (or `module_types`) weight and
        bias is converted to bf16 in place.
    Use `parameters(model)` for the optimizer (masters replace the converted
    parameters, order preserved), call `grads_to_master()` after backward and
    `master_to_model()` after the optimizer step, and hand `grad_params()` to
    `KFAC.set_grad_params` so K-FAC preconditions the fp32 master gradients.
    """

    def __init__(self, model, module_types=(nn.Conv2d, nn.Linear)):
        self.pairs = []            # (bf16 model parameter, fp32 master)
        self._master = {}
        for m in model.modules():
            if not isinstance(m, module_types):
                continue
            for name in ('weight', 'bias'):
                p = getattr(m, name, None)
                if p is None or not p.requires_grad or p.dtype != torch.float32:
                    continue
                master = nn.Parameter(p.detach().clone(memory_format=torch.preserve_format))
                with torch.no_grad():
                    p.data = p.data.to(torch.bfloat16)
                if p.stride() != master.stride():
                    raise ValueError('bf16 weight and master layouts differ: {} vs {}'.format(
                        p.stride(), master.stride()))
                master.grad = torch.zeros_like(master)
                self.pairs.append((p, master))
                self._master[id(p)] = master
        self._recs = {}

    def parameters(self, model):
        """model.parameters() with every converted weight replaced by its master."""
        return [self._master.get(id(p), p) for p in model.parameters()]

    def grad_params(self):
        """{bf16 model parameter: fp32 master} for KFAC.set_grad_params."""
        return {p: m for p, m in self.pairs}

    def _cast(self, pairs, mode):
        if not pairs:
            return
        if not _lib.use_native(pairs[0][0]):
            for src, dst in pairs:
                dst.copy_(src)
            return
        key = tuple((s.data_ptr(), d.data_ptr()) for s, d in pairs)
        cached = self._recs.get(mode)
        if cached is not None and cached[0] == key:
            recs = cached[1]
        else:
            recs = (_CastRec * len(pairs))()
            for r, (s, d) in zip(recs, pairs):
                if s.numel() != d.numel() or s.stride() != d.stride():
                    raise ValueError('cast operands differ in shape or layout')
                r.src, r.dst, r.n = s.data_ptr(), d.data_ptr(), s.numel()
            self._recs[mode] = (key, recs)
        _lib.check(_lib.lib().kfac_cast_grouped(recs, len(pairs), mode,
                                                _lib.stream(pairs[0][0].device)),
                   'kfac_cast_grouped')

    def master_of(self, p):
        """The fp32 master of a converted parameter, else `p` itself."""
        return self._master.get(id(p), p)

    def subset(self, params):
        """A BF16Weights view over the pairs whose model parameter is in
        `params` (e.g. one backward segment's, parallel/overlap.py): its own
        grads_to_master / master_to_model launches."""
        ids = {id(p) for p in params}
        sub = BF16Weights.__new__(BF16Weights)
        sub.pairs = [(p, m) for p, m in self.pairs if id(p) in ids]
        sub._master = {id(p): m for p, m in sub.pairs}
        sub._recs = {}
        return sub

    def zero_model_grads(self):
        """Drop the bf16 weight gradients (backward allocates fresh ones)."""
        for p, _ in self.pairs:
            p.grad = None

    @torch.no_grad()
    def grads_to_master(self):
        """master.grad = fp32(weight.grad) for every pair (zeros where the
        weight has no gradient).  The masters' .grad tensors may be rebound
        (e.g. to flat all-reduce arena views, parallel/grad_sync.py)."""
        todo = []
        for p, m in self.pairs:
            if m.grad is None:
                m.grad = torch.zeros_like(m)
            if p.grad is None:
                m.grad.zero_()
            else:
                todo.append((p.grad, m.grad))
        self._cast(todo, 0)

    @torch.no_grad()
    def master_to_model(self):
        """weight = bf16(master) for every pair (round to nearest even)."""
        self._cast([(m, p.data) for p, m in self.pairs], 1)
