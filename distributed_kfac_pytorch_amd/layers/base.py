"""Per-layer K-FAC state machine (factors, eigendata/inverses, preconditioned grad).

API parity with the reference KFACLayer (kfac/layers/base.py:10-484):
state_dict / load_state_dict, assign_inverse_workers / assign_gradient_workers,
allreduce_factors / broadcast_inverses / broadcast_gradient,
compute_A_inv / compute_G_inv, get_gradient, compute_preconditioned_gradient,
save_inputs / save_grad_outputs, update_A_factor / update_G_factor,
update_gradient.

What is different underneath:
  * On a GPU tensor every numeric step goes through the gfx950 kernels in
    ops/ (implicit-im2col MFMA SYRK with fused EMA, batched Jacobi, grouped
    KL/apply); the torch-op path below is the CPU plumbing path and the
    fp32 oracle for tests.
  * Subclasses describe their hook tensors twice: `_get_A_factor` /
    `_get_G_factor` (explicit torch math, reference numerics) and
    `_a_sources` / `_g_sources` (implicit patch-matrix descriptors for the
    SYRK kernel, never materialising im2col).
  * Preconditioned gradients, eigendata and packed factors live in flat
    arenas owned by the execution plan (parallel/plan.py); layer tensors are
    views, so bucketed collectives need no per-layer packing.
  * `.grad` is written in place (DDP bucket views stay valid).
  * Worker-assignment attributes start as None (reference defect #17).
"""
import warnings

import torch

from . import utils as lutils
from .. import comm
from ..ops import _lib
from ..ops import factors as factor_ops
from ..ops import eigen as eigen_ops
from ..ops import precond as precond_ops

__all__ = ['KFACLayer']

_INV_KEYS = ('QA', 'QG', 'dA', 'dG', 'dGdA', 'A_inv', 'G_inv')


class KFACLayer(object):
    def __init__(self, module, accumulate_data=True, batch_first=True, inv_dtype=torch.float32,
                 grad_scaler=None, factor_dtype=None, prediv_eigenvalues=True,
                 symmetry_aware_comm=False, use_eigen_decomp=True):
        self.module = module
        self.accumulate_data = accumulate_data
        self.batch_first = batch_first
        self.inv_dtype = inv_dtype if inv_dtype is not None else torch.float32
        self.grad_scaler = grad_scaler
        self.factor_dtype = factor_dtype
        self.prediv_eigenvalues = prediv_eigenvalues
        self.symmetry_aware_comm = symmetry_aware_comm
        self.use_eigen_decomp = use_eigen_decomp
        self.eps = 1e-10

        self.has_bias = False
        self.factors_are_symmetric = True

        self.a_inputs = []
        self.g_outputs = []
        self.state = {'A': None, 'G': None}
        self.preconditioned_gradient = None

        self.compute_A_inv_rank = None
        self.compute_G_inv_rank = None
        self.broadcast_A_inv_group = None
        self.broadcast_G_inv_group = None
        self.compute_grad_ranks = None
        self.broadcast_grad_groups = None
        self.keep_inv_copy = None
        # set by the execution plan: f32 (nG x nA) slice of the gradient arena
        self.pgrad_buffer = None

    def __repr__(self):
        return 'KFAC {}({})'.format(self.__class__.__name__, repr(self.module))

    # ------------------------------------------------------------------ state
    def state_dict(self, include_inverses=False):
        keys = ['A', 'G']
        if include_inverses:
            keys += [k for k in self.state if k in _INV_KEYS]
        out = {}
        for k in keys:
            t = self.state.get(k)
            # arena views would drag the whole arena storage into a checkpoint
            out[k] = t.clone() if (t is not None and t._base is not None) else t
        return out

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        if 'A' not in state_dict or 'G' not in state_dict:
            if 'A_factor' in state_dict and 'G_factor' in state_dict:
                state_dict['A'] = state_dict.pop('A_factor')
                state_dict['G'] = state_dict.pop('G_factor')
            else:
                raise KeyError('KFACLayer state_dict must contain keys "A" and "G"')
        device = next(self.module.parameters()).device
        for key, val in state_dict.items():
            if val is None:
                self.state[key] = None
                continue
            val = val.to(device)
            cur = self.state.get(key)
            if cur is not None and cur.shape == val.shape and cur.dtype == val.dtype:
                cur.copy_(val)      # keep arena aliasing intact
            else:
                self.state[key] = val.clone() if val is state_dict[key] else val

    # ------------------------------------------------------- work assignment
    def assign_inverse_workers(self, compute_A_inv_rank, compute_G_inv_rank,
                               broadcast_A_inv_group, broadcast_G_inv_group):
        if compute_A_inv_rank != compute_G_inv_rank and self.prediv_eigenvalues:
            raise ValueError('When precomputing 1 / (dG * dA.T + damping), A and G inverse '
                             'worker ranks must be equal. I.e. distribute_layer_factors=False.')
        self.compute_A_inv_rank = compute_A_inv_rank
        self.compute_G_inv_rank = compute_G_inv_rank
        self.broadcast_A_inv_group = broadcast_A_inv_group
        self.broadcast_G_inv_group = broadcast_G_inv_group

    def assign_gradient_workers(self, compute_grad_ranks, broadcast_grad_groups):
        if len(broadcast_grad_groups) != comm.backend.size():
            raise ValueError('len(broadcast_grad_groups) != world size')
        self.compute_grad_ranks = list(compute_grad_ranks)
        self.broadcast_grad_groups = broadcast_grad_groups
        self.keep_inv_copy = comm.backend.rank() in self.compute_grad_ranks

    # ---------------------------------------------------- per-layer collectives
    def allreduce_factors(self):
        """Per-layer async all-reduce (the KFAC orchestrator uses the bucketed
        arena path in parallel/collectives.py instead)."""
        if self.factors_are_symmetric and self.symmetry_aware_comm:
            self.state['A_flat'] = lutils.get_triu(self.state['A'])
            self.state['G_flat'] = lutils.get_triu(self.state['G'])
            return [comm.backend.allreduce(self.state['A_flat']),
                    comm.backend.allreduce(self.state['G_flat'])]
        return [comm.backend.allreduce(self.state['A']),
                comm.backend.allreduce(self.state['G'])]

    def broadcast_inverses(self):
        if not self.keep_inv_copy:
            return []
        b = comm.backend
        if self.use_eigen_decomp:
            ops = [b.broadcast(self.state['QA'], src=self.compute_A_inv_rank,
                               group=self.broadcast_A_inv_group),
                   b.broadcast(self.state['QG'], src=self.compute_G_inv_rank,
                               group=self.broadcast_G_inv_group)]
            if self.prediv_eigenvalues:
                ops.append(b.broadcast(self.state['dGdA'], src=self.compute_A_inv_rank,
                                       group=self.broadcast_A_inv_group))
            else:
                ops.append(b.broadcast(self.state['dA'], src=self.compute_A_inv_rank,
                                       group=self.broadcast_A_inv_group))
                ops.append(b.broadcast(self.state['dG'], src=self.compute_G_inv_rank,
                                       group=self.broadcast_G_inv_group))
            return ops
        return [b.broadcast(self.state['A_inv'], src=self.compute_A_inv_rank,
                            group=self.broadcast_A_inv_group),
                b.broadcast(self.state['G_inv'], src=self.compute_G_inv_rank,
                            group=self.broadcast_G_inv_group)]

    def broadcast_gradient(self):
        if self.compute_grad_ranks is None:
            raise ValueError('Gradient compute ranks have not been assigned yet. '
                             'Use assign_workers().')
        buf = self._pgrad_matrix()
        self.preconditioned_gradient = self._split_pgrad(buf)
        src, group = self.broadcast_grad_groups[comm.backend.rank()]
        return [comm.backend.broadcast(buf, src=src, group=group)]

    # ------------------------------------------------------------- inverses
    def _check_assigned(self, which):
        if getattr(self, 'compute_{}_inv_rank'.format(which)) is None:
            raise ValueError('Workers have not been assigned to layer yet.')
        if self.keep_inv_copy is None:
            raise ValueError('Grad workers have not been assigned to layer yet.')
        if self.state[which] is None:
            raise RuntimeError('update_{}_factor() must be called at least once before '
                               'calling compute_{}_inv().'.format(which, which))

    def _ensure_inv_buffers(self, which):
        """Receive buffers on ranks that keep a copy of the eigendata/inverse."""
        if not self.keep_inv_copy:
            return
        F = self.state[which]
        n = F.shape[0]
        dev = F.device
        if self.use_eigen_decomp:
            if self.state.get('Q' + which) is None:
                self.state['Q' + which] = torch.empty(n, n, dtype=self.inv_dtype, device=dev)
            if self.prediv_eigenvalues:
                if self.state.get('dGdA') is None and self.state['A'] is not None \
                        and self.state['G'] is not None:
                    self.state['dGdA'] = torch.empty(self.state['G'].shape[0],
                                                     self.state['A'].shape[0],
                                                     dtype=self.inv_dtype, device=dev)
            elif self.state.get('d' + which) is None:
                self.state['d' + which] = torch.empty(n, dtype=self.inv_dtype, device=dev)
        elif self.state.get(which + '_inv') is None:
            self.state[which + '_inv'] = torch.empty(n, n, dtype=self.inv_dtype, device=dev)

    def _store_result(self, key, value):
        cur = self.state.get(key)
        value = value.to(self.inv_dtype)
        if cur is not None and cur.shape == value.shape:
            cur.copy_(value)
        else:
            self.state[key] = value

    def _unfold_flat(self, which):
        if self.factors_are_symmetric and self.symmetry_aware_comm:
            flat = self.state.pop(which + '_flat', None)
            if flat is not None:
                self.state[which] = lutils.fill_triu(self.state[which].shape, flat)

    def compute_A_inv(self, damping=0.001, ignore_rank=False):
        self._compute_inv('A', damping, ignore_rank)

    def compute_G_inv(self, damping=0.001, ignore_rank=False):
        self._compute_inv('G', damping, ignore_rank)

    def _compute_inv(self, which, damping, ignore_rank):
        self._check_assigned(which)
        self._unfold_flat(which)
        self._ensure_inv_buffers(which)
        owner = getattr(self, 'compute_{}_inv_rank'.format(which))
        if ignore_rank or comm.backend.rank() == owner:
            self.finish_inverse(which, self._compute_factor_inverse(self.state[which], damping),
                                damping)

    def finish_inverse(self, which, result, damping):
        """Store an eigendecomposition (Q, d) or inverse for factor `which`."""
        if isinstance(result, tuple):
            self._store_result('Q' + which, result[0])
            self._store_result('d' + which, result[1])
            if which == 'G' and self.prediv_eigenvalues:
                self._store_outer_reciprocal(damping)
        else:
            self._store_result(which + '_inv', result)

    def _store_outer_reciprocal(self, damping):
        """dGdA = 1 / (dG dA^T + damping) from the stored eigenvalues, in place
        when the buffer exists."""
        if self.state.get('dA') is None:
            raise ValueError('compute_A_inv must be called before compute_G_inv if '
                             'prediv_eigenvalues is True.')
        cur = self.state.get('dGdA')
        out = cur if (cur is not None and cur.dtype == torch.float32) else None
        self._store_result('dGdA', precond_ops.outer_reciprocal(
            self.state['dG'], self.state['dA'], damping, out=out))

    def _compute_factor_inverse(self, factor, damping=0.001):
        F = factor.to(torch.float32)
        if self.use_eigen_decomp:
            if self.factors_are_symmetric:
                (Q, d), = eigen_ops.symeig_many([F], clip=0.0)
            else:
                Q, d = lutils.get_eigendecomp(F, concat=False, symmetric=False)
            return Q.to(self.inv_dtype), d.to(self.inv_dtype)
        if self.factors_are_symmetric:
            inv, = eigen_ops.inverse_many([F], damping)
        else:
            inv = lutils.get_inverse(F, damping=damping, symmetric=False)
        return inv.to(self.inv_dtype)

    # -------------------------------------------------------- preconditioning
    # The parameters whose .grad K-FAC reads and rewrites: the module's own, or
    # fp32 masters of bf16-stored weights (KFAC.set_grad_params, ops/mixed.py)
    grad_weight_param = None
    grad_bias_param = None

    def _wparam(self):
        return self.grad_weight_param if self.grad_weight_param is not None else self.module.weight

    def _bparam(self):
        return self.grad_bias_param if self.grad_bias_param is not None else self.module.bias

    def _get_weight_grad(self):
        return self._wparam().grad

    def _get_bias_grad(self):
        return self._bparam().grad

    def _set_weight_grad(self, grad):
        prm = self._wparam()
        g = prm.grad
        if g is not None and g.shape == grad.shape:
            g.copy_(grad)
        else:
            prm.grad = grad.contiguous()

    def _set_bias_grad(self, grad):
        prm = self._bparam()
        g = prm.grad
        if g is not None and g.shape == grad.shape:
            g.copy_(grad)
        else:
            prm.grad = grad.contiguous()

    def weight_grad_2d(self):
        g = self._get_weight_grad()
        return g.reshape(g.shape[0], -1)

    def get_gradient(self):
        """[out, in(*kh*kw)] gradient with the bias as the last column."""
        g = self.weight_grad_2d()
        if self.has_bias:
            g = torch.cat([g, self._get_bias_grad().reshape(-1, 1)], 1)
        return g

    @property
    def grad_shape(self):
        """(nG, nA) of the preconditioned gradient matrix."""
        w = self.module.weight
        cols = w[0].numel() + (1 if self.has_bias else 0)
        return (w.shape[0], cols)

    def _pgrad_matrix(self):
        if self.pgrad_buffer is None:
            nG, nA = self.grad_shape
            self.pgrad_buffer = torch.zeros(nG, nA, dtype=torch.float32,
                                            device=self.module.weight.device)
        return self.pgrad_buffer

    def _split_pgrad(self, buf):
        w = self.module.weight
        if self.has_bias:
            return [buf[:, :-1].view(w.shape), buf[:, -1:].view(self.module.bias.shape)]
        return [buf.view(w.shape)]

    def grad_pairs(self):
        """[(v 2-D view, .grad tensor)] for the grouped KL-dot / apply kernels.

        The .grad keeps its own memory layout (e.g. channels_last conv weights);
        the kernels map K-FAC column (c, kh, kw) onto its strides."""
        buf = self._pgrad_matrix()
        g = self._get_weight_grad()
        if g is None:
            raise RuntimeError('{} has no gradient; K-FAC needs every registered layer to '
                               'take part in backward'.format(self))
        if self.has_bias:
            return [(buf[:, :-1], g), (buf[:, -1:], self._get_bias_grad())]
        return [(buf, g)]

    def compute_preconditioned_gradient(self, damping=0.001):
        if self.compute_grad_ranks is None:
            raise ValueError('Gradient preconditioning workers have not been assigned yet. '
                             'Have you called assign_workers() yet?')
        if comm.backend.rank() not in self.compute_grad_ranks:
            return
        out = self._pgrad_matrix()
        grad = self.get_gradient().to(self.inv_dtype)
        if self.use_eigen_decomp:
            self._unfold_flat('A')
            if self.prediv_eigenvalues:
                precond_ops.precondition_eigen(grad, self.state['QA'], self.state['QG'],
                                               dGdA=self.state['dGdA'], out=out)
            else:
                precond_ops.precondition_eigen(grad, self.state['QA'], self.state['QG'],
                                               dA=self.state['dA'], dG=self.state['dG'],
                                               damping=damping, out=out)
        else:
            if self.factors_are_symmetric and self.symmetry_aware_comm:
                for which in ('A', 'G'):
                    inv = self.state[which + '_inv']
                    if inv.dim() == 1:
                        self.state[which + '_inv'] = lutils.fill_triu(self.state[which].shape,
                                                                      inv)
            precond_ops.precondition_inverse(grad, self.state['A_inv'], self.state['G_inv'],
                                             out=out)
        self.preconditioned_gradient = self._split_pgrad(out)

    def update_gradient(self, scale=None):
        if self.preconditioned_gradient is None:
            raise RuntimeError('self.compute_preconditioned_gradient() should be called '
                               'before update_gradient()')
        v = self.preconditioned_gradient
        if scale is not None:
            v = [scale * x for x in v]
        self._set_weight_grad(v[0])
        if self.has_bias:
            self._set_bias_grad(v[1])

    # ----------------------------------------------------------- hook data
    def save_inputs(self, input):
        x = input[0].detach()
        if self.accumulate_data:
            self.a_inputs.append(x)
        else:
            self.a_inputs = [x]

    def save_grad_outputs(self, grad_output):
        g = grad_output[0].detach()
        if self.grad_scaler is not None:
            # the loss scale as a DEVICE tensor (get_scale() is a host read that
            # breaks hipGraph capture); a copy, update() may change it later
            if g.is_cuda and hasattr(self.grad_scaler, '_get_scale_async') and \
                    self.grad_scaler._get_scale_async() is not None:
                sc = self.grad_scaler._get_scale_async().detach().reshape(1).float().clone()
            else:
                sc = self.grad_scaler.get_scale()
            g = (g, sc)
        if self.accumulate_data:
            self.g_outputs.append(g)
        else:
            self.g_outputs = [g]

    def _factor_out_dtype(self, x):
        return self.factor_dtype if self.factor_dtype is not None else x.dtype

    def take_factor_job(self, which):
        """Consume the saved hook data of factor `which` ('A' or 'G') and
        return (sources, out_dtype, keep) for the GPU factor kernels, or None
        when there is nothing to add.  G applies the AMP unscale / non-finite
        filter of the reference (base.py:392-417) ON THE DEVICE: each source's
        scale gets a device factor finite(g) / s^2 (0 drops an overflowed
        source without a host read) and `keep` (any source finite) leaves the
        factor untouched when none is -- graph-capturable under GradScaler."""
        if which == 'A':
            if len(self.a_inputs) == 0:
                return None
            inputs, self.a_inputs = self.a_inputs, []
            return self._a_sources(inputs), self._factor_out_dtype(inputs[0]), None
        outputs, self.g_outputs = self.g_outputs, []
        if not outputs:
            return None
        if self.grad_scaler is None:
            return self._g_sources(outputs), self._factor_out_dtype(outputs[0]), None
        gs = [g for g, _ in outputs]
        srcs = self._g_sources(gs)
        keep = None
        fins = []
        for s, (g, sc) in zip(srcs, outputs):
            fin = torch.isfinite(g).all().reshape(1)
            sc = sc if torch.is_tensor(sc) else torch.full((1,), float(sc), device=g.device)
            s.dscale = torch.where(fin, 1.0 / (sc * sc), torch.zeros_like(sc))
            keep = fin if keep is None else (keep | fin)
            fins.append(fin)
        rows = [self._g_rows(g) for g in gs]
        if len(gs) > 1 and rows[0] is not None:
            # the sources share one 1/total normalisation (all rows); the
            # reference averages over the KEPT rows only, so rescale by
            # total / kept on the device (no host read; 0 kept -> keep = 0)
            total = float(sum(rows))
            kept = sum(f.float() * float(r) for f, r in zip(fins, rows))
            renorm = total / torch.clamp(kept, min=1.0)
            for s in srcs:
                s.dscale = s.dscale * renorm
        return srcs, self._factor_out_dtype(gs[0]), keep.float()

    def _g_rows(self, g):
        """Rows source `g` contributes to the shared normalisation of the G
        factor, or None when every source is normalised on its own."""
        return None

    def _take_g_outputs(self):
        outputs, self.g_outputs = self.g_outputs, []
        if self.grad_scaler is None:
            return outputs, [1.0] * len(outputs)
        kept, unscale = [], []
        for g, s in outputs:     # CPU reference path (host checks are free here)
            if torch.isfinite(g).all():
                kept.append(g)
                unscale.append(float(s))
        if len(kept) != len(outputs):
            warnings.warn('Some gradients were discarded when computing G because they '
                          'were unable to be unscaled. Note this can degrade KFAC '
                          'performance if too many gradients are discarded.')
        return kept, unscale

    def update_A_factor(self, alpha=0.95):
        if len(self.a_inputs) == 0:
            return
        if _lib.use_native(self.a_inputs[0]):
            srcs, dtype, _ = self.take_factor_job('A')
            self.state['A'] = factor_ops.update_factor(self.state['A'], srcs, alpha, dtype)
            return
        inputs, self.a_inputs = self.a_inputs, []
        if self.factor_dtype is not None:
            inputs = [x.to(self.factor_dtype) for x in inputs]
        A_new = self._get_A_factor(inputs)
        if self.state['A'] is None:
            self.state['A'] = torch.eye(A_new.shape[0], dtype=A_new.dtype, device=A_new.device)
        lutils.update_running_avg(A_new, self.state['A'], alpha=alpha)

    def update_G_factor(self, alpha=0.95):
        if len(self.g_outputs) == 0:
            return
        first = self.g_outputs[0]
        if _lib.use_native(first[0] if isinstance(first, tuple) else first):
            job = self.take_factor_job('G')
            if job is not None:
                self.state['G'] = factor_ops.update_factor(self.state['G'], job[0], alpha, job[1],
                                                           keep=job[2])
            return
        kept, unscale = self._take_g_outputs()
        if len(kept) == 0:
            return
        if self.factor_dtype is not None:
            kept = [g.to(self.factor_dtype) for g in kept]
        if self.grad_scaler is not None:
            kept = [g / u for g, u in zip(kept, unscale)]
        G_new = self._get_G_factor(kept)
        if self.state['G'] is None:
            self.state['G'] = torch.eye(G_new.shape[0], dtype=G_new.dtype, device=G_new.device)
        lutils.update_running_avg(G_new, self.state['G'], alpha=alpha)

    # ----------------------------------------------------- subclass contract
    def _get_A_factor(self, a_inputs):
        raise NotImplementedError

    def _get_G_factor(self, g_outputs):
        raise NotImplementedError

    def _a_sources(self, a_inputs):
        raise NotImplementedError

    def _g_sources(self, g_outputs):
        raise NotImplementedError
