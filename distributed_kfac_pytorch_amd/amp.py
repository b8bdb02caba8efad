"""A GradScaler whose unscale / step / update can be captured in a hipGraph.

torch.amp.GradScaler.step() reads `found_inf` on the host to decide whether to
call optimizer.step(), which breaks graph capture (and fused optimizers' own
device-side skip let non-finite updates through on this ROCm build,
scripts/probes/probe_fp16_example.py).  `CapturableGradScaler` keeps every
decision on the device:

  unscale_graphable(opt)  the same `_amp_foreach_non_finite_check_and_unscale_`
                          as GradScaler.unscale_, into a persistent found_inf
  step_graphable(opt)     torch.optim.SGD's foreach update computed into
                          temporaries, then SELECTED (torch.where -- a 0 * inf
                          mask would propagate NaN) against the old parameters
                          and momentum buffers: an overflowed step leaves both
                          untouched, exactly like GradScaler's skipped step
  update_graphable()      `_amp_update_scale_` with that found_inf

The arithmetic is op for op the eager GradScaler + SGD (foreach) sequence, so
a replayed step equals the eager one bitwise (tests/test_amp.py on the CPU,
tests/test_gpu_examples.py graphed vs eager on the GPU).  It IS a GradScaler:
the eager loop's scale() / unscale_() / step() / update() and K-FAC's device
loss-scale reads (layers/base.py save_grad_outputs) share its state.
Reference: examples/cnn_utils/engine.py:73-82 (fp16 + GradScaler).
"""
import torch

__all__ = ['CapturableGradScaler']


class CapturableGradScaler(torch.amp.GradScaler):

    def __init__(self, device='cuda', **kw):
        super().__init__(device, **kw)
        self._found_inf_graph = None

    def _found(self, ref):
        if self._found_inf_graph is None or self._found_inf_graph.device != ref.device:
            self._found_inf_graph = torch.zeros((), dtype=torch.float32, device=ref.device)
        return self._found_inf_graph

    @staticmethod
    def _grads(optimizer):
        out = []
        for g in optimizer.param_groups:
            for p in g['params']:
                if p.grad is not None:
                    out.append(p.grad)
        return out

    def unscale_graphable(self, optimizer):
        """Unscale every gradient in place; overflow -> found_inf = 1 (device)."""
        if not self._enabled:
            return
        if self._scale is None:
            raise RuntimeError('scale() must run (eagerly) before unscale_graphable()')
        found = self._found(self._scale)
        found.zero_()
        inv_scale = self._scale.double().reciprocal().float()
        groups = {}
        for g in self._grads(optimizer):
            if g.is_sparse:
                raise RuntimeError('CapturableGradScaler: sparse gradients are not supported')
            groups.setdefault((g.device, g.dtype), []).append(g)
        for grads in groups.values():
            torch._amp_foreach_non_finite_check_and_unscale_(grads, found, inv_scale)

    @torch.no_grad()
    def step_graphable(self, optimizer):
        """torch.optim.SGD.step() (foreach), skipped on the device when the
        unscale found an overflow.  Momentum buffers are created (zeros) if
        missing: m * 0 + g equals SGD's first-step clone(g)."""
        if not isinstance(optimizer, torch.optim.SGD):
            raise TypeError('CapturableGradScaler.step_graphable supports torch.optim.SGD')
        if not self._enabled:
            optimizer.step()
            return
        skip = self._found(self._scale) > 0
        for group in optimizer.param_groups:
            if group.get('maximize', False):
                raise ValueError('maximize=True is not supported')
            params = [p for p in group['params'] if p.grad is not None]
            if not params:
                continue
            grads = [p.grad for p in params]
            lr, momentum = group['lr'], group['momentum']
            wd, damp, nesterov = group['weight_decay'], group['dampening'], group['nesterov']
            if damp != 0 and momentum != 0:
                # torch.optim.SGD's first step clones g into a fresh buffer and
                # ignores dampening; a zero buffer here would give (1 - d) g
                raise ValueError('step_graphable: dampening != 0 is not supported '
                                 '(SGD applies it only after the first step)')
            if wd != 0:
                grads = torch._foreach_add(grads, params, alpha=wd)
            bufs = None
            if momentum != 0:
                bufs = []
                for p in params:
                    st = optimizer.state[p]
                    if st.get('momentum_buffer') is None:
                        st['momentum_buffer'] = torch.zeros_like(p)
                    bufs.append(st['momentum_buffer'])
                new_bufs = torch._foreach_mul(bufs, momentum)
                torch._foreach_add_(new_bufs, grads, alpha=1 - damp)
                if nesterov:
                    grads = torch._foreach_add(grads, new_bufs, alpha=momentum)
                else:
                    grads = new_bufs
            new_params = torch._foreach_add(params, grads, alpha=-lr)
            for i, p in enumerate(params):
                p.copy_(torch.where(skip, p, new_params[i]))
                if bufs is not None:
                    bufs[i].copy_(torch.where(skip, bufs[i], new_bufs[i]))

    def update_graphable(self):
        """GradScaler.update() on the found_inf of unscale_graphable()."""
        if not self._enabled:
            return
        torch._amp_update_scale_(self._scale, self._growth_tracker, self._found(self._scale),
                                 self._growth_factor, self._backoff_factor,
                                 self._growth_interval)
