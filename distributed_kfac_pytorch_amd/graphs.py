"""Whole-training-step hipGraph capture for K-FAC training loops.

On MI355X a ResNet-50 step at per-GPU batch 32 is host-launch bound when run
eagerly: ~14 ms of Python/ATen dispatch for ~9 ms of GPU work
(profiles/r1_graph_step_probe.log).  `GraphedTrainStep` captures the whole
step -- forward, backward, K-FAC factor SYRKs, the fused preconditioning
chain, the device-side KL clip and the optimizer update -- into hipGraphs and
replays them, one graph per *step kind* (this is the MI355X replacement for a
tracing compiler):

  'plain'   no factor update, no inverse update       -> replayed graph
  'factor'  factor update (hooks + SYRK + EMA)         -> replayed graph
  'eager'   inverse-update steps (rocSOLVER D&C with host-side work, eigendata
            broadcast) and the very first steps        -> run eagerly

Step kinds follow the K-FAC schedule (`factor_update_freq`, `inv_update_freq`,
reference kfac/preconditioner.py:494-514); the K-FAC step counter that the
graph cannot advance is advanced here.  Python-level hyper-parameters baked
into a graph (learning rates, damping, KL clip, frequencies) form the graph
key, so a scheduler that changes them triggers a re-capture instead of a stale
replay.

Contract for `step_fn`: it reads its inputs from tensors whose storage does
not change between calls (copy each batch into them), calls
`optimizer.zero_grad(set_to_none=False)`, runs forward/backward,
`preconditioner.step()` and `optimizer.step()`, and returns a tensor (the
loss).  Eager fallback: `enabled=False`, a CPU device, or an exception during
capture (warned once).
"""
import warnings

import torch

__all__ = ['GraphedTrainStep']


class GraphedTrainStep(object):
    def __init__(self, step_fn, preconditioner=None, optimizers=(), warmup=2, enabled=True):
        self.step_fn = step_fn
        self.pre = preconditioner
        self.optimizers = list(optimizers) if isinstance(optimizers, (list, tuple)) \
            else [optimizers]
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.graphs = {}
        self.outputs = {}
        self._warm = {}
        self.replays = 0
        self.eager_steps = 0
        # warm-up and capture share one side stream, so the autograd
        # AccumulateGrad nodes created in warm-up live on the capture stream
        self.side = torch.cuda.Stream() if self.enabled else None

    def _kind(self):
        pre = self.pre
        if pre is None:
            return 'plain'
        p = pre.param_groups[0]
        if not pre.workers_assigned or p['step'] % p['inv_update_freq'] == 0:
            return 'eager'
        if p['step'] % p['factor_update_freq'] == 0:
            return 'factor'
        return 'plain'

    def _key(self, kind):
        hp = []
        for opt in self.optimizers:
            for g in opt.param_groups:
                hp.append(tuple(sorted((k, v) for k, v in g.items()
                                       if isinstance(v, (int, float, bool)))))
        if self.pre is not None:
            p = self.pre.param_groups[0]
            hp.append((p['lr'], p['damping'], p['kl_clip'], p['factor_decay'],
                       p['factor_update_freq'], p['inv_update_freq']))
        return (kind, tuple(hp))

    def _advance(self):
        if self.pre is not None:
            self.pre.param_groups[0]['step'] += 1

    def __call__(self):
        kind = self._kind()
        if not self.enabled or kind == 'eager':
            self.eager_steps += 1
            return self.step_fn()
        key = self._key(kind)
        g = self.graphs.get(key)
        if g is not None:
            g.replay()
            self._advance()
            self.replays += 1
            return self.outputs[key]
        if self._warm.get(key, 0) < self.warmup:
            self._warm[key] = self._warm.get(key, 0) + 1
            self.eager_steps += 1
            cur = torch.cuda.current_stream()
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                out = self.step_fn()
            cur.wait_stream(self.side)
            return out
        return self._capture(key)

    def prepare(self):
        """Warm up and capture every graphed step kind now (e.g. before a timed
        region), by temporarily moving the K-FAC step counter to a step of each
        kind.  Runs real training steps."""
        if not self.enabled:
            return
        if self.pre is None:
            for _ in range(self.warmup + 1):
                self()
            return
        if not self.pre.workers_assigned:
            self()
        p = self.pre.param_groups[0]
        saved = p['step']
        ff, inv = p['factor_update_freq'], p['inv_update_freq']
        probes = {'plain': None, 'factor': None}
        for s in range(1, 4 * inv + 2):
            if s % inv == 0:
                continue
            kind = 'factor' if s % ff == 0 else 'plain'
            if probes[kind] is None:
                probes[kind] = s
        for kind, s in probes.items():
            if s is None:
                continue
            for _ in range(self.warmup + 1):
                p['step'] = s
                self()
        p['step'] = saved

    def _capture(self, key):
        step0 = self.pre.param_groups[0]['step'] if self.pre is not None else None
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            # a private memory pool per graph: step kinds replay in any order,
            # so one graph's outputs must never alias another's temporaries
            with torch.cuda.graph(g, stream=self.side):
                out = self.step_fn()
        except Exception as e:  # pragma: no cover - depends on the HIP runtime
            warnings.warn('hipGraph capture of the training step failed ({}); running '
                          'eagerly from now on'.format(e))
            self.enabled = False
            if self.pre is not None:
                self.pre.param_groups[0]['step'] = step0
            return self.step_fn()
        if self.pre is not None:
            # capture recorded the work without running it; the step counter
            # was advanced by the captured preconditioner.step(): rewind
            self.pre.param_groups[0]['step'] = step0
        self.graphs[key] = g
        self.outputs[key] = out
        g.replay()
        self._advance()
        self.replays += 1
        return out
