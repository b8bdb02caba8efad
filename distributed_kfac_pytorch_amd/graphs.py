"""Whole-training-step hipGraph capture for K-FAC training loops.

On MI355X a ResNet-50 step at per-GPU batch 32 is host-launch bound when run
eagerly: ~14 ms of Python/ATen dispatch for ~9 ms of GPU work
(profiles/r1_graph_step_probe.log).  `GraphedTrainStep` captures the step --
forward, backward, K-FAC factor SYRKs, the fused preconditioning chain, the
device-side KL clip and the optimizer update -- into hipGraphs and replays
them, one graph per *step kind* (the MI355X replacement for a tracing
compiler):

  'plain'   no factor update, no inverse update       -> replayed graph(s)
  'factor'  factor update (hooks + SYRK + EMA)         -> replayed graph(s)
  'eager'   inverse-update steps (eigensolver launch sequences, eigendata
            broadcast) and the very first steps        -> the update runs
            eagerly; once the factor-step forward/backward graphs exist an
            inverse step replays them (it is a factor step too) and only
            the update is eager.  A single-segment trainer given
            `forward_backward` and `update` as well replays a forward/backward
            graph of its own on inverse steps (factors inside the captured
            hooks, KFAC.hook_factors) instead of running them eagerly

Two modes:
  single-segment  `step_fn` does everything (one process): one graph per kind.
  segmented       `forward_backward`, `communicate`, `update`: the forward +
                  backward segment is a graph per kind; `communicate` (the
                  data-parallel gradient all-reduce, parallel/grad_sync.py)
                  runs eagerly between replays -- no collective is ever
                  captured.  `forward_backward` / `communicate` may be equal-
                  length LISTS (a backward split into segments,
                  parallel/overlap.py): segment i's graph replays, then
                  communicate[i] issues its (async) collective, which runs
                  while segment i+1 replays; the first segment returns the
                  loss.  `update` (preconditioner.step() + optimizer.step())
                  is a graph when it issues no collective for that kind: one
                  rank, or COMM_OPT plain and factor steps -- at a factor step
                  the K-FAC factor all-reduce is issued eagerly first
                  (KFAC.step_factor_comm: pack + async RCCL all-reduce on the
                  K-FAC communicator) and joined at the next factor step,
                  before its forward/backward graph replays
                  (KFAC.prepare_factor_step), so the captured update holds no
                  collective.  With
                  `phased_update=True` (update == preconditioner.step() +
                  optimizer.step()), a plain or factor step that does
                  communicate (MEM_OPT / HYBRID_OPT gradient all-gather; a
                  factor step's factor all-reduce is issued eagerly first, as
                  above) runs as two graphs -- KFAC.step_precondition, then
                  KFAC.step_finish + optimizer.step() -- with
                  KFAC.step_communicate eager between them; only inverse
                  steps with collectives (eigendata all-gather) stay eager.

Step kinds follow the K-FAC schedule (`factor_update_freq`, `inv_update_freq`,
reference kfac/preconditioner.py:494-514); the K-FAC step counter that a graph
cannot advance is advanced here.  Python-level hyper-parameters baked into a
graph (learning rates, damping, KL clip, frequencies) are part of the graph
key, so a scheduler that changes them triggers a re-capture, never a stale
replay.

Contract: inputs are read from tensors whose storage does not change between
calls (copy each batch into them); `optimizer.zero_grad()` with either
`set_to_none` (True lets each graph's backward produce fresh .grad tensors from
its private pool; the K-FAC tail graph keys on the grad pointers); the step
returns a tensor (the loss).  Eager
fallback: `enabled=False`, no GPU, or an exception during capture (warned once).

Every graph is captured with keep_graph=True and its memset nodes are rewritten
into fill kernels before instantiation (ops/_lib.finalize_graph,
csrc/graph_fix.hip): on this ROCm runtime a captured memset node does not
reliably clear its target on replay, and MIOpen zeroes the accumulation
workspace of ResNet-50's channels_last weight-gradient convolutions that way --
replayed steps picked up whatever the previous user of that memory left
(NaN / 1e30 gradients in layer2.0.conv1, found in round 1).
Eager steps and replays run on one side stream, joined to the caller's
stream by events; the device is synchronised once after each eager
(inverse-update) step, which also drains the eigensolver's worker streams.
"""
import contextlib
import gc
import warnings

import torch

from .ops import _lib

__all__ = ['GraphedTrainStep']


def _world_size():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


class GraphedTrainStep(object):
    def __init__(self, step_fn=None, preconditioner=None, optimizers=(), warmup=2, enabled=True,
                 forward_backward=None, communicate=None, update=None, phased_update=False,
                 stream=None, post_update=None):
        if step_fn is None and (forward_backward is None or update is None):
            raise ValueError('give step_fn, or forward_backward and update')
        self.step_fn = step_fn
        if isinstance(forward_backward, (list, tuple)):
            comms = list(communicate) if isinstance(communicate, (list, tuple)) else \
                [None] * (len(forward_backward) - 1) + [communicate]
            if len(comms) != len(forward_backward):
                raise ValueError('communicate must match forward_backward segment by segment')
            self.fbs, self.comms = list(forward_backward), comms
        else:
            self.fbs, self.comms = [forward_backward], [communicate]
        self.fb, self.comm, self.update = forward_backward, communicate, update
        # phased updates run KFAC.step_finish + the optimizers themselves (not
        # `update`): `post_update` is what `update` does after the optimizer
        # (e.g. ops/mixed.BF16Weights.master_to_model)
        self.post_update = post_update
        self.segmented = step_fn is None
        # single-segment trainer that also names its forward/backward and
        # update: inverse steps replay an 'invfb' graph + the eager update
        self.hybrid = (not self.segmented and forward_backward is not None
                       and update is not None and preconditioner is not None
                       and not isinstance(forward_backward, (list, tuple))
                       and hasattr(preconditioner, 'hook_factors'))
        self.pre = preconditioner
        if self.segmented and preconditioner is not None:
            # no side-stream fork may span the fb / update graph boundary
            preconditioner._segmented_capture = True
        # 'force' phases the update even when it issues no collective (tests)
        self.phased_update = phased_update
        # inverse-update steps replay the factor-step forward/backward graph(s)
        self.graph_inverse_fb = True
        if preconditioner is not None and enabled:
            # the whole step is graphed: KFAC's own precondition-tail graph
            # is redundant
            preconditioner.use_hip_graphs = False
        if self.segmented and preconditioner is not None and \
                not preconditioner.compute_factor_in_hook:
            # a replayed forward/backward graph runs no Python hooks, so the
            # factors must be computed INSIDE the captured hooks
            raise ValueError('segmented GraphedTrainStep needs '
                             'KFAC(compute_factor_in_hook=True)')
        self.optimizers = list(optimizers) if isinstance(optimizers, (list, tuple)) \
            else [optimizers]
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        if self.enabled and not self.segmented and _world_size() > 1:
            # a single-segment capture would record the step's collectives (the
            # DDP reducer's all-reduce, K-FAC's factor / eigendata / gradient
            # communication); a capture that failed on only some ranks would
            # leave them running mismatched collectives.  Multi-rank steps
            # use the segmented mode (collectives between graph replays).
            warnings.warn('GraphedTrainStep: single-segment capture is disabled at world size '
                          '> 1; use the segmented mode (forward_backward / communicate / '
                          'update)')
            self.enabled = False
        self.graphs = {}
        self.outputs = {}
        self._warm = {}
        self.replays = 0
        self.eager_steps = 0
        self._plan_gen = None
        # warm-up and capture share one side stream, so the autograd
        # AccumulateGrad nodes created in warm-up live on the capture stream
        # (`stream`: reuse another GraphedTrainStep's, for the same model)
        self.side = (stream or torch.cuda.Stream()) if self.enabled else None

    # ------------------------------------------------------------ schedule
    def _kind(self):
        pre = self.pre
        if pre is None:
            return 'plain'
        p = pre.param_groups[0]
        if not pre.workers_assigned or p['step'] % p['inv_update_freq'] == 0:
            return 'eager'
        if getattr(pre, 'inverse_apply_due', None) is not None and pre.inverse_apply_due():
            return 'eager'    # a lagged inverse update is stored this step (host work)
        if p['step'] % p['factor_update_freq'] == 0:
            return 'factor'
        return 'plain'

    def _key(self, seg, kind):
        hp = []
        for opt in self.optimizers:
            for g in opt.param_groups:
                hp.append(tuple(sorted((k, v) for k, v in g.items()
                                       if isinstance(v, (int, float, bool)))))
        if self.pre is not None:
            p = self.pre.param_groups[0]
            hp.append((p['lr'], p['damping'], p['kl_clip'], p['factor_decay'],
                       p['factor_update_freq'], p['inv_update_freq'],
                       # a rebuilt execution plan moves every buffer a graph addresses
                       getattr(self.pre, 'plan_generation', 0)))
        return (seg, kind, tuple(hp))

    def _advance(self):
        if self.pre is not None:
            self.pre.param_groups[0]['step'] += 1

    def _update_capturable(self, kind):
        """update = preconditioner.step() + optimizer.step(): capturable when
        it issues no collective (one rank, or COMM_OPT plain steps)."""
        pre = self.pre
        if pre is None:
            return True
        if getattr(pre, 'comm_check', False):
            # the consistency checks join collectives and read checksums on
            # the host: never inside a capture (KFAC_COMM_CHECK=1 debug runs)
            return False
        from . import comm
        if comm.backend is None or comm.backend.size() == 1:
            return True
        from .preconditioner import CommMethod
        return kind in ('plain', 'factor') and pre.comm_method == CommMethod.COMM_OPT

    # ------------------------------------------------------------ execution
    def _inverse_fb_graphed(self):
        """An inverse-update step is also a factor step: its forward/backward
        (factor SYRK + EMA inside the captured hooks) can replay the 'factor'
        fb graph(s); only the update (eigensolves, eigendata distribution,
        preconditioning, optimizer) then runs eagerly.  Needs every factor fb
        segment captured already, workers assigned and no lagged solve due."""
        pre = self.pre
        if not (self.graph_inverse_fb and (self.segmented or self.hybrid) and pre is not None
                and pre.workers_assigned):
            return False
        p = pre.param_groups[0]
        if p['step'] % p['factor_update_freq'] != 0:
            return False
        if getattr(pre, 'inverse_apply_due', None) is not None and pre.inverse_apply_due():
            return False
        if self.hybrid:
            return True      # its own 'invfb' graph: warmed up / captured on the way
        return all(self._key('fb' if i == 0 else 'fb%d' % i, 'factor') in self.graphs
                   for i in range(len(self.fbs)))

    def _prepare_factor(self):
        # a factor step's captured hooks run the EMA on the averaged factors:
        # join the previous factor step's deferred all-reduce first
        if self.pre is not None and hasattr(self.pre, 'prepare_factor_step'):
            self.pre.prepare_factor_step()

    def _issue_factor_comm(self, kind):
        # multi-rank factor step: issue the factor all-reduce eagerly so the
        # update segment holds no collective (KFAC.step_factor_comm)
        if kind == 'factor' and self.pre is not None and hasattr(self.pre, 'step_factor_comm'):
            self.pre.step_factor_comm()

    def _purge_stale_plans(self):
        """A re-plan (KFAC._assign_workers) moved every buffer the captured
        graphs address: drop graphs of older plan generations (their keys can
        never match again) so their memory pools are released."""
        gen = getattr(self.pre, 'plan_generation', 0) if self.pre is not None else 0
        if gen == self._plan_gen:
            return
        self._plan_gen = gen
        for d in (self.graphs, self.outputs, self._warm):
            for k in [k for k in d if k[2] and k[2][-1][-1] != gen]:
                del d[k]

    def _join_side_streams(self):
        """After an eager step: order the current stream after every side
        stream the step used (this trainer's update stream, K-FAC's factor /
        fused-chain / eigensolver streams) with device-side event waits, so the
        next replay cannot overtake them.  No host sync: a full
        torch.cuda.synchronize() would also drain a deferred factor all-reduce
        and a lagged inverse update that are meant to keep running."""
        cur = torch.cuda.current_stream()
        streams = [self.side] if self.side is not None else []
        if self.pre is not None and hasattr(self.pre, 'side_streams'):
            streams += self.pre.side_streams()
        for s in streams:
            if s is not None and s != cur:
                cur.wait_stream(s)

    def __call__(self):
        self._purge_stale_plans()
        kind = self._kind()
        if self.enabled and kind == 'eager' and self._inverse_fb_graphed():
            self.eager_steps += 1
            self._prepare_factor()
            with (self.pre.hook_factors() if self.hybrid else contextlib.nullcontext()):
                # early inverse update (KFAC.arm_early_inverse): this
                # forward/backward runs EAGERLY and its first gradient hook
                # launches the leading eigensolve group under the rest of the
                # backward (a replayed graph would hold it to the graph's end)
                early = self.hybrid and hasattr(self.pre, 'arm_early_inverse') and \
                    self.pre.arm_early_inverse()
                loss = None
                for i, (fb, cm) in enumerate(zip(self.fbs, self.comms)):
                    if early:
                        out = self._run_eager(fb)
                    else:
                        seg = 'invfb' if self.hybrid else ('fb' if i == 0 else 'fb%d' % i)
                        out = self._run_segment(seg, 'factor', fb, advances=False)
                    if i == 0:
                        loss = out
                    if cm is not None:
                        cm()
                if early:
                    self.pre.disarm_early_inverse()
                cur = torch.cuda.current_stream()
                self.side.wait_stream(cur)
                with torch.cuda.stream(self.side):
                    self.update()
                cur.wait_stream(self.side)
            self._join_side_streams()
            return loss
        if not self.enabled or kind == 'eager':
            self.eager_steps += 1
            out = self._eager()
            if self.enabled:
                self._join_side_streams()
            return out
        if kind == 'factor':
            self._prepare_factor()
        if not self.segmented:
            return self._run_segment('step', kind, self.step_fn, advances=True)
        loss = None
        for i, (fb, cm) in enumerate(zip(self.fbs, self.comms)):
            out = self._run_segment('fb' if i == 0 else 'fb%d' % i, kind, fb, advances=False)
            if i == 0:
                loss = out
            if cm is not None:
                cm()
        self._issue_factor_comm(kind)
        if self.phased_update and kind in ('plain', 'factor') and self.pre is not None and \
                (self.phased_update == 'force' or not self._update_capturable(kind)):
            self._run_segment('upd_pre', kind, self.pre.step_precondition, advances=False)
            self.pre.step_communicate()
            self._run_segment('upd_post', kind, self._finish, advances=True)
        elif self._update_capturable(kind):
            self._run_segment('update', kind, self.update, advances=True)
        else:
            self.update()
        return loss

    def _finish(self):
        self.pre.step_finish()
        for opt in self.optimizers:
            opt.step()
        if self.post_update is not None:
            self.post_update()

    def _eager(self):
        if not self.enabled:
            return self._eager_body()
        # eager steps run on the capture stream too: every AccumulateGrad node
        # (created once per parameter and kept alive across steps, e.g. by
        # K-FAC's saved activations) then belongs to that stream, and no
        # capture records a cross-stream dependency on the legacy stream
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            out = self._eager_body()
        cur.wait_stream(self.side)
        return out

    def _run_eager(self, fn):
        """One segment eagerly on the capture stream (as a warm-up run)."""
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            out = fn()
        cur.wait_stream(self.side)
        return out

    def _eager_body(self):
        if not self.segmented:
            return self.step_fn()
        loss = None
        for i, (fb, cm) in enumerate(zip(self.fbs, self.comms)):
            out = fb()
            if i == 0:
                loss = out
            if cm is not None:
                cm()
        self.update()
        return loss

    def _run_segment(self, seg, kind, fn, advances):
        key = self._key(seg, kind)
        g = self.graphs.get(key)
        if g is not None:
            self._replay(g)
            if advances:
                self._advance()
            self.replays += 1
            return self.outputs[key]
        if self._warm.get(key, 0) < self.warmup:
            self._warm[key] = self._warm.get(key, 0) + 1
            cur = torch.cuda.current_stream()
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                out = fn()
            cur.wait_stream(self.side)
            return out
        return self._capture(key, fn, advances)

    def _replay(self, g):
        """Replay on the capture stream, joined to the caller's stream by events."""
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            g.replay()
        cur.wait_stream(self.side)

    def _capture(self, key, fn, advances):
        step0 = self.pre.param_groups[0]['step'] if self.pre is not None else None
        if self.pre is not None and hasattr(self.pre, 'wait_inverses'):
            self.pre.wait_inverses()   # no solver-thread library calls during a capture
        torch.cuda.synchronize()
        g = _lib.new_graph()
        # no Python garbage collection inside the capture: a collected cycle
        # holding a HIP event or graph destroys it mid-capture (an illegal
        # call under global capture mode -> abort from the destructor; seen
        # with the LSTM LM's many per-time-step objects)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            # a private memory pool per graph: segments and kinds replay in
            # any order, so one graph's outputs must never alias another's
            # temporaries
            with torch.cuda.graph(g, stream=self.side):
                out = fn()
            # memset nodes (MIOpen's zeroed workspaces) -> fill kernels
            _lib.finalize_graph(g)
        except Exception as e:  # pragma: no cover - depends on the HIP runtime
            if gc_on:
                gc.enable()
            warnings.warn('hipGraph capture of the training step failed ({}); running '
                          'eagerly from now on'.format(e))
            self.enabled = False
            if self.pre is not None:
                self.pre.param_groups[0]['step'] = step0
            return fn()
        if gc_on:
            gc.enable()
        if self.pre is not None:
            # capture recorded the work without running it; a captured
            # preconditioner.step() advanced the step counter: rewind
            self.pre.param_groups[0]['step'] = step0
        self.graphs[key] = g
        self.outputs[key] = out
        self._replay(g)
        if advances:
            self._advance()
        self.replays += 1
        return out

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
        if self.hybrid and self.pre.inverse_lag == 0:
            # the inverse steps' forward/backward graph too (real inverse
            # updates: each runs the eigensolver once)
            for _ in range(self.warmup + 1):
                p['step'] = 0
                self()
        p['step'] = saved
