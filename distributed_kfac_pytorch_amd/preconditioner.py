"""KFAC: distributed K-FAC gradient preconditioner (public orchestrator).

Drop-in for the reference `kfac.KFAC` (kfac/preconditioner.py:39-735): same
constructor contract, same `param_groups[0]` keys so
LambdaLR / KFACParamScheduler drive it, same state_dict layout, same
COMM_OPT / MEM_OPT / HYBRID_OPT semantics and LPT worker goldens.  Usage:

    preconditioner = KFAC(model, ...)
    loss.backward()                 # DDP has averaged the gradients
    preconditioner.step()           # rewrites .grad in place
    optimizer.step()

MI355X-first internals:
  * factors:   one implicit-im2col MFMA SYRK + fused EMA per factor (ops/factors.py)
  * comm:      triu-packed bucketed factor all-reduce, one broadcast per owner
               for eigendata, one per block for gradients (parallel/collectives.py)
  * inverses:  every owned factor of the step in one batched call (small factors
               in ONE Jacobi launch; ops/eigen.py)
  * KL clip:   one grouped dot kernel + one grouped apply kernel, scale kept on
               the device (no host sync in step())
  * hooks:     forward hook + tensor hook on the module output (no module
               full-backward-hook wrapping).

Reference defects fixed: #3 prediv with
distribute_layer_factors auto-coallocates with a warning instead of raising at
world > 1; #4 HYBRID validation uses max(1, round(W*f)); #7 group averaging;
#11 register_shared_module forwards every layer kwarg; #16 device KL scale;
#17 unassigned ranks start as None.
"""
import contextlib
import enum
import functools
import gc
import warnings

import torch
import torch.optim as optim

from . import comm
from . import layers as kfac_layers
from .ops import _lib
from .ops import precond as precond_ops
from .ops import eigen as eigen_ops
from .ops import precond_fused
from .ops import factors as factor_ops
from .parallel.plan import ExecutionPlan
from .parallel import collectives
from .utils import distribution
from .utils.tracing import PhaseTimer
from .utils import comm_check

__all__ = ['CommMethod', 'KFAC']

# KFAC_DEBUG_EIG=1: host-check every eigendecomposition of an inverse step
# (finite results, residual) -- a debugging aid, syncs the device
_DEBUG_EIG = bool(int(__import__('os').environ.get('KFAC_DEBUG_EIG', '0')))


def _debug_check_eig(jobs, mats, results):
    for (layer, which), A, (Q, d) in zip(jobs, mats, results):
        fin = bool(torch.isfinite(Q).all()) and bool(torch.isfinite(d).all())
        A64 = A.double()
        res = float((A64 @ Q.double() - Q.double() * d.double()).norm() / A64.norm()) \
            if fin else float('nan')
        if not fin or res > 1e-4:
            print('KFAC_DEBUG_EIG: {} {} n={} finite={} input_finite={} resid={:.2e}'.format(
                layer, which, A.shape[0], fin, bool(torch.isfinite(A).all()), res), flush=True)


def _factors_finite(mats):
    """Device flags, one per factor: finite (one multi-tensor norm, no host
    read).  An inverse update over NaN factors once ended in an
    illegal-address GPU fault instead of an error (the solvers' data-dependent
    deflation / iteration logic is not NaN-safe): a flagged factor reaches the
    solvers as the identity (eigen.sanitize) and _raise_nonfinite raises after
    the step's work is enqueued."""
    return torch.isfinite(torch.stack(torch._foreach_norm(mats, 1)))


def _raise_nonfinite(jobs, ok):
    if bool(ok.all()):
        return
    bad = ['{} {}'.format(l, w) for (l, w), f in zip(jobs, ok.tolist()) if not f]
    raise FloatingPointError('non-finite K-FAC factor(s) at an inverse update: {}'.format(
        ', '.join(bad[:8])))


def _check_factors_finite(jobs, mats):
    """Raise on a non-finite factor now (one host read)."""
    if mats:
        _raise_nonfinite(jobs, _factors_finite(mats))


class CommMethod(enum.Enum):
    """How preconditioning work and eigendata are distributed.

    COMM_OPT:   every rank receives all eigendata and preconditions every layer
                ('KFAC_opt', arXiv:2007.00784).
    MEM_OPT:    the owner of a layer preconditions it and broadcasts the
                gradient ('KFAC_lw').
    HYBRID_OPT: a fraction of ranks per layer receives the eigendata and
                preconditions; the rest receive the gradient.
    """
    COMM_OPT = 1
    MEM_OPT = 2
    HYBRID_OPT = 3


class _DeviceKLScale(object):
    """KL-clip scale kept on the device: nu = min(1, sqrt(kl_clip/|vg*lr^2|))."""
    __slots__ = ('vg', 'lr', 'kl_clip')

    def __init__(self, vg, lr, kl_clip):
        self.vg, self.lr, self.kl_clip = vg, lr, kl_clip

    def item(self):
        return precond_ops.kl_scale(self.vg, self.lr, self.kl_clip)


_INV_EXECUTOR = None


def _inverse_executor():
    global _INV_EXECUTOR
    if _INV_EXECUTOR is None:
        import concurrent.futures
        _INV_EXECUTOR = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix='kfac-inv')
    return _INV_EXECUTOR


# Measured cost of one factor's eigendecomposition on MI355X with the fused
# solver (reduction + divide and conquer + back-transformation), fitted to
# probe timings of (n, batch) classes: T(n, b) = a n + b (c2 n^2 + c3 n^3) ms
# (profiles/r2_eig_cost_fit.log).  The per-column term dominates: the
# reduction is a latency-bound chain of n columns, so the reference's n^3
# (kfac/preconditioner.py:625-631) overstates big factors ~5x against small.
MEASURED_COST_MS = (1.622e-2, 1.963e-7, 1.389e-10)


def measured_cost(n):
    a, c2, c3 = MEASURED_COST_MS
    return a * n + c2 * n * n + c3 * n ** 3


# Batched per-rank cost (ms) of the fused solver on MI355X: a rank solves all
# its factors in ONE ragged launch sequence, so its time is a set function --
# the column chain of its largest factor (latency per column) plus the
# traffic / flops of all of them -- not a sum of single-factor costs (the
# 'measured' table summed to 1,432 ms for ResNet-50's 108 factors against
# 157 ms measured batched).  T(S) = a n_max + b3 sum n^3 + b2 sum n^2 + b0 |S|,
# least-squares fit to one-GPU solves of per-rank sets
# (scripts/probes/probe_inverse_share.py; refit in round 6 on the solver with
# single-launch tail columns: mean error 2.7 %, max 11.7 %, where the round-3
# table was off by 15.1 % mean; profiles/r6_inverse_share.log).
BATCHED_COST_MS = (8.814e-3, 4.811e-11, 2.840e-7, -8.399e-3)


def batched_cost(sizes):
    """Modelled wall time (ms) of solving every factor in `sizes` together."""
    if not sizes:
        return 0.0
    a, b3, b2, b0 = BATCHED_COST_MS
    return (a * max(sizes) + b3 * sum(float(n) ** 3 for n in sizes) +
            b2 * sum(float(n) ** 2 for n in sizes) + b0 * len(sizes))


def assignment_cost(strategy):
    """n -> LPT cost of a factor: 'compute' n^3 and 'memory' n^2 (reference
    semantics, kfac/preconditioner.py:625-631), 'measured' the MI355X table,
    or a user callable."""
    if callable(strategy):
        return strategy
    return {'compute': lambda n: n ** 3, 'memory': lambda n: n ** 2,
            'measured': measured_cost, 'batched': measured_cost}[strategy]


class KFAC(optim.Optimizer):
    def __init__(self, model, damping=0.001, factor_decay=0.95, factor_update_freq=10,
                 inv_update_freq=100, kl_clip=0.001, lr=0.1, accumulate_data=False,
                 assignment_strategy='compute', batch_first=True,
                 comm_method=CommMethod.COMM_OPT, compute_factor_in_hook=False,
                 distribute_layer_factors=True, inv_dtype=torch.float32, grad_scaler=None,
                 grad_worker_fraction=0.25, factor_dtype=None, precompute_outer_eigen=True,
                 use_eigen_decomp=True, skip_layers=[], verbose=False,
                 bucket_cap_mb=64.0, symmetry_aware_comm=True, eigen_solver='auto',
                 profile=False, use_hip_graphs=True, precond_precision='fp32',
                 fused_precondition=True, inverse_lag=0, comm_check=False,
                 overlap_precondition=False, defer_factor_comm=True, early_factors=False):
        if not 0.0 <= lr:
            raise ValueError('Invalid learning rate: {}'.format(lr))
        if not 0.0 < factor_decay <= 1:
            raise ValueError('Invalid factor decay rate: {}'.format(factor_decay))
        if not 0.0 < damping:
            raise ValueError('Invalid damping: {}'.format(damping))
        if kl_clip is not None and not 0.0 < kl_clip:
            raise ValueError('Invalid clipping value: {}'.format(kl_clip))
        if not 0 < factor_update_freq:
            raise ValueError('Invalid factor update frequency: {}'.format(factor_update_freq))
        if not 0 < inv_update_freq:
            raise ValueError('Invalid K-FAC update frequency: {}'.format(inv_update_freq))
        if not 0 <= inverse_lag < inv_update_freq:
            raise ValueError('inverse_lag must be in [0, inv_update_freq): {}'.format(inverse_lag))
        if inv_update_freq % factor_update_freq != 0:
            warnings.warn('It is suggested that inv_update_freq be a multiple of '
                          'factor_update_freq')
        if not callable(assignment_strategy) and \
                assignment_strategy not in ('compute', 'memory', 'measured', 'batched'):
            raise ValueError('assignment_strategy must be "compute", "memory", "measured", '
                             '"batched" or '
                             'a callable n -> cost')
        if not isinstance(comm_method, CommMethod):
            raise ValueError('comm_method must be a kfac.CommMethod')
        if comm_method in (CommMethod.MEM_OPT, CommMethod.HYBRID_OPT) and \
                distribute_layer_factors:
            warnings.warn('MEM_OPT or HYBRID_OPT and distribute_layer_factors=True cannot be '
                          'used at the same time. Defaulting to distribute_layer_factors=False')
            distribute_layer_factors = False

        known = {m.lower() for m in kfac_layers.KNOWN_MODULES}
        if skip_layers is None:
            skip_layers = []
        elif isinstance(skip_layers, str):
            skip_layers = [skip_layers.lower()]
        else:
            skip_layers = [s.lower() for s in skip_layers]
        # an entry names a module class ('linear', reference semantics) or,
        # extension, a submodule by attribute or dotted name ('head',
        # 'blocks.0.fc1'): e.g. a 10k-vocabulary output projection whose
        # 10k x 10k gradient factor would dominate the inverse update
        for s in skip_layers:
            known.discard(s)

        defaults = dict(damping=damping, factor_decay=factor_decay,
                        factor_update_freq=factor_update_freq, inv_update_freq=inv_update_freq,
                        kl_clip=kl_clip, lr=lr, step=0)
        # K-FAC owns no parameters; a placeholder keeps optim.Optimizer and
        # the LR schedulers working on param_groups[0]
        super(KFAC, self).__init__([torch.tensor(0.0)], defaults)

        self.accumulate_data = accumulate_data
        self.assignment_strategy = assignment_strategy
        self.batch_first = batch_first
        self.comm_method = comm_method
        self.compute_factor_in_hook = compute_factor_in_hook
        self.distribute_layer_factors = distribute_layer_factors
        self.inv_dtype = inv_dtype
        self.grad_scaler = grad_scaler
        self.factor_dtype = factor_dtype
        self.precompute_outer_eigen = precompute_outer_eigen
        self.use_eigen_decomp = use_eigen_decomp
        self.skip_layers = skip_layers
        self.known_modules = known
        self.verbose = verbose
        self.bucket_cap_mb = bucket_cap_mb
        self.symmetry_aware_comm = symmetry_aware_comm
        self.eigen_solver = eigen_solver
        # host-checks the eigensolver status once per inverse step (one sync)
        self.check_solver = True
        self._solver_check_due = False
        self._deferred_checks = []
        # debug mode: checksum-compare the buffers each collective phase must
        # leave identical on every rank (utils/comm_check.py)
        self.comm_check = bool(comm_check) or \
            bool(int(__import__('os').environ.get('KFAC_COMM_CHECK', '0')))
        # the factor all-reduce of a factor step is issued asynchronously and
        # joined where the averaged factors are consumed (next EMA / inverse
        # update / state_dict): parallel/collectives.FactorAllreduce
        self.defer_factor_comm = bool(defer_factor_comm)
        self._factor_comm_step = None   # step whose factor comm step_factor_comm() issued
        self.workers_assigned = False
        self.plan = None
        self.plan_generation = 0
        self._plan_shapes = None
        self._retired_plans = []
        self.timer = PhaseTimer(enabled=profile)
        self.use_hip_graphs = use_hip_graphs
        if precond_precision not in precond_fused.PRECISIONS:
            raise ValueError('precond_precision must be one of {}'.format(
                sorted(precond_fused.PRECISIONS)))
        self.precond_precision = precond_precision
        self.fused_precondition = fused_precondition
        # single rank, one backward per step: the last layers' chain starts on a
        # side stream from a gradient hook, under the rest of the backward
        self.overlap_precondition = bool(overlap_precondition)
        self._top_hooks = []
        self._top_seen = 0
        self._eigen_gen = 0         # bumped whenever new eigendata is in place
        # all factors of a step in a few grouped launches (GPU)
        self.grouped_factors = True
        # early_factors: on a factor step the A factors (this step's layer
        # inputs, complete once backward starts) are computed on a side stream
        # from the first gradient hook, under the backward; step() joins them
        # before the G factors.  Same kernels, same per-factor reduction order:
        # bitwise the same factors as computing everything in step()
        self.early_factors = bool(early_factors)
        self._factor_stream = None
        self._early_a = None        # the A jobs in flight (keeps the activations alive)
        self._early_a_step = None
        self._fwd_step = None       # forward passes per step (_count_forward)
        self._fwd_calls = 0
        self._prev_fwd_calls = None
        self._reverse_hooked = False
        self._segmented_capture = False   # set by graphs.GraphedTrainStep
        # compute_factor_in_hook on the GPU: gradient hooks of this step seen /
        # registered (the last one runs the grouped factor launches)
        self._hook_step = None
        self._defer_hook = False     # defer_hook_factors(): save only, compute later
        self._hook_flush_warned = False
        self._g_seen = 0
        self._g_expected = 0
        self.fused = None
        self._fused_kl = None
        self._graph = None
        self._graph_sig = None
        self._graph_scale = None
        self._graph_warm = False
        self._sync_before_replay = False
        # lagged inverses (inverse_lag > 0): the eigendecompositions of step k
        # run on a side stream, launched by a host thread, while steps
        # k .. k+lag-1 keep preconditioning with the previous eigendata
        self.inverse_lag = int(inverse_lag)
        self._pending_inv = None
        self._inv_stream = None
        self._have_inverses = False
        # early inverse update (GPU, one rank, graphs.GraphedTrainStep's
        # inverse steps): the factors of the solve's leading group (the
        # largest, all A factors -- ResNet-50's three 4608^2) are updated from
        # the backward's FIRST gradient hook and their eigensolve is launched
        # there, on the eigensolver's worker stream, while the backward and
        # the other factors still run; compute_inverses() solves the rest and
        # joins it.  Same inputs, same kernels as the one-batch solve.
        # Opt-in (KFAC_EARLY_INVERSE=1 or this attribute): the armed
        # forward/backward runs eagerly, and its host-bound backward slows
        # the early chain about as much as the early start wins -- ResNet-50
        # inverse step 120.7-123.7 ms against 121.7-122.7 without
        # (profiles/README.md, round 6)
        self.early_inverse = __import__('os').environ.get('KFAC_EARLY_INVERSE', '0') == '1'
        self._early_inv_armed = False
        self._early_inv_a_done = False
        self._early_inv = None          # the solve in flight: jobs, results, stream, flags
        self._early_inv_key = None
        self._early_inv_jobs = None
        self.early_inverse_launches = 0

        comm.init_comm_backend()
        size = comm.backend.size()
        if self.comm_method == CommMethod.COMM_OPT:
            self.grad_worker_fraction = 1
        elif self.comm_method == CommMethod.MEM_OPT:
            self.grad_worker_fraction = 0
        else:
            if not 0 <= grad_worker_fraction <= 1:
                raise ValueError('grad_worker_fraction must in (0, 1) when using HYBRID_OPT')
            workers = max(1, int(round(size * grad_worker_fraction)))
            if size % workers != 0:
                raise ValueError('grad_worker_fraction must produce groups of equal size')
            if 1.0 / size >= grad_worker_fraction:
                warnings.warn('grad_worker_fraction <= 1/world_size, for best performance, '
                              'use COMM_OPT')
            elif 1 - 1.0 / size <= grad_worker_fraction:
                warnings.warn('grad_worker_fraction >= 1-1/world_size, for best performance, '
                              'use COMM_OPT')
            elif 0.5 < grad_worker_fraction:
                warnings.warn('grad_worker_fraction={}, for best performance use a value in '
                              '[0, 0.5] when using HYBRID_OPT.'.format(grad_worker_fraction))
            self.grad_worker_fraction = grad_worker_fraction
        if self.precompute_outer_eigen and self.distribute_layer_factors and size > 1:
            warnings.warn('precompute_outer_eigen=True requires the A and G eigendecompositions '
                          'of a layer on one rank; using distribute_layer_factors=False')
            self.distribute_layer_factors = False

        self.layers = []
        self.hook_layers = {}
        self._hook_handles = []
        self._factor_allreduce = collectives.FactorAllreduce(
            self.layers, bucket_cap_mb=bucket_cap_mb, symmetric=symmetry_aware_comm)
        self.register_model(model)

    # ------------------------------------------------------------------ repr
    def __repr__(self):
        extra = {
            'accumulate_data': self.accumulate_data,
            'assignment_strategy': self.assignment_strategy,
            'batch_first': self.batch_first,
            'comm_method': self.comm_method,
            'compute_factor_in_hook': self.compute_factor_in_hook,
            'distribute_layer_factors': self.distribute_layer_factors,
            'inv_dtype': self.inv_dtype,
            'grad_scaler': self.grad_scaler is not None,
            'grad_worker_fraction': self.grad_worker_fraction,
            'factor_dtype': self.factor_dtype,
            'known_modules': self.known_modules,
            'precompute_outer_eigen': self.precompute_outer_eigen,
            'use_eigen_decomp': self.use_eigen_decomp,
            'skip_layers': self.skip_layers,
            'verbose': self.verbose,
            'registered_layers': len(self.layers),
        }
        s = self.__class__.__name__ + ' ('
        for i, group in enumerate(self.param_groups + [extra]):
            s += '\nParameter Group {0}\n'.format(i)
            for key in sorted(group.keys()):
                if key != 'params':
                    s += '    {0}: {1}\n'.format(key, group[key])
        return s + ')'

    # ------------------------------------------------------------ state dict
    def state_dict(self, include_layer_factors=True, include_layer_inverses=False):
        self.wait_inverses()
        self.join_factor_comm()
        sd = super(KFAC, self).state_dict()
        layers = None
        if include_layer_factors:
            if self.comm_method is CommMethod.MEM_OPT and include_layer_inverses:
                warnings.warn('Layer inverses cannot be saved to the state dict when using '
                              'CommMethod.MEM_OPT. Skipping saving inverses.')
                include_layer_inverses = False
            layers = [l.state_dict(include_layer_inverses) for l in self.layers]
        sd['layers'] = layers
        return sd

    def load_state_dict(self, state_dict, compute_inverses=True):
        self.join_factor_comm()    # an in-flight all-reduce would overwrite the loaded factors
        if state_dict.get('layers') is not None:
            if len(state_dict['layers']) != len(self.layers):
                raise ValueError('loaded state dict contains a different number of layers')
            for layer, ls in zip(self.layers, state_dict['layers']):
                layer.load_state_dict(ls)
            state_dict = {k: v for k, v in state_dict.items() if k != 'layers'}
        else:
            warnings.warn('Layer factors are not included in the state_dict so inverses cannot '
                          'be computed. Skipping inverse computation.')
            compute_inverses = False
            state_dict = {k: v for k, v in state_dict.items() if k != 'layers'}
        super(KFAC, self).load_state_dict(state_dict)
        if compute_inverses:
            # keep the plan (and the arenas / fused operand buffers a captured
            # graph addresses) when the factor shapes did not change
            if not (self.workers_assigned and self.plan is not None and
                    self._plan_shapes == self._factor_shapes()):
                self._assign_workers()
            self.workers_assigned = True
            self.compute_inverses(damping=self.param_groups[0]['damping'])
            if self.comm_method in (CommMethod.COMM_OPT, CommMethod.HYBRID_OPT):
                self.broadcast_inverses()
            self._eigendata_updated()

    # ---------------------------------------------------------- registration
    def _layer_kwargs(self):
        return dict(accumulate_data=self.accumulate_data, batch_first=self.batch_first,
                    inv_dtype=self.inv_dtype, grad_scaler=self.grad_scaler,
                    factor_dtype=self.factor_dtype,
                    prediv_eigenvalues=self.precompute_outer_eigen,
                    use_eigen_decomp=self.use_eigen_decomp)

    def _attach_hooks(self, module, reverse=False):
        if reverse:
            self._reverse_hooked = True   # A of such layers arrives in backward
        h = module.register_forward_hook(functools.partial(self._forward_hook, reverse=reverse))
        self._hook_handles.append(h)

    def register_module(self, module, name=None):
        for mod, layer in kfac_layers.get_kfac_layers(module, **self._layer_kwargs()):
            if comm.backend.rank() == 0 and self.verbose:
                print('Registered {}: {}'.format(name if name is not None else '', layer))
            self.hook_layers[mod] = layer
            self.layers.append(layer)
            self._attach_hooks(mod)

    def register_submodules(self, parent_module, prefix=''):
        for name, module in parent_module.named_children():
            full = prefix + ('.' if prefix else '') + name
            cls = module.__class__.__name__.lower()
            if cls in self.skip_layers or name.lower() in self.skip_layers or \
                    full.lower() in self.skip_layers:
                continue
            if cls not in self.known_modules:
                self.register_submodules(module, prefix=full)
            elif kfac_layers.module_requires_grad(module) and module not in self.hook_layers:
                self.register_module(module, full)

    def register_model(self, model):
        if len(list(model.children())) == 0:
            cls = model.__class__.__name__.lower()
            if cls in self.known_modules and cls not in self.skip_layers:
                self.register_module(model)
        else:
            self.register_submodules(model)

    def register_shared_module(self, main_module, second_module, reverse_hooks=False):
        warnings.warn('Registering shared weight modules with KFAC is experimental and may '
                      'produce poor results')
        if not isinstance(main_module, torch.nn.Module):
            raise ValueError('main_module must be of type torch.nn.Module')
        if not isinstance(second_module, torch.nn.Module):
            raise ValueError('second_module must be of type torch.nn.Module')
        if not self.accumulate_data:
            raise ValueError('shared weight module registration will not work is '
                             'self.accumulate_data=False')
        pairs = kfac_layers.get_kfac_layers(main_module, **self._layer_kwargs())
        if len(pairs) > 1:
            raise ValueError('KFAC registering for shared weight modules does not work for '
                             'modules with multiple KFACLayers (e.g. LSTMCells)')
        _, layer = pairs[0]
        if comm.backend.rank() == 0 and self.verbose:
            print('Registered: {} (shared weight)'.format(layer))
        self.hook_layers[main_module] = layer
        self.hook_layers[second_module] = layer
        self.layers.append(layer)
        self._attach_hooks(main_module)
        self._attach_hooks(second_module, reverse=reverse_hooks)

    # ----------------------------------------------------------------- hooks
    def _factor_step(self):
        g = self.param_groups[0]
        return g['step'] % g['factor_update_freq'] == 0

    def _no_autocast(self, t):
        return torch.autocast(device_type=t.device.type, enabled=False)

    def _count_forward(self, module):
        """Forward passes per step, counted at the first K-FAC layer's hook
        and closed by step() (_close_forward_count): early_factors launches the
        A update from a step's FIRST backward, which is the step() result only
        with one forward/backward per step (several micro-batches apply the
        EMA from the last one).  Counting between step() calls, not per value
        of the step counter, keeps callers that rewind the counter
        (GraphedTrainStep.prepare, a bench restarting its window) from
        looking like micro-batching."""
        if not self.layers or module is not self.layers[0].module:
            return
        st = self.param_groups[0]['step']
        self._fwd_step = st
        self._fwd_calls += 1
        if self._fwd_calls > 1 and self._early_a_step == st:
            # the pattern changed under an early launch: this step's A got
            # the first micro-batch's EMA as well; stop launching early
            warnings.warn('K-FAC early_factors: several forward passes in one step (micro-'
                          'batching); early A-factor launches disabled')
            self.early_factors = False

    def _close_forward_count(self):
        """End of a step (step() / step_finish()): this step's forward count
        becomes the previous one."""
        self._prev_fwd_calls = self._fwd_calls
        self._fwd_calls = 0

    @contextlib.contextmanager
    def defer_hook_factors(self):
        """With compute_factor_in_hook: the forward / backward passes inside
        this block only SAVE their hook data (the next pass overwrites it
        unless accumulate_data), computing no factor.  A micro-batched step
        runs all but its last micro-batch under it, so the factors come from
        the last micro-batch with ONE running-average update per factor step
        -- the reference's default (accumulate_data=False, factors in step(),
        kfac/preconditioner.py:494-497, kfac/layers/base.py:364-379) -- not k
        EMA updates, one per micro-batch.  Also captured correctly: the hooks
        run (and read the flag) while a graph is being captured."""
        prev, self._defer_hook = self._defer_hook, True
        try:
            yield
        finally:
            self._defer_hook = prev

    @contextlib.contextmanager
    def hook_factors(self):
        """Inside this block the hooks compute this step's factors themselves
        (as with compute_factor_in_hook=True) and step() does not compute them
        again.  graphs.GraphedTrainStep uses it for a one-process (single-
        segment) trainer's inverse-update steps: their forward/backward replays
        a graph with the factor launches inside, and only the update runs
        eagerly (a replayed graph runs no Python hooks, so factors computed in
        step() from hook-saved tensors would read another graph's buffers)."""
        prev = self.compute_factor_in_hook
        self.compute_factor_in_hook = True
        try:
            yield
        finally:
            self.compute_factor_in_hook = prev

    def _forward_hook(self, module, input, output, reverse=False):
        if torch.is_grad_enabled() and self.early_factors:
            self._count_forward(module)
        if not (torch.is_grad_enabled() and self._factor_step()):
            return
        layer = self.hook_layers[module]
        alpha = self.param_groups[0]['factor_decay']
        if self._defer_hook and self.compute_factor_in_hook:
            if reverse:
                layer.save_grad_outputs(input)
            else:
                layer.save_inputs(input)
            if isinstance(output, torch.Tensor) and output.requires_grad:
                output.register_hook(functools.partial(self._grad_hook_deferred, module, reverse))
            return
        grouped = self._hook_factors_grouped()
        if grouped:
            self._hook_counters()
        if reverse:
            layer.save_grad_outputs(input)
        else:
            layer.save_inputs(input)
            if self.compute_factor_in_hook and not grouped:
                self.join_factor_comm()     # the EMA reads the averaged factors
                with self._no_autocast(input[0]):
                    layer.update_A_factor(alpha=alpha)
        if isinstance(output, torch.Tensor) and output.requires_grad:
            if grouped:
                self._g_expected += 1
            output.register_hook(functools.partial(self._grad_hook, module, reverse))

    def _grad_hook_deferred(self, module, reverse, grad):
        if not self._factor_step():
            return
        layer = self.hook_layers[module]
        if reverse:
            layer.save_inputs((grad,))
        else:
            layer.save_grad_outputs((grad,))

    def _grad_hook(self, module, reverse, grad):
        if not self._factor_step():
            return
        layer = self.hook_layers[module]
        if reverse:
            layer.save_inputs((grad,))
            return
        if self._early_a_due():
            self._launch_early_a()
        if self._early_inv_armed and not self._early_inv_a_done:
            self._early_inverse_factors()
        layer.save_grad_outputs((grad,))
        if self.compute_factor_in_hook:
            if self._hook_factors_grouped():
                # the last gradient hook of this backward: every factor of the
                # step in the grouped launches, still inside the backward (and
                # inside a captured forward/backward graph)
                self._hook_counters()
                self._g_seen += 1
                if self._g_seen == self._g_expected:
                    self._g_seen = self._g_expected = 0
                    with self._no_autocast(grad):
                        self.compute_factors(alpha=self.param_groups[0]['factor_decay'])
                return
            self.join_factor_comm()
            with self._no_autocast(grad):
                layer.update_G_factor(alpha=self.param_groups[0]['factor_decay'])

    def _hook_factors_grouped(self):
        """compute_factor_in_hook on the GPU: save in the hooks, and run the
        grouped SYRK + EMA launches from the backward's last gradient hook
        instead of ~3 launches per factor from every hook.  With
        accumulate_data (an LSTM: every gate Linear runs once per time step)
        the last hook folds ALL of the backward's sources into one EMA per
        factor -- the factors of computing them in step() after that
        backward (reference accumulate semantics, kfac/layers/base.py:364-379),
        instead of one EMA per time step."""
        return (self.compute_factor_in_hook and self.grouped_factors and bool(self.layers)
                and self.layers[0].module.weight.is_cuda and not self._reverse_hooked)

    def _hook_counters(self):
        st = self.param_groups[0]['step']
        if self._hook_step != st:
            self._hook_step = st
            self._g_seen = self._g_expected = 0

    def _flush_hook_factors(self):
        """Grouped in-hook factors whose last gradient hook never came (a
        hooked output the loss does not use, an output recomputed under
        activation checkpointing): compute the saved factors now, in step(),
        so no layer loses this step's update (the per-hook path and the
        reference, kfac/base_preconditioner.py, only lose the factor of the
        layer whose hook did not run)."""
        if not (self._g_expected and self._hook_step == self.param_groups[0]['step']
                and self._hook_factors_grouped()):
            return
        if not self._hook_flush_warned:
            self._hook_flush_warned = True
            warnings.warn('K-FAC: %d of %d hooked module outputs received no gradient in this '
                          'backward; the grouped in-hook factor update runs in step() instead '
                          '(every later such step too)' % (self._g_expected - self._g_seen,
                                                           self._g_expected))
        self._g_seen = self._g_expected = 0
        with torch.autocast(device_type='cuda', enabled=False):
            self.compute_factors(alpha=self.param_groups[0]['factor_decay'])

    # ----------------------------------------------- early A factors
    def _early_a_due(self):
        p = self.param_groups[0]
        return (self.early_factors and self._early_a is None and self.grouped_factors
                and self._early_a_step != p['step'] and not self.compute_factor_in_hook
                # exactly one forward pass in the previous step and so far in
                # this one (micro-batching: the early A would not be step()'s)
                and self._prev_fwd_calls == 1 and self._fwd_calls == 1
                and not self.accumulate_data and not self._reverse_hooked
                and bool(self.layers) and self.layers[0].module.weight.is_cuda
                # a segmented capture would fork in the forward/backward graph and
                # join in the separately captured update graph
                and not (self._segmented_capture and torch.cuda.is_current_stream_capturing()))

    def _launch_early_a(self):
        """First gradient hook of a factor step: every layer's A factor (its
        forward inputs are all saved) on the factor stream, under the backward."""
        p = self.param_groups[0]
        self._early_a_step = p['step']
        self.join_factor_comm()     # the EMA reads the averaged factors
        items, refs = [], []
        for layer in self.layers:
            job = layer.take_factor_job('A')
            if job is None:
                continue
            if layer.state['A'] is None:     # allocated on the main stream
                n = job[0][0].ncols
                layer.state['A'] = torch.eye(n, dtype=job[1], device=layer.module.weight.device)
            items.append((layer.state['A'], job[0], job[1], job[2]))
            refs.append(layer)
        if not items:
            return
        cur = torch.cuda.current_stream()
        if self._factor_stream is None:
            self._factor_stream = torch.cuda.Stream(device=cur.device)
        side = self._factor_stream
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            outs = factor_ops.update_factors_grouped(items, p['factor_decay'], tag='_early')
        for layer, st in zip(refs, outs):
            layer.state['A'] = st
        self._early_a = items

    # ----------------------------------------------- early inverse update
    def early_inverse_jobs(self):
        """The (layer, 'A') jobs of the eigensolve's leading group
        (eigen.leading_group over this step's factor sizes) when the early
        inverse update applies: eigen path on the GPU, one rank, grouped
        factors, synchronous inverses, and a leading group of A factors only.
        [] otherwise.  Fixed per execution plan."""
        key = self.plan_generation
        if self._early_inv_key == key and self._early_inv_jobs is not None:
            return self._early_inv_jobs
        jobs = []
        if (self.early_inverse and self.workers_assigned and self.use_eigen_decomp
                and self.inverse_lag == 0 and self.grouped_factors and self.layers
                and self.eigen_solver == 'auto' and not eigen_ops.TWO_STAGE
                and self.layers[0].module.weight.is_cuda and comm.backend.size() == 1
                and not self._reverse_hooked and not self.accumulate_data
                and _lib.use_native(self.layers[0].module.weight)):
            every = [(l, w) for l in self.layers for w in ('A', 'G')]
            sizes = [l.state[w].shape[0] if l.state.get(w) is not None else 0
                     for l, w in every]
            if not all(sizes):
                return []       # factors not allocated yet: decide later
            lead = eigen_ops.leading_group(sizes)
            if lead and len(lead) < len(every) and all(every[i][1] == 'A' for i in lead) \
                    and all(1 < sizes[i] <= eigen_ops.FUSED_MAX_N for i in lead):
                jobs = [every[i] for i in lead]
        self._early_inv_key, self._early_inv_jobs = key, jobs
        return jobs

    def arm_early_inverse(self):
        """graphs.GraphedTrainStep, before an inverse step's forward/backward,
        which it then runs EAGERLY: the first gradient hook updates the
        leading group's A factors and launches their solve on the
        eigensolver's worker stream right there, under the rest of the
        backward (_early_inverse_factors).  A replayed graph cannot be the
        gate: on this ROCm an event recorded inside a graph, or a forked
        branch of it, completes with the whole graph (profiles/README.md).
        True when armed."""
        self._early_inv_armed = bool(self.early_inverse_jobs())
        self._early_inv_a_done = False
        if self._early_inv_armed and eigen_ops.STAGE_LOG:
            # KFAC_EIG_STAGE_LOG=1: the stage times of this step's solves
            # are printed from the start of its forward/backward
            eigen_ops.STAGE_EVENTS = []
            eigen_ops._mark(-1, 'step', torch.cuda.current_stream())
        return self._early_inv_armed

    def disarm_early_inverse(self):
        """After the armed forward/backward: True when its solve was launched
        (compute_inverses() picks it up)."""
        armed, self._early_inv_armed = self._early_inv_armed, False
        done, self._early_inv_a_done = self._early_inv_a_done, False
        return armed and done and self._early_inv is not None

    def _early_inverse_factors(self):
        self._early_inv_a_done = True
        if torch.cuda.is_current_stream_capturing():
            return      # never gated inside a graph (arm_early_inverse); step() solves all
        alpha = self.param_groups[0]['factor_decay']
        items, refs = [], []
        for layer, _ in self._early_inv_jobs:
            job = layer.take_factor_job('A')
            if job is None:
                continue
            items.append((layer.state['A'], job[0], job[1], job[2]))
            refs.append(layer)
        self.join_factor_comm()
        if items:
            with self._no_autocast(items[0][0]):
                outs = factor_ops.update_factors_grouped(items, alpha, tag='_early_inv')
            for layer, st in zip(refs, outs):
                layer.state['A'] = st
        jobs = list(self._early_inv_jobs)
        cur = torch.cuda.current_stream()
        st = eigen_ops.early_stream(cur.device)
        st.wait_stream(cur)
        eigen_ops._mark(-1, 'early gate', st)
        with torch.cuda.stream(st):
            mats = [l.state[w].to(torch.float32) for l, w in jobs]
            finite = _factors_finite(mats)
            results = eigen_ops.symeig_group(mats, 0.0, st, finite=finite)
        self._early_inv = dict(jobs=jobs, results=results, stream=st, finite=finite)
        self.early_inverse_launches += 1

    def _join_early_inverses(self):
        """The early solve's jobs and (Q, d) results, ordered before the
        current stream; (None, None) when none is in flight."""
        e, self._early_inv = self._early_inv, None
        if e is None:
            return None, None
        cur = torch.cuda.current_stream()
        cur.wait_stream(e['stream'])
        for Q, d in e['results']:
            Q.record_stream(cur)
            d.record_stream(cur)
        e['finite'].record_stream(cur)
        return e, [(Q.to(l.inv_dtype), d.to(l.inv_dtype))
                   for (l, _), (Q, d) in zip(e['jobs'], e['results'])]

    def side_streams(self):
        """The streams other than the current one that K-FAC's last step may
        have left work on: the factor stream, the fused chain's side stream,
        the eigensolver's workers and the lagged-inverse stream -- the last
        two only when no lagged update is in flight (that one runs on purpose
        on both).  Not the
        deferred factor all-reduce, which is joined by join_factor_comm()."""
        out = []
        if self._factor_stream is not None:
            out.append(self._factor_stream)
        side = getattr(self.fused, '_side', None)
        if side is not None:
            out.append(side)
        if self.inverses_in_flight:
            # the lagged solve owns _inv_stream AND the eigensolver's worker
            # streams until it is joined: waiting on either would serialise
            # the overlap inverse_lag exists for
            return out
        if self._inv_stream is not None:
            out.append(self._inv_stream)
        if self.layers and self.layers[0].module.weight.is_cuda:
            from .ops import eigen as eigen_ops
            out += eigen_ops.side_streams(self.layers[0].module.weight.device)
        return out

    def join_early_factors(self):
        """Order the current stream after an early A-factor update in flight."""
        if self._early_a is not None:
            torch.cuda.current_stream().wait_stream(self._factor_stream)
            self._early_a = None

    def set_grad_params(self, mapping):
        """Precondition the gradients of other parameters than the modules'
        own: `mapping` {module parameter: parameter whose .grad K-FAC reads and
        rewrites}, e.g. the fp32 masters of bf16-stored weights
        (ops/mixed.BF16Weights.grad_params()).  Factors still come from the
        modules' hooks.  The caller fills the masters' .grad between backward
        and step() (BF16Weights.grads_to_master)."""
        if self.overlap_precondition:
            raise ValueError('overlap_precondition launches from gradient hooks on the module '
                             'parameters; it cannot precondition remapped gradients')
        for layer in self.layers:
            m = layer.module
            layer.grad_weight_param = mapping.get(m.weight)
            bias = getattr(m, 'bias', None)
            layer.grad_bias_param = mapping.get(bias) if bias is not None else None
        self._graph = None            # the tail graph addressed the old .grad tensors
        if self.fused is not None:
            self.fused._gather_sig = None

    def remove_hooks(self):
        for h in self._hook_handles:
            h.remove()
        self._hook_handles = []
        for h in self._top_hooks:
            h.remove()
        self._top_hooks = []

    # -------------------------------------------- early top-layer precondition
    def _early_launch_ok(self):
        p = self.param_groups[0]
        return (isinstance(self.fused, precond_fused.SplitFused) and self._have_inverses
                and self._pending_inv is None and p['step'] % p['inv_update_freq'] != 0
                and not self._graph_eligible() and torch.is_grad_enabled() is False
                # a segmented GraphedTrainStep capture: the side-stream fork would
                # be joined only in the separately captured update graph
                and not torch.cuda.is_current_stream_capturing())

    def _early_tag(self):
        """Identifies the step and eigenbasis an early top-half launch
        belongs to (SplitFused.run reuses it only under the same tag)."""
        return (self.param_groups[0]['step'], self._eigen_gen)

    def _top_grad_hook(self, param):
        self._top_seen += 1
        if self._top_seen == len(self._top_hooks):
            self._top_seen = 0
            if self._early_launch_ok():
                self.fused.launch_top(damping=self.param_groups[0]['damping'],
                                      with_kl=self._fused_all, tag=self._early_tag())

    def _register_top_hooks(self):
        for h in self._top_hooks:
            h.remove()
        self._top_hooks = []
        self._top_seen = 0
        if not isinstance(self.fused, precond_fused.SplitFused):
            return
        for layer in self.fused.top.layers:
            for prm in (layer.module.weight, getattr(layer.module, 'bias', None)):
                if prm is not None and prm.requires_grad:
                    self._top_hooks.append(prm.register_post_accumulate_grad_hook(self._top_grad_hook))

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None):
        """One K-FAC step: call after gradients are averaged, before optimizer.step()."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        p = self.param_groups[0]
        t = self.timer
        if p['step'] % p['factor_update_freq'] == 0 and self._factor_comm_step != p['step']:
            if not self.compute_factor_in_hook:
                with t('factors'):
                    self.compute_factors(alpha=p['factor_decay'])
            else:
                self._flush_hook_factors()
            with t('factor_comm'):
                self.allreduce_factors()
        if self.comm_check and p['step'] % p['factor_update_freq'] == 0:
            self.join_factor_comm()
            self._check_comm('factor all-reduce', ('A', 'G'))
        if not self.workers_assigned:
            self._assign_workers()
            self.workers_assigned = True
        inv_step = p['step'] % p['inv_update_freq'] == 0
        if self._pending_inv is not None and (inv_step or self.inverse_apply_due()):
            with t('inverses'):
                self._apply_lagged_inverses()
        if inv_step:
            if self.inverse_lag > 0 and self._have_inverses:
                with t('inverses'):
                    self._launch_lagged_inverses(p['damping'])
            else:
                with t('inverses'):
                    self.compute_inverses(damping=p['damping'], defer_check=True)
                if self.comm_method in (CommMethod.COMM_OPT, CommMethod.HYBRID_OPT):
                    with t('inverse_comm'):
                        self.broadcast_inverses()
                    if self.comm_check and self.comm_method == CommMethod.COMM_OPT:
                        self._check_comm('eigendata broadcast', self._broadcast_keys())
                self._eigendata_updated()
        if self._graph_eligible():
            with t('precondition'):
                self._graph_replay()
        else:
            with t('precondition'):
                self.compute_preconditioned_gradients(damping=p['damping'])
            if self.comm_method in (CommMethod.MEM_OPT, CommMethod.HYBRID_OPT):
                with t('grad_comm'):
                    self.broadcast_gradients()
                if self.comm_check and self.comm_method == CommMethod.MEM_OPT:
                    self._check_comm('gradient broadcast', None)
            with t('update'):
                scale = None if p['kl_clip'] is None else self._compute_grad_scale()
                self.update_gradients(scale)
        self._finish_solver_check()
        p['step'] += 1
        self._close_forward_count()
        return loss

    # ------------------------------------------------- phased plain steps
    # A plain step (no factor or inverse update) split at its one collective:
    # graphs.GraphedTrainStep(phased_update=True) replays the two compute
    # phases as hipGraphs and issues the MEM_OPT / HYBRID_OPT gradient
    # all-gather eagerly between them, so those steps are no longer eager.
    # step() == step_precondition(); step_communicate(); step_finish().
    def is_plain_step(self):
        """No inverse update this step, and no factor collective left to
        issue (a plain step, or a factor step whose all-reduce
        step_factor_comm() has issued): the rest of step() is capturable."""
        p = self.param_groups[0]
        return (self.workers_assigned and self._pending_inv is None
                and (p['step'] % p['factor_update_freq'] != 0 or
                     self._factor_comm_step == p['step'])
                and p['step'] % p['inv_update_freq'] != 0)

    @torch.no_grad()
    def step_factor_comm(self):
        """Factor step (not an inverse step), graphed training loops: compute
        the factors unless the hooks did, and issue their all-reduce now,
        eagerly; the rest of this step's step() then issues no collective and
        is captured / replayed (graphs.GraphedTrainStep).  Joined at the
        next consumer like any deferred factor all-reduce."""
        p = self.param_groups[0]
        if p['step'] % p['factor_update_freq'] != 0 or p['step'] % p['inv_update_freq'] == 0:
            return
        if not self.compute_factor_in_hook:
            self.compute_factors(alpha=p['factor_decay'])
        else:
            self._flush_hook_factors()
        self.allreduce_factors()
        self._factor_comm_step = p['step']

    def join_factor_comm(self):
        """Join a deferred factor all-reduce (device-side wait + unpack of
        the averaged factors); no-op when none is in flight."""
        if self._factor_allreduce.pending:
            self._factor_allreduce.finish()

    def prepare_factor_step(self):
        """Before a factor step's forward/backward replays (its captured
        hooks run the EMA on the factors): join the previous all-reduce."""
        self.join_factor_comm()

    @torch.no_grad()
    def step_precondition(self):
        if not self.is_plain_step():
            raise RuntimeError('step_precondition() is for plain steps only; use step()')
        self.compute_preconditioned_gradients(damping=self.param_groups[0]['damping'])

    @torch.no_grad()
    def step_communicate(self):
        if self.comm_method in (CommMethod.MEM_OPT, CommMethod.HYBRID_OPT):
            self.broadcast_gradients()

    @torch.no_grad()
    def step_finish(self):
        p = self.param_groups[0]
        scale = None if p['kl_clip'] is None else self._compute_grad_scale()
        self.update_gradients(scale)
        p['step'] += 1
        self._close_forward_count()

    # ------------------------------------------------------------ hipGraphs
    def _precondition_and_apply(self):
        p = self.param_groups[0]
        self.compute_preconditioned_gradients(damping=p['damping'])
        scale = None if p['kl_clip'] is None else self._compute_grad_scale()
        self.update_gradients(scale)
        return scale

    def _graph_eligible(self):
        """The steady-state tail (precondition -> KL dot -> apply) is captured
        into one hipGraph when it contains no collective (single rank or
        COMM_OPT) and runs on a GPU."""
        if not self.use_hip_graphs or self.plan is None or not self.layers:
            return False
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return False    # an outer whole-step graph (graphs.GraphedTrainStep) is capturing
        if not self.layers[0].module.weight.is_cuda:
            return False
        return comm.backend.size() == 1 or self.comm_method == CommMethod.COMM_OPT

    def _graph_signature(self):
        p = self.param_groups[0]
        ptrs = []
        for layer in self.layers:
            w = layer._get_weight_grad()
            ptrs.append(None if w is None else (w.data_ptr(), tuple(w.stride())))
            if layer.has_bias:
                b = layer._get_bias_grad()
                ptrs.append(None if b is None else b.data_ptr())
            for k in ('QA', 'QG', 'dGdA', 'dA', 'dG', 'A_inv', 'G_inv'):
                v = layer.state.get(k)
                if v is not None:
                    ptrs.append(v.data_ptr())
        return (tuple(ptrs), p['lr'], p['kl_clip'], p['damping'])

    def _graph_replay(self):
        sig = self._graph_signature()
        if self._graph is not None and sig == self._graph_sig:
            if self._sync_before_replay:
                # new eigendata came from side streams this step: order the
                # replay after them on the device (event waits, no host sync:
                # the host keeps issuing while the eigensolver runs)
                cur = torch.cuda.current_stream()
                for st in self.side_streams():
                    if st != cur:
                        cur.wait_stream(st)
                self._sync_before_replay = False
            self._graph.replay()
            return
        if not self._graph_warm or sig != self._graph_sig:
            # eager run doubles as the capture warm-up (allocator / library handles)
            self._graph = None
            self._graph_sig = sig
            self._graph_warm = True
            self._precondition_and_apply()
            return
        self.wait_inverses()   # no solver thread may run library calls during a capture
        gc_on = gc.isenabled()
        gc.disable()     # no collected HIP object destroyed mid-capture (graphs.py)
        try:
            g = _lib.new_graph()
            # the captured ops read .grad; run them on a clean copy of the
            # current grads after capture (capture itself does not execute)
            with torch.cuda.graph(g):
                self._graph_scale = self._precondition_and_apply()
            if gc_on:
                gc.enable()
            _lib.finalize_graph(g)
            self._graph = g
            self._graph.replay()
        except Exception as e:  # pragma: no cover - depends on the HIP runtime
            if gc_on:
                gc.enable()
            warnings.warn('hipGraph capture of the K-FAC step failed ({}); running eagerly'
                          .format(e))
            self.use_hip_graphs = False
            self._graph = None
            self._precondition_and_apply()

    def _broadcast_keys(self):
        # the per-layer state the eigendata broadcast delivers to every rank
        if not self.use_eigen_decomp:
            return ('A_inv', 'G_inv')
        return ('QA', 'QG', 'dGdA') if self.precompute_outer_eigen else ('QA', 'QG', 'dA', 'dG')

    def _check_comm(self, phase, keys):
        """Debug mode: raise comm_check.CommConsistencyError unless the
        `keys` of every layer's state (or, with keys=None, every layer's
        preconditioned gradient) are identical on every rank."""
        if comm.backend.size() == 1:
            return
        named = []
        for i, layer in enumerate(self.layers):
            tag = '{}:{}'.format(i, type(layer.module).__name__)
            if keys is None:
                g = layer.preconditioned_gradient
                parts = list(g) if isinstance(g, (list, tuple)) else [g]
                named += [('{}.grad{}'.format(tag, j), x) for j, x in enumerate(parts)
                          if x is not None]
            else:
                named += [('{}.{}'.format(tag, k), layer.state[k]) for k in keys
                          if layer.state.get(k) is not None]
        comm_check.assert_consistent(named, phase)

    def allreduce_factors(self):
        """Issue the bucketed factor all-reduce; with defer_factor_comm it is
        joined at the averaged factors' next consumer (join_factor_comm)."""
        if comm.backend.size() == 1:
            return
        self._factor_allreduce.start()
        if not self.defer_factor_comm:
            self._factor_allreduce.finish()

    def broadcast_inverses(self):
        if comm.backend.size() == 1:
            return
        if self.plan is not None and self.plan.eig_arena is not None:
            collectives.broadcast_eigendata(self.plan)
            return
        handles = []
        for layer in self.layers:
            handles.extend(layer.broadcast_inverses())
        comm.backend.sync(handles)

    def broadcast_gradients(self):
        if comm.backend.size() == 1:
            return
        if self.plan is not None:
            collectives.broadcast_gradients(self.plan)
            for layer in self.layers:
                layer.preconditioned_gradient = layer._split_pgrad(layer._pgrad_matrix())
            return
        handles = []
        for layer in self.layers:
            handles.extend(layer.broadcast_gradient())
        comm.backend.sync(handles)

    def _inverse_jobs(self):
        rank = comm.backend.rank()
        jobs = []
        for layer in self.layers:
            for which in ('A', 'G'):
                layer._check_assigned(which)
                layer._unfold_flat(which)
                layer._ensure_inv_buffers(which)
                if getattr(layer, 'compute_{}_inv_rank'.format(which)) == rank:
                    jobs.append((layer, which))
        return jobs

    def _solve_inverses(self, jobs, mats, damping, finite=None, split=True):
        if self.use_eigen_decomp:
            results = eigen_ops.symeig_many(mats, clip=0.0, solver=self.eigen_solver,
                                            finite=finite, split=split)
            if _DEBUG_EIG:
                _debug_check_eig(jobs, mats, results)
            return [(Q.to(l.inv_dtype), d.to(l.inv_dtype))
                    for (l, _), (Q, d) in zip(jobs, results)]
        return [r.to(l.inv_dtype)
                for (l, _), r in zip(jobs, eigen_ops.inverse_many(mats, damping))]

    @staticmethod
    def _store_inverses(jobs, results, damping):
        # A before G: the G owner forms dGdA from both eigenvalue sets
        order = sorted(zip(jobs, results), key=lambda x: x[0][1])
        if not (order and all(isinstance(r, tuple) for _, r in order) and order[0][1][0].is_cuda):
            for (layer, which), res in order:
                layer.finish_inverse(which, res, damping)
            return
        # the eigendata of every factor into the layers' buffers in one grouped
        # copy (layer.finish_inverse's stores, ~2 launches per factor before)
        dsts, srcs = [], []
        for (layer, which), (Q, d) in order:
            for key, v in (('Q' + which, Q), ('d' + which, d)):
                v = v.to(layer.inv_dtype)
                cur = layer.state.get(key)
                if cur is not None and cur.shape == v.shape and cur.dtype == v.dtype:
                    dsts.append(cur)
                    srcs.append(v)
                else:
                    layer.state[key] = v
        if dsts:
            torch._foreach_copy_(dsts, srcs)
        for (layer, which), _ in order:
            if which == 'G' and layer.prediv_eigenvalues:
                layer._store_outer_reciprocal(damping)

    @torch.no_grad()
    def compute_inverses(self, damping=0.001, defer_check=False):
        """Eigendecompose / invert every factor this rank owns, in one batch.

        defer_check (step()): the solver-status check -- a host read that waits
        for the whole solve -- runs at the end of step(), after the eigendata
        store, the preconditioning and the gradient update are enqueued behind
        the solve, so the device never idles while the host issues them."""
        self._drop_lagged_inverses()
        self.join_factor_comm()
        jobs = self._inverse_jobs()
        self._have_inverses = True
        early = self._early_inv
        if early is not None:
            # the leading group is already being solved (_early_inverse_factors):
            # the rest as one group on this stream, beside it
            ek = {(id(l), w) for l, w in early['jobs']}
            if not defer_check or not ek <= {(id(l), w) for l, w in jobs}:
                raise RuntimeError('early inverse update in flight outside step()')
            jobs = [(l, w) for l, w in jobs if (id(l), w) not in ek]
        if not jobs and early is None:
            return
        mats = [l.state[w].to(torch.float32) for l, w in jobs]
        if early is not None:
            results = []
            if jobs:
                finite = _factors_finite(mats)
                results = self._solve_inverses(jobs, mats, damping, finite, split=False)
            e, eres = self._join_early_inverses()
            every = [(l, w) for l in self.layers for w in ('A', 'G')]
            self._deferred_checks.append(
                (every, _factors_finite([l.state[w] for l, w in every])))
            if self.check_solver:
                self._solver_check_due = True
            self._store_inverses(jobs + e['jobs'], results + eres, damping)
            return
        if defer_check and self.use_eigen_decomp and mats[0].is_cuda:
            # no host read before the solve: flagged factors are solved as the
            # identity and the flags are checked at the end of step().  The
            # raise then comes AFTER this step's state changes (the identity
            # eigendata of a flagged factor is stored, broadcast and applied).
            # Every rank checks EVERY layer's factors (they are replicated by
            # the factor all-reduce), not only the ones it solved, so all
            # ranks raise at the same step -- none trains on from a
            # broadcast identity -- with no extra collective.
            finite = _factors_finite(mats)
            results = self._solve_inverses(jobs, mats, damping, finite)
            every = [(l, w) for l in self.layers for w in ('A', 'G')]
            self._deferred_checks.append(
                (every, _factors_finite([l.state[w] for l, w in every])))
        else:
            _check_factors_finite(jobs, mats)
            results = self._solve_inverses(jobs, mats, damping)
        if self.use_eigen_decomp and self.check_solver:
            if defer_check:
                self._solver_check_due = True
            else:
                eigen_ops.check_solver_status()
        self._store_inverses(jobs, results, damping)

    def _finish_solver_check(self):
        """The host reads step() deferred past its enqueued work: non-finite
        factors of this step's inverse update, then the solver status."""
        checks, self._deferred_checks = self._deferred_checks, []
        for jobs, finite in checks:
            _raise_nonfinite(jobs, finite)
        if self._solver_check_due:
            self._solver_check_due = False
            eigen_ops.check_solver_status()

    # ------------------------------------------------------ lagged inverses
    # inverse_lag = L > 0 (opt-in; 0 is the reference's synchronous schedule,
    # kfac/preconditioner.py:506-510): the inverse update of step k
    # snapshots the factors, launches their eigendecompositions on a side
    # stream from a host thread and returns; steps k .. k+L-1 precondition
    # with the previous eigendata, step k+L waits for the solve, stores and
    # broadcasts the result.  The eigensolver is panel-latency bound
    # (profiles/README.md), so the model's kernels fill the CUs it leaves
    # idle.  Asynchronous, stale curvature inverses as in Ba, Grosse and
    # Martens, "Distributed second-order optimization using Kronecker-factored
    # approximations" (ICLR 2017).  All ranks apply at the same step, so the
    # eigendata broadcast stays a matched collective.

    def inverse_apply_due(self):
        """True when this step stores the lagged inverse update."""
        pend = self._pending_inv
        return pend is not None and self.param_groups[0]['step'] >= pend['apply_at']

    @property
    def inverses_in_flight(self):
        return self._pending_inv is not None

    def _launch_lagged_inverses(self, damping):
        self.join_factor_comm()
        jobs = self._inverse_jobs()
        pend = dict(jobs=jobs, damping=damping, results=None, future=None, event=None,
                    apply_at=self.param_groups[0]['step'] + self.inverse_lag)
        self._pending_inv = pend
        if not jobs:
            return
        # private fp32 snapshot: factor updates of steps k+1.. must not race the solve
        mats = [l.state[w].to(torch.float32, copy=True) for l, w in jobs]
        if not mats[0].is_cuda:
            try:
                _check_factors_finite(jobs, mats)
                pend['results'] = self._solve_inverses(jobs, mats, damping)
            except BaseException:
                self._pending_inv = None
                raise
            return
        dev = mats[0].device
        cur = torch.cuda.current_stream(dev)
        if self._inv_stream is None:
            self._inv_stream = torch.cuda.Stream(device=dev)
        s = self._inv_stream
        s.wait_stream(cur)
        for m in mats:
            m.record_stream(s)

        def work():
            torch.cuda.set_device(dev)
            with torch.cuda.stream(s):
                _check_factors_finite(jobs, mats)
                res = self._solve_inverses(jobs, mats, damping)
                ev = torch.cuda.Event()
                ev.record(s)
            return res, ev

        pend['future'] = _inverse_executor().submit(work)

    def wait_inverses(self):
        """Host-join the solver thread of a lagged inverse update (its GPU
        work may still run; it is applied at its step).  Called before any
        graph capture and by state_dict()."""
        pend = self._pending_inv
        if pend is not None and pend['future'] is not None:
            fut, pend['future'] = pend['future'], None
            try:
                pend['results'], pend['event'] = fut.result()
            except BaseException:
                # the solve failed (e.g. non-finite factors): drop the update so
                # the next step does not store a half-initialised result, and
                # surface the original error
                self._pending_inv = None
                raise

    def _apply_lagged_inverses(self):
        self.wait_inverses()
        pend, self._pending_inv = self._pending_inv, None
        jobs, results = pend['jobs'], pend['results']
        if jobs:
            if pend['event'] is not None:
                cur = torch.cuda.current_stream()
                cur.wait_event(pend['event'])
                for r in results:
                    for t in (r if isinstance(r, tuple) else (r,)):
                        t.record_stream(cur)
                if self.use_eigen_decomp and self.check_solver:
                    eigen_ops.check_solver_status()
            self._store_inverses(jobs, results, pend['damping'])
        if self.comm_method in (CommMethod.COMM_OPT, CommMethod.HYBRID_OPT):
            self.broadcast_inverses()
            if self.comm_check and self.comm_method == CommMethod.COMM_OPT:
                self._check_comm('eigendata broadcast', self._broadcast_keys())
        self._eigendata_updated()

    def _drop_lagged_inverses(self):
        if self._pending_inv is not None:
            self.wait_inverses()
            ev = self._pending_inv['event']
            if ev is not None:
                # the solver's persistent buffers are reused by the next solve
                torch.cuda.current_stream().wait_event(ev)
            self._pending_inv = None

    @torch.no_grad()
    def compute_factors(self, alpha=0.95):
        """Update every layer's A and G.  On the GPU all factors of the step go
        through a handful of grouped SYRK + EMA launches (ops/factors.py
        update_factors_grouped) instead of ~3 launches per factor."""
        self.join_factor_comm()     # the EMA reads the averaged factors
        self.join_early_factors()
        if self.layers and self.layers[0].module.weight.is_cuda and self.grouped_factors:
            items, refs = [], []
            for layer in self.layers:
                for which in ('A', 'G'):
                    job = layer.take_factor_job(which)
                    if job is not None:
                        items.append((layer.state[which], job[0], job[1], job[2]))
                        refs.append((layer, which))
            for (layer, which), st in zip(refs, factor_ops.update_factors_grouped(items, alpha)):
                layer.state[which] = st
            return
        for layer in self.layers:
            layer.update_A_factor(alpha=alpha)
            layer.update_G_factor(alpha=alpha)

    def _eigendata_updated(self):
        """New eigendata is in place: refresh the fused kernels' operand copies."""
        self._sync_before_replay = True
        self._eigen_gen += 1
        if self.fused is not None:
            self.fused.refresh_eigen()

    def _build_fused(self):
        """The grouped MFMA preconditioning chain (ops/precond_fused.py) for
        every layer this rank preconditions, on the GPU: 4 grouped stages on
        the eigen path, 2 (G_inv Grad A_inv) on the damped-inverse path."""
        self.fused = None
        if self.inv_dtype == torch.float32:
            precision = self.precond_precision
        else:
            # the reference's 16-bit inv_dtype (kfac/layers/base.py:435-441,
            # 463, 470): 16-bit eigenvector operands, one MFMA per product
            precision = precond_fused.INV_DTYPE_PRECISION.get(self.inv_dtype)
        if not (self.fused_precondition and self.layers and precision is not None):
            return
        if not self.layers[0].module.weight.is_cuda:
            return
        rank = comm.backend.rank()
        mine = [l for l in self.layers if rank in l.compute_grad_ranks]
        if mine:
            split = self._overlap_split(mine)
            if split:
                self.fused = precond_fused.SplitFused(mine, precision, split)
            else:
                self.fused = precond_fused.FusedPreconditioner(mine, precision)
            self._fused_all = len(mine) == len(self.layers)
        self._register_top_hooks()

    def _overlap_split(self, mine):
        """Index splitting `mine` (forward order) so the suffix carries ~60 % of
        the chain's flops (n_G n_A (n_G + n_A) per layer), or 0 = no split:
        only on one rank (the hook sees local, final gradients), eigen path,
        GPU, at least two layers."""
        if not (self.overlap_precondition and comm.backend.size() == 1 and len(mine) >= 2
                and self.use_eigen_decomp):
            return 0
        cost = []
        for l in mine:
            nG, nA = l.grad_shape[0], l.grad_shape[1]
            cost.append(float(nG) * nA * (nG + nA))
        total, acc = sum(cost), 0.0
        for i in range(len(mine) - 1, 0, -1):
            acc += cost[i]
            if acc >= 0.6 * total:
                return i
        return 0

    @torch.no_grad()
    def compute_preconditioned_gradients(self, damping=0.001):
        self._fused_kl = None
        if self.fused is not None:
            if isinstance(self.fused, precond_fused.SplitFused):
                self._fused_kl = self.fused.run(damping=damping, with_kl=self._fused_all,
                                                tag=self._early_tag())
            else:
                self._fused_kl = self.fused.run(damping=damping, with_kl=self._fused_all)
            return
        for layer in self.layers:
            layer.compute_preconditioned_gradient(damping=damping)


    def _grad_pairs(self):
        pairs = []
        for layer in self.layers:
            pairs.extend(layer.grad_pairs())
        return pairs

    @torch.no_grad()
    def update_gradients(self, scale=None):
        if not self.layers:
            return
        if isinstance(scale, _DeviceKLScale):
            precond_ops.apply_gradients(self._grad_pairs(), scale.vg, scale.lr, scale.kl_clip)
        elif scale is None:
            precond_ops.apply_gradients(self._grad_pairs())
        else:
            for layer in self.layers:
                layer.update_gradient(scale=scale)

    def memory_usage(self):
        """Approximate bytes held by K-FAC layer state, hook data and gradients."""
        def size(t):
            if isinstance(t, (list, tuple)):
                return sum(size(x) for x in t)
            return t.nelement() * t.element_size() if isinstance(t, torch.Tensor) else 0
        b = 0
        for layer in self.layers:
            b += sum(size(v) for v in layer.state.values())
            b += sum(size(x) for x in layer.a_inputs)
            b += sum(size(g[0] if isinstance(g, tuple) else g) for g in layer.g_outputs)
            b += size(layer.preconditioned_gradient)
        return b

    def comm_summary(self):
        """How this rank's K-FAC communication is laid out (JSON-able): the
        backend and world it saw, how the K-FAC world communicator and the
        inverse / gradient sub-groups were built (ncclCommSplit via
        dist.split_group, or new_group), the factor all-reduce buckets and the
        eigendata / gradient arena sizes, and the collectives issued so far.
        Reference: kfac/comm.py:53-64 (CommGroup -> dist.new_group),
        kfac/preconditioner.py:525-553 (one collective per layer and factor)."""
        import torch.distributed as dist
        be = comm.backend
        out = {'backend': dist.get_backend() if (dist.is_available() and dist.is_initialized())
               else 'none',
               'world_size': be.size() if be is not None else 1,
               'kfac_world': None, 'groups': [], 'factor_allreduce': None,
               'eig_arena_bytes': None, 'grad_arena_bytes': None,
               'collectives': be.counters() if be is not None else {}}
        for rec in comm.build_log:
            if rec['what'] == 'kfac_world':
                out['kfac_world'] = {'size': len(rec['ranks']), 'built_by': rec['method']}
            else:
                out['groups'].append({'built_by': rec['method'], 'ranks': rec['ranks']})
        far = self._factor_allreduce
        if far is not None and far.buckets:
            sizes = []
            for dtype, st, en, _ in far.buckets:
                esize = torch.tensor([], dtype=dtype).element_size()
                sizes.append((en - st) * esize)
            out['factor_allreduce'] = {'buckets': len(sizes), 'bucket_bytes': sizes,
                                       'bucket_cap_mb': self.bucket_cap_mb,
                                       'triu_packed': far.symmetric}
        if self.plan is not None:
            p = self.plan
            out['grad_arena_bytes'] = p.grad_arena.numel() * 4
            out['grad_group_size'] = p.grad_group.size if p.grad_group is not None else 1
            if p.eig_arena is not None:
                out['eig_arena_bytes'] = p.eig_arena.numel() * p.eig_arena.element_size()
                out['eig_group_size'] = len(p.eig_ranks)
        return out

    # ------------------------------------------------------------ assignment
    def _assign_workers(self):
        """LPT-balance inverse work over ranks and lay out the execution plan."""
        if len(self.layers) == 0:
            return
        cost = assignment_cost(self.assignment_strategy)
        a_sizes = [l.state['A'].shape[0] for l in self.layers]
        g_sizes = [l.state['G'].shape[0] for l in self.layers]
        a_times = [cost(n) for n in a_sizes]
        g_times = [cost(n) for n in g_sizes]
        world = comm.backend.size()
        rank = comm.backend.rank()
        if self.assignment_strategy == 'batched':
            a_locs, g_locs = self._assign_batched(world, a_sizes, g_sizes)
        elif self.distribute_layer_factors:
            locs = distribution.load_balance(world, a_times + g_times)
            a_locs, g_locs = locs[:len(a_times)], locs[len(a_times):]
        else:
            locs = distribution.load_balance(world, [a + g for a, g in zip(a_times, g_times)])
            a_locs, g_locs = locs, locs
        allocator = distribution.WorkerAllocator(world, self.grad_worker_fraction)
        for i, layer in enumerate(self.layers):
            layer.assign_inverse_workers(a_locs[i], g_locs[i], allocator.get_inv_group(a_locs[i]),
                                         allocator.get_inv_group(g_locs[i]))
            src_ranks = allocator.get_inv_ranks(a_locs[i])
            layer.assign_gradient_workers(src_ranks, allocator.get_grad_groups(src_ranks))
        device = self.layers[0].module.weight.device
        if self.plan is not None:
            # buffers of a superseded plan stay alive: a captured graph may
            # still address them (GraphedTrainStep re-captures on the new
            # plan_generation)
            # Only the latest superseded plan is kept: GraphedTrainStep keys
            # its graphs on plan_generation and KFAC's tail graph on buffer
            # pointers, so no graph older than that can replay again, and
            # work already enqueued on the old buffers is ordered before
            # anything that reuses their memory on the same stream.  Work on
            # OTHER streams (a lagged inverse solve, the communicator's
            # eigendata all-gather, the early-factor stream) is not: the
            # host joins the solver thread and the device drains before the
            # plan retired earlier is released (re-plans are rare).
            if self._retired_plans:
                self.wait_inverses()
                if device.type == 'cuda':
                    torch.cuda.synchronize(device)
            self._retired_plans = [(self.plan, self.fused)]
        self.plan = ExecutionPlan(self.layers, world, rank, a_locs, g_locs, allocator,
                                  self.use_eigen_decomp, self.precompute_outer_eigen,
                                  self.inv_dtype, build_eig_arena=True, device=device)
        self._plan_shapes = self._factor_shapes()
        self.plan_generation += 1
        self._graph = None
        self._build_fused()

    def _assign_batched(self, world, a_sizes, g_sizes):
        """assignment_strategy='batched': makespan-greedy over the batched
        per-rank solve model (batched_cost), then byte balancing of the
        eigendata all-gather slots (utils.distribution.balance_batched)."""
        esize = 4 if self.inv_dtype == torch.float32 else 2
        pre = self.use_eigen_decomp and self.precompute_outer_eigen

        def nbytes(nA, nG, which):
            if not self.use_eigen_decomp:
                return esize * ((nA * nA if 'A' in which else 0) + (nG * nG if 'G' in which else 0))
            b = (nA * nA + (0 if pre else nA)) if 'A' in which else 0
            b += (nG * nG + (0 if pre else nG)) if 'G' in which else 0
            if pre and 'A' in which:
                b += nA * nG         # dGdA lives with the A owner (parallel/plan.py)
            return esize * b
        if self.distribute_layer_factors:
            units = [[n] for n in a_sizes] + [[n] for n in g_sizes]
            ub = ([nbytes(a, g, 'A') for a, g in zip(a_sizes, g_sizes)] +
                  [nbytes(a, g, 'G') for a, g in zip(a_sizes, g_sizes)])
            locs = distribution.balance_batched(world, units, batched_cost, ub)
            return locs[:len(a_sizes)], locs[len(a_sizes):]
        units = [[a, g] for a, g in zip(a_sizes, g_sizes)]
        ub = [nbytes(a, g, 'AG') for a, g in zip(a_sizes, g_sizes)]
        locs = distribution.balance_batched(world, units, batched_cost, ub)
        return locs, locs

    def _factor_shapes(self):
        return tuple((tuple(l.state['A'].shape), tuple(l.state['G'].shape)) for l in self.layers)

    def _compute_grad_scale(self):
        """sum_layers <v, g> * lr^2 -> KL-clip scale, kept on the device."""
        g = self.param_groups[0]
        if self._fused_kl is not None:
            return _DeviceKLScale(self._fused_kl, g['lr'], g['kl_clip'])
        pairs = self._grad_pairs()
        if not pairs[0][0].is_cuda:
            # host path: the reference's own arithmetic, so a CPU run
            # reproduces its trajectory (tests/test_training_quality.py)
            return precond_ops.kl_scale_reference(pairs, g['lr'], g['kl_clip'])
        vg = precond_ops.kl_dot(pairs)
        return _DeviceKLScale(vg, g['lr'], g['kl_clip'])
