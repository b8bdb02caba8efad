"""Headline benchmark: ResNet-50 K-FAC + SGD training throughput on MI355X.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Metric (BASELINE.json): images/sec (whole node) for ResNet-50 / ImageNet-1k
shaped synthetic data, K-FAC (COMM_OPT) preconditioning SGD, bf16 autocast,
per-GPU batch 32 (reference: examples/torch_imagenet_resnet.py:49-60), factor
update every 10 steps, eigendecomposition every 100 steps, damping 1e-3,
kl_clip 1e-3 (reference: scripts/slurm/horovod_imagenet_kfac.slurm:26-31).

Timing: W untimed warmup steps, then exactly K steps bracketed by a barrier +
device synchronize on both sides; the max over ranks is reported.  The K-FAC
step counter is reset to 0 at the start of the timed window so the window
always OPENS with an inverse (eigendecomposition) step: with K < 100 the
window contains more inverse work per step than steady state (conservative),
with K = 100 exactly the steady-state mix.  Nothing is skipped inside the
timed region (factors, inverses, preconditioning, KL clip, DDP all-reduce,
SGD update all run).  Random-init weights, synthetic data (no network).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import launch  # noqa: E402
from distributed_kfac_pytorch_amd import graphs  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import grad_sync as grad_sync_mod  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import overlap  # noqa: E402
from distributed_kfac_pytorch_amd.ops import mixed  # noqa: E402

METRIC = 'images/sec (whole node) ResNet-50 K-FAC+SGD'
# the reference K-FAC on one MI355X, same config and timing (not a BASELINE number):
# a STALE constant measured once by this repository's builders in round 2
# (profiles/r2_reference_kfac_mi355x.log, scripts/bench_reference.py), not re-run per
# bench.  Its images/sec ratio includes model-side work (graphs, channels_last, fused
# BN, bf16-stored weights); the K-FAC-only comparison is kfac_cost_ms_by_kind.
REFERENCE_MI355X_IMG_S = 296.8
# ...its step time by kind (ms) and the same model's stock-module SGD-only eager
# step (profiles/r2_reference_kfac_mi355x.log, profiles/README.md): the
# reference's K-FAC cost per step kind is the difference
REFERENCE_MI355X_STEP_MS = {'plain': 25.283, 'factor': 45.982, 'inverse': 1655.206}
REFERENCE_MI355X_SGD_MS = 13.8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--model', default='resnet50')
    ap.add_argument('--batch-size', type=int, default=32, help='per-GPU batch')
    ap.add_argument('--image-size', type=int, default=224)
    ap.add_argument('--kfac-update-freq', type=int, default=100)
    ap.add_argument('--kfac-cov-update-freq', type=int, default=10)
    ap.add_argument('--damping', type=float, default=0.001)
    ap.add_argument('--kl-clip', type=float, default=0.001)
    ap.add_argument('--comm-method', default='comm-opt',
                    choices=['comm-opt', 'mem-opt', 'hybrid-opt'])
    ap.add_argument('--grad-worker-fraction', type=float, default=0.25)
    ap.add_argument('--no-kfac', action='store_true', help='SGD-only baseline')
    ap.add_argument('--channels-last', type=int, default=1)
    ap.add_argument('--eigen-solver', default='auto')
    ap.add_argument('--profile-phases', action='store_true')
    ap.add_argument('--check-finite', action='store_true',
                    help='debug: sync and print the loss of every timed step')
    ap.add_argument('--precond-precision', default='fp16x3',
                    choices=['fp32', 'bf16x3', 'bf16x6', 'fp16x3'],
                    help='fused preconditioning GEMM precision: fp16x3 (the default: scaled '
                         'fp16 hi/lo planes, 22 significand bits, three MFMAs per product, fp32 '
                         'accumulation; error below torch fp32 GEMMs on every ResNet-50 layer, '
                         'tests/test_gpu_resnet50_parity.py), bf16x6 (three bf16 planes, six '
                         'MFMAs), fp32 (exact-f32 MFMA) or bf16x3 (~1e-5 relative error)')
    ap.add_argument('--sgd-delta', type=int, default=1,
                    help='also time the same steps without K-FAC (hooks removed) and report '
                         'the per-step K-FAC cost (kfac_step_ms)')
    ap.add_argument('--graphs', type=int, default=1,
                    help='hipGraph capture of the training step (1/0)')
    ap.add_argument('--set-to-none', type=int, default=1,
                    help='optimizer.zero_grad(set_to_none=...) (single-rank / DDP paths); '
                         '1 skips the gradient fill + accumulate kernels (~0.8 ms/step); the '
                         'earlier NaNs with 1 were MIOpen workspace memsets inside captured '
                         'graphs (csrc/graph_fix.hip)')
    ap.add_argument('--inverse-lag', type=int, default=0,
                    help='KFAC(inverse_lag=L): eigendecompositions of an inverse step run on a '
                         'side stream and take effect L steps later (0 = reference schedule)')
    ap.add_argument('--assignment-strategy', default='batched',
                    choices=['batched', 'measured', 'compute', 'memory'],
                    help="inverse work distribution: 'batched' = makespan over the MI355X "
                         "batched per-rank solve model + eigendata arena balance "
                         "(preconditioner.BATCHED_COST_MS, profiles/r3_inverse_share.log); "
                         "'measured' = additive per-factor table + LPT; 'compute' = n^3 LPT "
                         "(reference)")
    ap.add_argument('--overlap-grad-comm', type=int, default=1,
                    help='world > 1 with graphs: backward in two graph segments, the top '
                         "half's gradient all-reduce overlapped with the bottom half's backward "
                         '(parallel/overlap.py)')
    ap.add_argument('--overlap-precond', type=int, default=0,
                    help='one rank: the last layers\' preconditioning chain starts on a side '
                         'stream as soon as their gradients exist, under the rest of the '
                         'backward (KFAC(overlap_precondition=True)); off by default: the '
                         'backward already fills the GPU, 11.05 vs 10.91 ms per plain step '
                         '(profiles/r2_final_bench20*.log)')
    ap.add_argument('--early-factors', type=int, default=1,
                    help='factor steps: the A factors (layer inputs) are computed on a side '
                         'stream from the first gradient hook, under the backward '
                         '(KFAC(early_factors=True)); bitwise the same factors')
    ap.add_argument('--fused-sgd', type=int, default=1,
                    help='torch.optim.SGD(fused=True): one multi-tensor kernel for the whole '
                         'momentum + weight-decay update (same math as the reference optimizer)')
    ap.add_argument('--bf16-weights', type=int, default=1,
                    help='graphed steps: Conv/Linear weights stored in bf16 with fp32 masters in '
                         'the optimizer and K-FAC (ops/mixed.BF16Weights): the numerics of '
                         'autocast without its ~110 per-tensor cast launches per step, two '
                         'grouped cast launches instead')
    ap.add_argument('--ddp', action='store_true',
                    help='eager torch DDP instead of the graphed flat-arena all-reduce')
    return ap.parse_args()


def _mark(device):
    if device.type == 'cuda':
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev
    return time.perf_counter()


def step_kind(pre):
    if pre is None:
        return 'plain'
    p = pre.param_groups[0]
    if p['step'] % p['inv_update_freq'] == 0:
        return 'inverse'
    if p['step'] % p['factor_update_freq'] == 0:
        return 'factor'
    return 'plain'


def time_sgd_only(args, model, opt, pre, forward_backward, grad_sync, use_graphs, device,
                  communicate=None, stream=None, weights=None):
    """The same training step without K-FAC (hooks removed, plain SGD update),
    timed over the same number of steps: the baseline for kfac_step_ms."""
    pre.remove_hooks()

    def update():
        opt.step()
        if weights is not None:
            weights.master_to_model()

    if grad_sync is not None:
        step = graphs.GraphedTrainStep(None, None, [opt], enabled=use_graphs,
                                       forward_backward=forward_backward,
                                       communicate=communicate or grad_sync, update=update,
                                       stream=stream)
    else:
        def train_step():
            loss = forward_backward()
            update()
            return loss
        step = graphs.GraphedTrainStep(train_step, None, [opt], enabled=use_graphs,
                                       stream=stream)
    for _ in range(3):
        step()
    step.prepare()
    if dist.is_initialized():
        dist.barrier()
    if device.type == 'cuda':
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if device.type == 'cuda':
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()) / args.steps * 1e3


def main():
    args = parse()
    device = launch.init_distributed()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if world != args.gpus and rank == 0:
        print('warning: --gpus {} but world size {}'.format(args.gpus, world), file=sys.stderr)
    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True

    model = resnet.get_model(args.model).to(device)
    mf = torch.channels_last if args.channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    use_graphs = bool(args.graphs) and device.type == 'cuda' and not args.profile_phases
    grad_sync = None
    # bf16-stored weights + fp32 masters (autocast numerics, two grouped cast
    # launches per step instead of one per tensor and direction); the masters
    # are derived after rank 0's weights are broadcast
    weights = None
    if args.bf16_weights and device.type == 'cuda' and use_graphs and not args.ddp \
            and not args.overlap_precond:
        if world > 1:
            grad_sync_mod.GradientAllreduce.broadcast_model(model)
        weights = mixed.BF16Weights(model)
    bcast = None if weights is not None else 0
    if args.ddp or not use_graphs:
        model = launch.wrap_ddp(model, device, broadcast_buffers=False)
    elif world > 1 and args.overlap_grad_comm and hasattr(model, 'forward_bottom'):
        # backward in two graph segments; the top half's all-reduce runs
        # while the bottom half's backward replays (parallel/overlap.py)
        grad_sync = overlap.SplitBackward(
            model, lambda out: F.cross_entropy(out, y, label_smoothing=0.1), lambda: x,
            autocast=torch.bfloat16, weights=weights, broadcast_from=bcast)
    elif world > 1:
        # one flat-arena all-reduce between graph replays (parallel/grad_sync.py)
        grad_sync = grad_sync_mod.GradientAllreduce(
            model, params=weights.parameters(model) if weights is not None else None,
            broadcast_from=bcast)
    base_lr = 0.0125 * world
    sgd_kw = dict(lr=base_lr, momentum=0.9, weight_decay=5e-5)
    if args.fused_sgd and device.type == 'cuda':
        sgd_kw['fused'] = True
    opt = torch.optim.SGD(weights.parameters(model) if weights is not None
                          else model.parameters(), **sgd_kw)
    pre = None
    if not args.no_kfac:
        method = {'comm-opt': kfac.CommMethod.COMM_OPT, 'mem-opt': kfac.CommMethod.MEM_OPT,
                  'hybrid-opt': kfac.CommMethod.HYBRID_OPT}[args.comm_method]
        pre = kfac.KFAC(model, damping=args.damping, factor_decay=0.95,
                        factor_update_freq=args.kfac_cov_update_freq,
                        inv_update_freq=args.kfac_update_freq, kl_clip=args.kl_clip, lr=base_lr,
                        comm_method=method, grad_worker_fraction=args.grad_worker_fraction,
                        distribute_layer_factors=False, eigen_solver=args.eigen_solver,
                        assignment_strategy=args.assignment_strategy,
                        profile=args.profile_phases, precond_precision=args.precond_precision,
                        compute_factor_in_hook=grad_sync is not None,
                        inverse_lag=args.inverse_lag,
                        overlap_precondition=bool(args.overlap_precond) and world == 1,
                        early_factors=bool(args.early_factors),
                        use_hip_graphs=not os.environ.get('KFAC_NO_TAIL_GRAPH'))
        if weights is not None:
            pre.set_grad_params(weights.grad_params())

    B, S = args.batch_size, args.image_size
    g = torch.Generator(device=device).manual_seed(rank)
    x = torch.randn(B, 3, S, S, device=device, generator=g).to(memory_format=mf)
    y = torch.randint(0, 1000, (B,), device=device, generator=g)

    def forward_backward():
        if grad_sync is not None:
            grad_sync.zero_grad()            # one fill of the gradient arena
            if weights is not None:
                weights.zero_model_grads()
        elif weights is not None:
            # the module gradients (bf16 weights, fp32 BN); the masters' .grad
            # is overwritten by grads_to_master
            model.zero_grad(set_to_none=bool(args.set_to_none))
        else:
            opt.zero_grad(set_to_none=bool(args.set_to_none))
        with torch.autocast(device_type=device.type, dtype=torch.bfloat16):
            out = model(x)
            loss = F.cross_entropy(out, y, label_smoothing=0.1)
        loss.backward()
        if weights is not None:
            weights.grads_to_master()
        return loss

    def update():
        if pre is not None:
            pre.step()
        opt.step()
        if weights is not None:
            weights.master_to_model()

    def train_step():
        loss = forward_backward()
        update()
        return loss

    split = isinstance(grad_sync, overlap.SplitBackward)
    fb_segments = grad_sync.segments if split else forward_backward
    comm_segments = grad_sync.communicate if split else grad_sync
    if grad_sync is not None:
        # phased_update: MEM_OPT / HYBRID_OPT plain steps replay as two graphs
        # around the gradient all-gather instead of running eagerly
        step = graphs.GraphedTrainStep(None, pre, [opt], enabled=use_graphs,
                                       forward_backward=fb_segments,
                                       communicate=comm_segments, update=update,
                                       phased_update=True,
                                       post_update=weights.master_to_model
                                       if weights is not None else None)
    else:
        # forward_backward / update as well: inverse steps replay a forward/
        # backward graph (factors in its captured hooks), only the update is eager
        step = graphs.GraphedTrainStep(train_step, pre, [opt], enabled=use_graphs,
                                       forward_backward=forward_backward, update=update)

    for _ in range(args.warmup):
        step()
    step.prepare()   # capture every graphed step kind outside the timed window
    if pre is not None:
        pre.param_groups[0]['step'] = 0
        pre.timer.reset()
    if dist.is_initialized():
        dist.barrier()
    if device.type == 'cuda':
        if os.environ.get('KFAC_PROFILE_MARKER'):
            torch.cuda._sleep(1000)   # 'spin' kernel: start of the timed window in a trace
        torch.cuda.synchronize()
    # per-step device time by step kind: events between steps (graphs stay on)
    kinds, events = [], []
    kfac_comm = kfac.comm.backend
    coll_by_kind = {}
    t0 = time.perf_counter()
    for i in range(args.steps):
        kinds.append(step_kind(pre))
        events.append(_mark(device))
        c0 = kfac_comm.counters() if (kfac_comm is not None and kinds[-1] not in coll_by_kind) \
            else None
        loss = step()
        if c0 is not None:
            # the K-FAC collectives this step kind issued (host-side counters)
            c1 = kfac_comm.counters()
            coll_by_kind[kinds[-1]] = {k: [v[0] - c0.get(k, (0, 0))[0], v[1] - c0.get(k, (0, 0))[1]]
                                       for k, v in c1.items() if v != c0.get(k)}
        if args.check_finite:
            kl = float(pre.fused.kl) if (pre is not None and pre.fused is not None) else 0.0
            print('step', i, 'loss', float(loss.item()), 'kl', kl, flush=True)
    if pre is not None:
        pre.wait_inverses()   # a lagged solve launched in the window is timed in full
    events.append(_mark(device))
    if device.type == 'cuda':
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if device.type == 'cuda' and os.environ.get('KFAC_PROFILE_MARKER'):
        torch.cuda._sleep(1000)   # end of the timed window (the SGD-only run follows)
    per_kind = {}
    for k, a, b in zip(kinds, events[:-1], events[1:]):
        per_kind.setdefault(k, []).append(a.elapsed_time(b) if device.type == 'cuda'
                                          else (b - a) * 1e3)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    ms = elapsed / args.steps * 1e3
    gbatch = B * world
    value = gbatch * args.steps / elapsed
    phases = pre.timer.summary() if (pre is not None and args.profile_phases) else None
    sgd_ms = None
    if pre is not None and args.sgd_delta:
        # same capture stream as the K-FAC run: the model's AccumulateGrad
        # nodes live on it (a new stream makes every backward sync across)
        sgd_ms = time_sgd_only(args, model, opt, pre, fb_segments, grad_sync, use_graphs,
                               device, communicate=comm_segments,
                               stream=getattr(step, 'side', None), weights=weights)
    if rank == 0:
        rec = {
            'metric': METRIC if pre is not None else 'images/sec (whole node) ResNet-50 SGD-only',
            'value': round(value, 2),
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'bf16',
            'data': 'synthetic (random ImageNet-shaped 3x224x224 images, random labels, '
                    'random-init weights)',
            'config': {'model': args.model, 'global_batch': gbatch, 'per_gpu_batch': B,
                       'image_size': S, 'seq_len': None, 'parallelism': 'dp{}'.format(world),
                       'kfac': None if pre is None else {
                           'comm_method': args.comm_method,
                           'assignment_strategy': args.assignment_strategy,
                           'factor_update_freq': args.kfac_cov_update_freq,
                           'inv_update_freq': args.kfac_update_freq,
                           'damping': args.damping, 'kl_clip': args.kl_clip,
                           'precond_precision': args.precond_precision,
                           'inverse_lag': args.inverse_lag,
                           'overlap_precondition': bool(args.overlap_precond) and world == 1,
                           'early_factors': bool(args.early_factors),
                           'early_inverse_launches': pre.early_inverse_launches},
                       'hip_graphs': use_graphs,
                       'fused_sgd': bool(args.fused_sgd and device.type == 'cuda'),
                       'weights': 'bf16 + fp32 masters' if weights is not None
                                  else 'fp32 (autocast casts)',
                       'grad_allreduce': 'ddp' if grad_sync is None and world > 1 else
                                         (('split-backward-overlap' if split else 'flat-arena')
                                          if world > 1 else None),
                       'final_loss': round(float(loss.item()), 4)},
        }
        if per_kind:
            rec['step_ms_by_kind'] = {k: round(sum(v) / len(v), 3) for k, v in per_kind.items()}
            rec['steps_by_kind'] = {k: len(v) for k, v in per_kind.items()}
        if pre is not None and sgd_ms is not None:
            rec['sgd_only_ms_per_step'] = round(sgd_ms, 3)
            kk = {k: round(sum(v) / len(v) - sgd_ms, 3) for k, v in per_kind.items()}
            ff, inv = args.kfac_cov_update_freq, args.kfac_update_freq
            mix = {'inverse': 1.0 / inv, 'factor': (inv // ff - 1.0) / inv}
            mix['plain'] = 1.0 - mix['inverse'] - mix['factor']
            steady = sum(mix[k] * (sum(v) / len(v)) for k, v in per_kind.items()) \
                if set(per_kind) >= set(mix) else None
            rec['kfac_step_ms'] = {
                'window_mean': round(ms - sgd_ms, 3),
                'by_kind': kk,
                'steady_state_mix': None if steady is None else round(steady - sgd_ms, 3),
                'steady_state_images_per_sec': None if steady is None else
                round(gbatch * 1e3 / steady, 1),
                'note': 'K-FAC cost per step over the same model/steps without K-FAC; '
                        'steady_state_mix weights the measured kinds by the reference '
                        'schedule (1 inverse + {} factor steps per {})'.format(
                            inv // ff - 1, inv)}
        if pre is not None and world == 1 and args.model == 'resnet50' and B == 32:
            # BASELINE.md publishes no number (vs_baseline stays null); the
            # reference K-FAC itself, timed the same way on one MI355X
            # (scripts/bench_reference.py, profiles/r2_reference_kfac_mi355x.log)
            rec['reference_kfac_same_gpu'] = {
                'source': 'stale constant: reference K-FAC measured by the builders in round 2 '
                          '(profiles/r2_reference_kfac_mi355x.log), not re-run by this bench; '
                          'the images/sec speedup includes model-side work, the K-FAC-only '
                          'comparison is kfac_cost_ms_by_kind',
                'images_per_sec': REFERENCE_MI355X_IMG_S,
                'speedup': round(value / REFERENCE_MI355X_IMG_S, 2)}
            if sgd_ms is not None and per_kind:
                # K-FAC's own cost per step kind (step minus the same model's
                # SGD-only step), ours vs the reference's: separates the K-FAC
                # speedup from the model-side one (graphs, channels_last, BN)
                ours = {k: round(sum(v) / len(v) - sgd_ms, 3) for k, v in per_kind.items()}
                rec['reference_kfac_same_gpu']['kfac_cost_ms_by_kind'] = {
                    k: {'ours': ours[k],
                        'reference': round(REFERENCE_MI355X_STEP_MS[k] - REFERENCE_MI355X_SGD_MS, 3),
                        'speedup': round((REFERENCE_MI355X_STEP_MS[k] - REFERENCE_MI355X_SGD_MS) /
                                         max(ours[k], 1e-3), 2)}
                    for k in ours if k in REFERENCE_MI355X_STEP_MS}
        if pre is not None:
            # how the communication was built and what it moved: lets a
            # multi-GPU record be checked from itself (RCCL world size, split vs
            # new_group communicators, bucket / arena bytes, calls per step kind)
            cs = pre.comm_summary()
            cs['kfac_collectives_per_step_kind'] = coll_by_kind
            if grad_sync is not None:
                syncs = [grad_sync.sync_top, grad_sync.sync_bottom] if split else [grad_sync]
                cs['grad_allreduce'] = {
                    'kind': 'split-backward-overlap' if split else 'flat-arena',
                    'calls_per_step': sum(len(sy.arenas) for sy in syncs) if world > 1 else 0,
                    'arena_bytes': [a.numel() * a.element_size() for sy in syncs
                                    for a in sy.arenas]}
            elif world > 1:
                cs['grad_allreduce'] = {'kind': 'ddp'}
            rec['comm'] = cs
        if phases is not None:
            rec['kfac_phase_ms_total'] = {k: round(v, 2) for k, v in phases.items()}
            rec['kfac_phase_ms_per_step'] = round(sum(phases.values()) / args.steps, 3)
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
