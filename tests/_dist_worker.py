"""Worker bodies for the multi-process (gloo, CPU) tests in test_distributed.py.

Each function runs inside one spawned rank, writes its results with
torch.save into `out_dir`, and never raises silently (an exception in a rank
makes torch.multiprocessing.spawn fail the test).
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _init(rank, world, port):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(world)
    os.environ['LOCAL_RANK'] = str(rank)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from distributed_kfac_pytorch_amd import comm
    comm.reset_comm_backend()
    comm.init_comm_backend()


def _count_collectives(pre):
    """Record how many backend collectives each eigendata / gradient
    distribution issues: {'eig': [n per inverse step], 'grad': [n per step]}."""
    from distributed_kfac_pytorch_amd import comm
    backend = comm.backend
    count = [0]
    for name in ('broadcast', 'allgather_into', 'allreduce', 'allgather', 'reduce'):
        fn = getattr(backend, name)

        def wrapped(*a, _fn=fn, **k):
            count[0] += 1
            return _fn(*a, **k)
        setattr(backend, name, wrapped)
    calls = {'eig': [], 'grad': []}
    for attr, key in (('broadcast_inverses', 'eig'), ('broadcast_gradients', 'grad')):
        orig = getattr(pre, attr)

        def wrapped(_orig=orig, _key=key):
            c0 = count[0]
            _orig()
            calls[_key].append(count[0] - c0)
        setattr(pre, attr, wrapped)
    return calls


def kfac_strategy(rank, world, port, out_dir, cfg):
    """Identical data on every rank: the K-FAC result must equal world=1."""
    _init(rank, world, port)
    import distributed_kfac_pytorch_amd as kfac
    from tests._oracle_common import build_case, run_steps
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': cfg['steps']})
    method = getattr(kfac.CommMethod, cfg['method'])
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=cfg.get('inv_freq', 2),
                    lr=0.05, damping=0.003, comm_method=method,
                    grad_worker_fraction=cfg.get('fraction', 0.25),
                    distribute_layer_factors=cfg.get('distribute', False),
                    precompute_outer_eigen=cfg.get('prediv', True),
                    use_eigen_decomp=cfg.get('eigen', True),
                    inverse_lag=cfg.get('lag', 0),
                    assignment_strategy=cfg.get('assign', 'compute'))
    calls = _count_collectives(pre)
    grads, factors = run_steps(model, pre, data, cfg['steps'])
    torch.save({'grads': grads, 'factors': factors, 'calls': calls,
                'eig_empty': bool(pre.plan is not None and pre.plan.eig_empty)},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def kfac_split_strategy(rank, world, port, out_dir, cfg):
    """The ncclCommSplit path (comm._can_split / dist.split_group) on gloo:
    split_group is replaced by a recorder that builds the same groups with
    new_group, so the construction sequence of every rank can be compared
    and the strategies still checked against world 1."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(world)
    os.environ['LOCAL_RANK'] = str(rank)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from distributed_kfac_pytorch_amd import comm
    calls = []

    def fake_split_group(parent_pg=None, split_ranks=None, timeout=None, pg_options=None,
                         group_desc=None):
        parent = 'default' if parent_pg is None else (
            'kfac_world' if parent_pg is getattr(comm.backend, 'kfac_world', None) else 'other')
        calls.append({'parent': parent, 'split_ranks': [list(r) for r in split_ranks],
                      'desc': group_desc})
        mine = None
        for ranks in split_ranks:           # collective: same order on every rank
            g = dist.new_group(list(ranks))
            if rank in ranks:
                mine = g
        return mine

    dist.split_group = fake_split_group
    comm._can_split = lambda: True
    comm.reset_comm_backend()
    comm.init_comm_backend()
    import distributed_kfac_pytorch_amd as kfac
    from tests._oracle_common import build_case, run_steps
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': cfg['steps']})
    method = getattr(kfac.CommMethod, cfg['method'])
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=cfg.get('inv_freq', 2),
                    lr=0.05, damping=0.003, comm_method=method,
                    grad_worker_fraction=cfg.get('fraction', 0.25),
                    distribute_layer_factors=False)
    grads, factors = run_steps(model, pre, data, cfg['steps'])
    summary = pre.comm_summary()
    torch.save({'grads': grads, 'factors': factors, 'splits': calls,
                'build_log': list(comm.build_log),
                'groups': summary['groups'], 'kfac_world': summary['kfac_world']},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def deferred_factor_comm(rank, world, port, out_dir, cfg):
    """Different data per rank.  The factor all-reduce of a factor-only step
    must stay in flight after step() returns (no wait inside step()), be
    joined by the next consumer, and leave factors bit-identical to the
    joined-inside-step() schedule."""
    _init(rank, world, port)
    import distributed_kfac_pytorch_amd as kfac
    from tests._oracle_common import build_case
    out = {}
    for defer in (True, False):
        model, data = build_case({'seed': 0, 'batch': 6, 'steps': 6})
        pre = kfac.KFAC(model, factor_update_freq=2, inv_update_freq=4, lr=0.05,
                        damping=0.003, defer_factor_comm=defer)
        fa = pre._factor_allreduce
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        g = torch.Generator().manual_seed(100 + rank)
        record = []
        for i in range(6):
            x, y = data[i]
            x = x + 0.1 * torch.randn(x.shape, generator=g)     # rank-specific data
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            w0 = fa.waits
            pre.step()
            record.append((i, fa.pending, fa.waits - w0))
            opt.step()
        sd = pre.state_dict()
        out[defer] = {'record': record,
                      'factors': [(l['A'].clone(), l['G'].clone()) for l in sd['layers']],
                      'params': [p.detach().clone() for p in model.parameters()]}
    torch.save(out, os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def grad_allreduce(rank, world, port, out_dir, cfg):
    """Different data per rank; GradientAllreduce must average gradients and
    start every rank from rank 0's parameters."""
    _init(rank, world, port)
    import torch.nn as nn
    from distributed_kfac_pytorch_amd.parallel.grad_sync import GradientAllreduce
    torch.manual_seed(100 + rank)     # deliberately different initialisation
    model = nn.Sequential(nn.Conv2d(3, 8, 3), nn.ReLU(), nn.Flatten(), nn.Linear(8 * 6 * 6, 5))
    model[0].to(memory_format=torch.channels_last)
    sync = GradientAllreduce(model)
    params0 = [p.detach().clone() for p in model.parameters()]
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(4, 3, 8, 8, generator=g)
    model.zero_grad(set_to_none=False)
    model(x).square().mean().backward()
    local = [p.grad.detach().clone() for p in model.parameters()]
    sync()
    avg = [p.grad.detach().clone() for p in model.parameters()]
    views_ok = all(p.grad.data_ptr() >= sync.arenas[0].data_ptr() for p in model.parameters())
    torch.save({'params0': params0, 'local': local, 'avg': avg, 'views_ok': views_ok},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def bench_cpu(rank, world, port, out_dir, cfg):
    """bench.py's distributed path end to end on CPU/gloo (tiny model)."""
    _init(rank, world, port)
    import subprocess  # noqa: F401  (keeps the import surface identical to the GPU run)
    sys.argv = ['bench.py'] + cfg['argv']
    import runpy
    from contextlib import redirect_stdout
    import io
    buf = io.StringIO()
    with redirect_stdout(buf):
        runpy.run_path(os.path.join(ROOT, 'bench.py'), run_name='__main__')
    with open(os.path.join(out_dir, 'rank{}.txt'.format(rank)), 'w') as f:
        f.write(buf.getvalue())


def comm_check(rank, world, port, out_dir, cfg):
    """KFAC(comm_check=True): clean runs pass; a sabotaged collective (factor
    all-reduce skipped with rank-dependent data, or one rank's eigendata
    perturbed after the broadcast) raises CommConsistencyError."""
    _init(rank, world, port)
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd.utils.comm_check import CommConsistencyError
    from tests._oracle_common import build_case, run_steps
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 3})
    if cfg['mode'] == 'skip_allreduce':
        # rank-dependent inputs: the local factors differ across ranks
        data = [(x + rank, y) for x, y in data]
    method = getattr(kfac.CommMethod, cfg['method'])
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1, lr=0.05, damping=0.003,
                    comm_method=method, comm_check=True)
    if cfg['mode'] == 'skip_allreduce':
        pre.allreduce_factors = lambda: None
    elif cfg['mode'] == 'corrupt_eigendata':
        orig = pre.broadcast_inverses

        def bad_broadcast():
            orig()
            if rank == 1:
                st = pre.layers[0].state
                key = 'QA' if st.get('QA') is not None else 'A_inv'
                st[key].mul_(1.0 + 1e-6)
        pre.broadcast_inverses = bad_broadcast
    err = None
    try:
        run_steps(model, pre, data, 3)
    except CommConsistencyError as e:
        err = str(e)
    torch.save({'err': err}, os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    # no barrier on the error path: the failing check is itself collective, so
    # every rank raised at the same phase
    dist.destroy_process_group()


def split_backward(rank, world, port, out_dir, cfg):
    """parallel/overlap.SplitBackward (two backward segments, two async
    all-reduces) vs one backward + one flat-arena all-reduce: identical."""
    _init(rank, world, port)
    import copy
    import torch.nn.functional as F
    from distributed_kfac_pytorch_amd.models import resnet
    from distributed_kfac_pytorch_amd.parallel.grad_sync import GradientAllreduce
    from distributed_kfac_pytorch_amd.parallel.overlap import SplitBackward
    torch.manual_seed(0)
    m1 = resnet.resnet_tiny(num_classes=10)
    m2 = copy.deepcopy(m1)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(4, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    sb = SplitBackward(m1, lambda out: F.cross_entropy(out, y), lambda: x)
    loss1 = None
    for i, (seg, cm) in enumerate(zip(sb.segments, sb.communicate)):
        out = seg()
        loss1 = out if i == 0 else loss1
        cm()
    ga = GradientAllreduce(m2)
    ga.zero_grad()
    loss2 = F.cross_entropy(m2(x), y)
    loss2.backward()
    ga()
    same = all(torch.equal(p.grad, q.grad) for p, q in zip(m1.parameters(), m2.parameters()))
    torch.save({'same': same, 'loss': (loss1.item(), loss2.item())},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def split_backward_bf16_weights(rank, world, port, out_dir, cfg):
    """SplitBackward over bf16-stored weights (ops/mixed.BF16Weights: each
    segment widens its weight gradients into the fp32 masters, the arenas
    all-reduce the masters' gradients) vs fp32 weights under bf16 autocast
    with one backward + one flat-arena all-reduce: identical gradients."""
    _init(rank, world, port)
    import copy
    import torch.nn.functional as F
    from distributed_kfac_pytorch_amd.models import resnet
    from distributed_kfac_pytorch_amd.ops.mixed import BF16Weights
    from distributed_kfac_pytorch_amd.parallel.grad_sync import GradientAllreduce
    from distributed_kfac_pytorch_amd.parallel.overlap import SplitBackward
    torch.manual_seed(rank)           # ranks start different: rank 0's weights win
    m1 = resnet.resnet_tiny(num_classes=10)
    m2 = copy.deepcopy(m1)
    GradientAllreduce.broadcast_model(m1)
    w = BF16Weights(m1)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(4, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    sb = SplitBackward(m1, lambda out: F.cross_entropy(out, y), lambda: x,
                       autocast=torch.bfloat16, weights=w, broadcast_from=None)
    loss1 = None
    for i, (seg, cm) in enumerate(zip(sb.segments, sb.communicate)):
        out = seg()
        loss1 = out if i == 0 else loss1
        cm()
    ga = GradientAllreduce(m2)       # broadcasts rank 0's fp32 weights
    ga.zero_grad()
    with torch.autocast('cpu', dtype=torch.bfloat16):
        loss2 = F.cross_entropy(m2(x), y)
    loss2.backward()
    ga()
    same = all(torch.equal(w.master_of(p).grad, q.grad)
               for p, q in zip(m1.parameters(), m2.parameters()))
    torch.save({'same': same, 'loss': (loss1.item(), loss2.item())},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()


def example_graphs(rank, world, port, out_dir, cfg):
    """The ImageNet example at world 2 (gloo), --graphs 1 (flat-arena gradient
    all-reduce between step segments, factors in hooks, deferred factor
    all-reduce) vs the reference-style eager DDP loop (--graphs 0)."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(world)
    os.environ['LOCAL_RANK'] = str(rank)
    torch.set_num_threads(1)
    from examples import torch_imagenet_resnet as ex
    argv = ['--model', 'resnet_tiny', '--synthetic-size', '16', '--batch-size', '2',
            '--val-batch-size', '4', '--image-size', '32', '--checkpoint-freq', '0',
            '--epochs', '1', '--kfac-update-freq', '4', '--kfac-cov-update-freq', '2',
            '--log-dir', os.path.join(out_dir, 'log{}'.format(rank)),
            '--graphs', str(cfg['graphs'])]
    hist = ex.main(argv)
    torch.save(hist, os.path.join(out_dir, 'rank{}_g{}.pt'.format(rank, cfg['graphs'])))


def kfac_collective_counts(rank, world, port, out_dir, cfg):
    """The K-FAC collectives each step kind issues on this rank, as bench.py
    reports them (comm.kfac_collectives_per_step_kind: counter deltas of the
    first step of each kind), plus the plan facts an independent expectation
    needs (layer sizes, owners)."""
    _init(rank, world, port)
    import torch.nn as nn
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd import comm
    from tests._oracle_common import build_case
    steps = 6
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': steps})
    pre = kfac.KFAC(model, factor_update_freq=2, inv_update_freq=4, lr=0.05, damping=0.003,
                    comm_method=getattr(kfac.CommMethod, cfg['method']),
                    grad_worker_fraction=cfg.get('fraction', 0.25),
                    precompute_outer_eigen=cfg.get('prediv', True))
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    by_kind = {}
    for i in range(steps):
        p = pre.param_groups[0]
        kind = 'inverse' if p['step'] % p['inv_update_freq'] == 0 else \
            'factor' if p['step'] % p['factor_update_freq'] == 0 else 'plain'
        c0 = comm.backend.counters()
        x, y = data[i]
        opt.zero_grad()
        nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        opt.step()
        c1 = comm.backend.counters()
        delta = {k: [v[0] - c0.get(k, (0, 0))[0], v[1] - c0.get(k, (0, 0))[1]]
                 for k, v in c1.items() if v != c0.get(k)}
        by_kind.setdefault(kind, []).append(delta)
    pre.join_factor_comm()
    layers = [{'nA': l.state['A'].shape[0], 'nG': l.state['G'].shape[0],
               'grad_numel': int(torch.Size(l.grad_shape).numel())} for l in pre.layers]
    torch.save({'by_kind': by_kind, 'layers': layers, 'a_locs': list(pre.plan.a_locs),
                'g_locs': list(pre.plan.g_locs), 'summary': pre.comm_summary()},
               os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    dist.barrier()
    dist.destroy_process_group()
