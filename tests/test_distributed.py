"""Multi-process K-FAC on CPU with gloo (world 2 and 4), 127.0.0.1 rendezvous.

Strategy equivalence: with identical data on
every rank, COMM_OPT / MEM_OPT / HYBRID_OPT must reproduce the single-process
preconditioned gradients and factors BIT-FOR-BIT on every rank (the reference
achieves this once its eigenvector-contiguity bug is fixed).  Also covers the
flat-arena gradient all-reduce used by the graphed bench and bench.py's
distributed path end to end.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import distributed_kfac_pytorch_amd as kfac
from tests import _dist_worker
from tests._oracle_common import build_case, run_steps


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, tmp_path, cfg):
    mp.spawn(fn, args=(world, _port(), str(tmp_path), cfg), nprocs=world, join=True)


def _single(cfg):
    # the ranks run single-threaded; the BLAS reduction order (and so the last
    # bit of every matmul) depends on the thread count
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        return _single_run(cfg)
    finally:
        torch.set_num_threads(threads)


def _single_run(cfg):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': cfg['steps']})
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=cfg.get('inv_freq', 2),
                    lr=0.05, damping=0.003, precompute_outer_eigen=cfg.get('prediv', True),
                    use_eigen_decomp=cfg.get('eigen', True),
                    inverse_lag=cfg.get('lag', 0))
    return run_steps(model, pre, data, cfg['steps'])


CASES = [
    (2, {'method': 'COMM_OPT'}),
    (2, {'method': 'MEM_OPT'}),
    (4, {'method': 'HYBRID_OPT', 'fraction': 0.5}),
    (4, {'method': 'HYBRID_OPT', 'fraction': 0.25}),
    (4, {'method': 'COMM_OPT', 'prediv': False}),
    (2, {'method': 'COMM_OPT', 'eigen': False}),
    (4, {'method': 'MEM_OPT', 'eigen': False}),
    # world 8 = one MI355X node's rank count
    (8, {'method': 'COMM_OPT'}),
    (8, {'method': 'MEM_OPT'}),
    (8, {'method': 'HYBRID_OPT', 'fraction': 0.25}),
    # the batched-solver assignment (set-valued rank cost + arena byte balance)
    (4, {'method': 'COMM_OPT', 'assign': 'batched'}),
    (4, {'method': 'HYBRID_OPT', 'fraction': 0.5, 'assign': 'batched', 'distribute': True,
         'prediv': False}),
]


@pytest.mark.parametrize('world,cfg', CASES,
                         ids=['-'.join([str(w)] + ['{}={}'.format(k, v) for k, v in c.items()])
                              for w, c in CASES])
def test_strategy_equivalence(tmp_path, world, cfg):
    cfg = dict(cfg, steps=4)
    ref_grads, ref_factors = _single(cfg)
    _spawn(_dist_worker.kfac_strategy, world, tmp_path, cfg)
    # world 2 and 4: the averaged sum of identical tensors is exact (x+x,
    # (x+x)+(x+x)), so every strategy is BIT-identical to world 1.  World 8:
    # gloo's ring accumulates 3x, 5x, ... which round, so the factors differ
    # from world 1 in the last bit (~1e-8); there the ranks must still agree
    # bit for bit with each other and match world 1 to fp32 round-off.
    exact = world in (2, 4)

    def same(a, b):
        return torch.equal(a, b) if exact else torch.allclose(a, b, rtol=1e-4, atol=1e-6)

    res0 = None
    for r in range(world):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
        for step, (gs, rs) in enumerate(zip(res['grads'], ref_grads)):
            for a, b in zip(gs, rs):
                assert same(a, b), (r, step, (a - b).abs().max().item())
        for (a, g), (ra, rg) in zip(res['factors'], ref_factors):
            assert same(a, ra) and same(g, rg)
        if res0 is None:
            res0 = res
        else:
            for gs, g0 in zip(res['grads'], res0['grads']):
                assert all(torch.equal(a, b) for a, b in zip(gs, g0)), r
        # one collective per distribution (round 2): the eigendata of every
        # owner in ONE all-gather per inverse step, the MEM/HYBRID gradients
        # in ONE all-gather per step
        calls = res['calls']
        gw = max(1, int(round(world * {'COMM_OPT': 1.0, 'MEM_OPT': 0.0}.get(
            cfg['method'], cfg.get('fraction', 0.25)))))
        if cfg['method'] != 'MEM_OPT':
            # inverse groups of gw ranks: one all-gather when gw > 1 (none for
            # a group that owns no factor: more groups than layers)
            want = 1 if (gw > 1 and not res['eig_empty']) else 0
            assert calls['eig'] and all(c == want for c in calls['eig']), calls
        if cfg['method'] != 'COMM_OPT':
            # gradient groups of world / gw ranks
            assert calls['grad'] and all(c == (1 if gw < world else 0)
                                         for c in calls['grad']), calls


SPLIT_CASES = [{'method': 'COMM_OPT'}, {'method': 'MEM_OPT'},
               {'method': 'HYBRID_OPT', 'fraction': 0.25}]


@pytest.mark.parametrize('cfg', SPLIT_CASES, ids=[c['method'] for c in SPLIT_CASES])
def test_comm_split_path_world8(tmp_path, cfg):
    """The RCCL ncclCommSplit construction (comm._can_split() true,
    dist.split_group) rehearsed on gloo at world 8: every rank issues the
    same split sequence (K-FAC world from the default group, then one split
    of the K-FAC world per partition with more than one multi-rank group),
    the partitions are the reference's (tests/worker_allocator.py goldens),
    and the strategies still match world 1 (kfac/comm.py:53-64)."""
    world = 8
    cfg = dict(cfg, steps=3)
    ref_grads, ref_factors = _single(cfg)
    _spawn(_dist_worker.kfac_split_strategy, world, tmp_path, cfg)
    res = [torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=False)
           for r in range(world)]
    splits0 = res[0]['splits']
    assert splits0[0] == {'parent': 'default', 'split_ranks': [list(range(world))],
                          'desc': 'kfac_world'}, splits0
    for r in range(world):
        assert res[r]['splits'] == splits0, (r, res[r]['splits'], splits0)
        assert res[r]['build_log'] == res[0]['build_log']
        assert res[r]['kfac_world'] == {'size': world, 'built_by': 'split_group'}
        for gs, rs in zip(res[r]['grads'], ref_grads):
            for a, b in zip(gs, rs):
                assert torch.allclose(a, b, rtol=1e-4, atol=1e-6), (r, (a - b).abs().max())
        for gs, g0 in zip(res[r]['grads'], res[0]['grads']):
            assert all(torch.equal(a, b) for a, b in zip(gs, g0)), r
    subs = [c for c in splits0[1:]]
    assert all(c['parent'] == 'kfac_world' and c['desc'] == 'kfac_sub' for c in subs), subs
    got = [c['split_ranks'] for c in subs]
    if cfg['method'] == 'HYBRID_OPT':
        # grad_workers = 2: inverse groups of 2 contiguous ranks, gradient
        # groups of 4 strided ranks (reference goldens)
        assert [[0, 1], [2, 3], [4, 5], [6, 7]] in got, got
        assert [[0, 2, 4, 6], [1, 3, 5, 7]] in got, got
    else:
        # COMM_OPT: inverse group = world, gradient groups singletons; MEM_OPT:
        # the reverse -- no partition has a multi-rank group below the world
        assert got == [], got


def test_distribute_layer_factors_without_prediv(tmp_path):
    """A and G of a layer on different ranks (reference default for COMM_OPT
    once prediv is off): still bit-identical."""
    cfg = {'method': 'COMM_OPT', 'prediv': False, 'distribute': True, 'steps': 3}
    ref_grads, _ = _single(cfg)
    _spawn(_dist_worker.kfac_strategy, 2, tmp_path, cfg)
    for r in range(2):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
        for gs, rs in zip(res['grads'], ref_grads):
            for a, b in zip(gs, rs):
                assert torch.equal(a, b)


def test_gradient_allreduce(tmp_path):
    world = 2
    _spawn(_dist_worker.grad_allreduce, world, tmp_path, {})
    res = [torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
           for r in range(world)]
    for r in range(world):
        assert res[r]['views_ok']
        for p, p0 in zip(res[r]['params0'], res[0]['params0']):
            assert torch.equal(p, p0)        # broadcast from rank 0
        for a, l0, l1 in zip(res[r]['avg'], res[0]['local'], res[1]['local']):
            assert torch.allclose(a, (l0 + l1) / 2, atol=1e-7, rtol=1e-6)


@pytest.mark.parametrize('method', ['comm-opt', 'hybrid-opt'])
def test_bench_distributed_cpu(tmp_path, method):
    """bench.py prints ONE JSON line on rank 0 with the whole-job throughput."""
    argv = ['--gpus', '2', '--steps', '2', '--warmup', '1', '--model', 'resnet_tiny',
            '--batch-size', '2', '--image-size', '32', '--comm-method', method,
            '--kfac-update-freq', '2', '--kfac-cov-update-freq', '1']
    _spawn(_dist_worker.bench_cpu, 2, tmp_path, {'argv': argv})
    out0 = open(os.path.join(str(tmp_path), 'rank0.txt')).read().strip().splitlines()
    out1 = open(os.path.join(str(tmp_path), 'rank1.txt')).read().strip()
    assert out1 == ''
    assert len(out0) == 1
    rec = json.loads(out0[0])
    assert rec['n_gpus'] == 2 and rec['steps'] == 2 and rec['warmup'] == 1
    assert rec['config']['global_batch'] == 4
    assert rec['value'] > 0 and rec['config']['parallelism'] == 'dp2'


@pytest.mark.parametrize('method,mode', [('COMM_OPT', 'clean'), ('MEM_OPT', 'clean'),
                                         ('COMM_OPT', 'skip_allreduce'),
                                         ('COMM_OPT', 'corrupt_eigendata')])
def test_comm_consistency_check(tmp_path, method, mode):
    """Debug mode: cross-rank checksums after each collective
    phase pass on clean runs and name the buffers of a sabotaged one."""
    _spawn(_dist_worker.comm_check, 2, tmp_path, {'method': method, 'mode': mode})
    errs = [torch.load(os.path.join(tmp_path, 'rank{}.pt'.format(r)))['err'] for r in range(2)]
    if mode == 'clean':
        assert errs == [None, None], errs
    elif mode == 'skip_allreduce':
        assert all(e is not None and 'factor all-reduce' in e and '.A' in e for e in errs), errs
    else:
        assert all(e is not None and 'eigendata broadcast' in e and '0:' in e for e in errs), errs


def test_split_backward_overlap_equals_single(tmp_path):
    """The overlapped gradient all-reduce (backward in two segments, the top
    half's all-reduce issued before the bottom half's backward) gives exactly
    the gradients of one backward + one flat-arena all-reduce."""
    _spawn(_dist_worker.split_backward, 2, tmp_path, {})
    for r in range(2):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
        assert res['same'], res
        assert res['loss'][0] == res['loss'][1]


def test_split_backward_bf16_weights_equals_autocast(tmp_path):
    """bf16-stored weights + fp32 masters through the overlapped two-segment
    all-reduce give the gradients of fp32 weights under bf16 autocast."""
    _spawn(_dist_worker.split_backward_bf16_weights, 2, tmp_path, {})
    for r in range(2):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
        assert res['same'], res
        assert res['loss'][0] == res['loss'][1]


def test_deferred_factor_allreduce(tmp_path):
    """Verdict r2 item 3: the factor all-reduce is issued in step() and
    joined only by its consumers (next EMA / inverse update / state_dict):
    no wait inside step() on factor-only steps, results bit-identical to the
    joined-in-step schedule, ranks agree."""
    _spawn(_dist_worker.deferred_factor_comm, 2, tmp_path, {})
    outs = [torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=False)
            for r in range(2)]
    for o in outs:
        rec = o[True]['record']
        # step 0: factor + inverse step: joined by the inverse update inside step()
        assert rec[0] == (0, False, 1), rec
        # step 2: factor-only: still in flight after step(), no wait inside it
        assert rec[2] == (2, True, 0), rec
        assert rec[3] == (3, True, 0), rec        # plain step: untouched
        # step 4: the EMA joins step 2's all-reduce, the inverse update joins step 4's
        assert rec[4] == (4, False, 2), rec
        assert o[False]['record'][2] == (2, False, 1)
        for (a1, g1), (a2, g2) in zip(o[True]['factors'], o[False]['factors']):
            assert torch.equal(a1, a2) and torch.equal(g1, g2)
        for p1, p2 in zip(o[True]['params'], o[False]['params']):
            assert torch.equal(p1, p2)
    for (a0, g0), (a1, g1) in zip(outs[0][True]['factors'], outs[1][True]['factors']):
        assert torch.equal(a0, a1) and torch.equal(g0, g1)


def test_example_graphs_path_world2(tmp_path):
    """Verdict r2 item 7: the examples' fast path (--graphs 1) at world 2 on
    gloo trains like the eager DDP loop (same losses to fp32 rounding)."""
    for g in (1, 0):
        _spawn(_dist_worker.example_graphs, 2, tmp_path, {'graphs': g})
    h1 = torch.load(os.path.join(str(tmp_path), 'rank0_g1.pt'), weights_only=False)
    h0 = torch.load(os.path.join(str(tmp_path), 'rank0_g0.pt'), weights_only=False)
    a, b = h1[0]['train'], h0[0]['train']
    assert abs(a['loss'] - b['loss']) <= 1e-5 * max(1.0, abs(b['loss'])), (a, b)
    assert abs(h1[0]['val']['loss'] - h0[0]['val']['loss']) <= 1e-4, (h1, h0)


COUNT_CASES = [{'method': 'COMM_OPT'}, {'method': 'MEM_OPT'},
               {'method': 'HYBRID_OPT', 'fraction': 0.25}]


def _expected_collectives(world, method, fraction, layers, a_locs, g_locs, rank, prediv=True):
    """What each step kind must issue on `rank`, derived from the reference's
    group layout (kfac/utils.py:59-159: inverse groups = contiguous blocks of
    gw ranks, gradient groups = stride gw) and the layer sizes alone:
      factor steps   ONE SUM all-reduce of every factor's upper triangle, fp32
                     (the triu-packed bucket, X1/X2; one bucket at 64 MB)
      inverse steps  + ONE all-gather of the inverse group's eigendata arena:
                     an equal 64-element-aligned slot per group rank, sized
                     by the largest owner's QA + QG + dGdA (X3)
      every step     (MEM_OPT / HYBRID) ONE all-gather of the gradient arena
                     over the gradient group: an equal slot per block of gw
                     ranks, sized by the largest block's gradients (X5)."""
    gw = max(1, int(round(world * {'COMM_OPT': 1.0, 'MEM_OPT': 0.0}.get(method, fraction))))
    tri = sum(L['nA'] * (L['nA'] + 1) // 2 + L['nG'] * (L['nG'] + 1) // 2 for L in layers)
    factor = {'all_reduce': [1, 4 * tri]}
    out = {'plain': {}, 'factor': dict(factor), 'inverse': dict(factor)}
    inv_group = list(range(rank // gw * gw, rank // gw * gw + gw))
    if method != 'MEM_OPT' and gw > 1:
        owned = {o: 0 for o in inv_group}
        for L, a, g in zip(layers, a_locs, g_locs):
            items = [('A', L['nA'] ** 2), ('G', L['nG'] ** 2)]
            items += [('A', L['nG'] * L['nA'])] if prediv else [('A', L['nA']), ('G', L['nG'])]
            for f, n in items:
                o = a if f == 'A' else g
                if o in owned:
                    owned[o] += n
        slot = (max(owned.values()) + 63) // 64 * 64
        if slot:      # a group that owns no factor issues nothing
            out['inverse']['all_gather_into_tensor'] = [1, 4 * slot * gw]
    if method != 'COMM_OPT' and gw < world:
        nblocks = world // gw
        sizes = [0] * nblocks
        for L, a in zip(layers, a_locs):
            sizes[a // gw] += L['grad_numel']
        gbytes = 4 * nblocks * ((max(sizes) + 63) // 64 * 64)
        for k in out:
            # gradient and eigendata all-gathers share the counter key
            prev = out[k].get('all_gather_into_tensor', [0, 0])
            out[k]['all_gather_into_tensor'] = [prev[0] + 1, prev[1] + gbytes]
    return out


@pytest.mark.parametrize('cfg', COUNT_CASES, ids=[c['method'] for c in COUNT_CASES])
def test_collectives_per_step_kind_world8(tmp_path, cfg):
    """The exact K-FAC collective calls and bytes of each step kind at world
    8 (one MI355X node's ranks), per rank, against an expectation built from
    the reference's group layout and the layer sizes -- the numbers the
    bench's comm.kfac_collectives_per_step_kind reports, so the first RCCL
    scaling record can be checked against this test line for line."""
    world = 8
    _spawn(_dist_worker.kfac_collective_counts, world, tmp_path, cfg)
    for r in range(world):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=False)
        exp = _expected_collectives(world, cfg['method'], cfg.get('fraction', 0.25),
                                    res['layers'], res['a_locs'], res['g_locs'], r)
        assert sorted(res['by_kind']) == ['factor', 'inverse', 'plain'], res['by_kind']
        for kind, deltas in res['by_kind'].items():
            for d in deltas:
                assert d == exp[kind], (r, kind, d, exp[kind])
