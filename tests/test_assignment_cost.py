"""assignment_strategy='measured' (MI355X cost table) vs the reference's n^3
(kept as 'compute' for the goldens): ResNet-50's 108 factors over 8 ranks."""
import torch.nn as nn

from distributed_kfac_pytorch_amd import preconditioner as P
from distributed_kfac_pytorch_amd.models import resnet
from distributed_kfac_pytorch_amd.utils import distribution


def _resnet50_layers():
    """(nA, nG) of every K-FAC layer of ResNet-50 (convs without bias, fc with)."""
    out = []
    for m in resnet.resnet50().modules():
        if isinstance(m, nn.Conv2d):
            kh, kw = m.kernel_size
            out.append((m.in_channels * kh * kw + (m.bias is not None), m.out_channels))
        elif isinstance(m, nn.Linear):
            out.append((m.in_features + (m.bias is not None), m.out_features))
    return out


def _rank_costs(strategy, world=8):
    layers = _resnet50_layers()
    cost = P.assignment_cost(strategy)
    work = [cost(a) + cost(g) for a, g in layers]       # A and G of a layer on one rank
    locs = distribution.load_balance(world, work)
    true = P.measured_cost
    ranks = [0.0] * world
    for (a, g), r in zip(layers, locs):
        ranks[r] += true(a) + true(g)
    return ranks


def test_resnet50_has_108_factors():
    assert len(_resnet50_layers()) * 2 == 108


def test_measured_strategy_balances_8_ranks():
    ranks = _rank_costs('measured')
    mean = sum(ranks) / len(ranks)
    assert max(ranks) <= 1.3 * mean, (max(ranks), mean, ranks)


def test_compute_strategy_kept_for_goldens():
    assert P.assignment_cost('compute')(10) == 1000
    assert P.assignment_cost('memory')(10) == 100
    # n^3 overloads the ranks holding the 4608 factors against the measured cost
    ranks = _rank_costs('compute')
    assert max(ranks) > max(_rank_costs('measured'))


def _batched_sets(world, strategy):
    layers = _resnet50_layers()
    nbytes = [4 * (a * a + g * g + a * g) for a, g in layers]
    if strategy == 'batched':
        locs = distribution.balance_batched(world, [[a, g] for a, g in layers], P.batched_cost,
                                            nbytes)
    else:
        cost = P.assignment_cost(strategy)
        locs = distribution.load_balance(world, [cost(a) + cost(g) for a, g in layers])
    sets = [[] for _ in range(world)]
    loads = [0] * world
    for (a, g), r, b in zip(layers, locs, nbytes):
        sets[r] += [a, g]
        loads[r] += b
    return sets, loads, locs


def test_batched_strategy_arena_padding_bound_w8():
    """Verdict r2 item 4: the padded eigen arena at W=8 stays within 10 % of
    the real eigendata (27 % with the additive 'measured' LPT)."""
    _, loads, _ = _batched_sets(8, 'batched')
    pad = 8 * max(loads) / float(sum(loads)) - 1.0
    assert pad <= 0.10, pad
    _, loads_m, _ = _batched_sets(8, 'measured')
    assert 8 * max(loads_m) / float(sum(loads_m)) - 1.0 > pad


def test_batched_strategy_makespan_not_worse():
    """Under the batched per-rank model the 'batched' assignment's slowest
    rank is no slower than the additive LPT's, at every W."""
    for world in (2, 4, 8):
        sb, _, _ = _batched_sets(world, 'batched')
        sm, _, _ = _batched_sets(world, 'measured')
        tb = max(P.batched_cost(s) for s in sb)
        tm = max(P.batched_cost(s) for s in sm)
        assert tb <= tm + 1e-9, (world, tb, tm)


def test_batched_assignment_is_deterministic_and_complete():
    a = _batched_sets(8, 'batched')[2]
    b = _batched_sets(8, 'batched')[2]
    assert a == b
    assert sorted(set(a)) == list(range(8))


def test_batched_cost_is_a_set_function():
    # a rank's time is set by its largest factor's chain, not the sum
    one = P.batched_cost([4608])
    three = P.batched_cost([4608, 4608, 4608])
    assert three < 3 * one
    assert P.batched_cost([]) == 0.0
