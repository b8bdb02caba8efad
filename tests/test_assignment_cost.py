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
