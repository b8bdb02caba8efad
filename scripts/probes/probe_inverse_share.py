"""Probe: the inverse step at W ranks, projected on ONE GPU.

For W in {1, 2, 4, 8} and the assignment strategies 'measured' (additive
per-factor table + LPT) and 'batched' (set-valued per-rank model + arena byte
balance, KFAC(assignment_strategy='batched')), every rank's factor set of
ResNet-50 (54 layers, A and G of a layer on one rank as in the bench) is
solved alone on this GPU with the production eigensolver (ops/eigen.symeig_many,
random SPD factors of the right sizes).  The slowest rank's time is the
projected inverse-step compute at W (the eigendata all-gather comes on top;
its padded arena size is printed).  All measured sets plus random subsets
then refit BATCHED_COST_MS = (a, b3, b2, b0) of
T(S) = a n_max + b3 sum n^3 + b2 sum n^2 + b0 |S|  (least squares).

    python scripts/probes/probe_inverse_share.py [reps]
"""
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd import preconditioner as P  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402
from distributed_kfac_pytorch_amd.utils import distribution as D  # noqa: E402


def layers():
    out = []
    for m in resnet.resnet50().modules():
        if isinstance(m, torch.nn.Conv2d):
            kh, kw = m.kernel_size
            out.append((m.in_channels * kh * kw + (m.bias is not None), m.out_channels))
        elif isinstance(m, torch.nn.Linear):
            out.append((m.in_features + 1, m.out_features))
    return out


def unit_bytes(a, g):
    return 4 * (a * a + g * g + a * g)     # QA, QG, dGdA (precompute_outer_eigen)


def assign(strategy, W, L):
    if strategy == 'batched':
        return D.balance_batched(W, [[a, g] for a, g in L], P.batched_cost,
                                 [unit_bytes(a, g) for a, g in L])
    cost = P.assignment_cost(strategy)
    return D.load_balance(W, [cost(a) + cost(g) for a, g in L])


_MATS = {}


def mats_for(sizes, dev):
    out = []
    count = {}
    for n in sizes:
        k = (n, count.get(n, 0))
        count[n] = k[1] + 1
        if k not in _MATS:
            g = torch.Generator(device=dev).manual_seed(n * 131 + k[1])
            x = torch.randn(n, max(64, n // 2), device=dev, generator=g)
            _MATS[k] = x @ x.t() / x.shape[1] + 1e-3 * torch.eye(n, device=dev)
        out.append(_MATS[k])
    return out


def solve_ms(sizes, dev, reps):
    mats = mats_for(sizes, dev)
    eigen.symeig_many(mats)                 # plans, graphs
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        eigen.symeig_many(mats)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    eigen.check_solver_status()
    return min(ts)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device('cuda')
    torch.cuda.set_stream(torch.cuda.Stream())
    L = layers()
    data = []          # (sizes, ms)
    report = {}
    t0 = time.time()
    for W in (1, 2, 4, 8):
        for strat in ('measured', 'batched'):
            if W == 1 and strat == 'batched':
                continue
            locs = assign(strat, W, L)
            sets = [[] for _ in range(W)]
            nb = [0] * W
            for (a, g), r in zip(L, locs):
                sets[r] += [a, g]
                nb[r] += unit_bytes(a, g)
            times = []
            for s in sets:
                ms = solve_ms(s, dev, reps) if s else 0.0
                times.append(ms)
                if s:
                    data.append((s, ms))
            pad = W * max(nb) / float(sum(nb)) - 1.0
            model = [P.batched_cost(s) for s in sets]
            report['W%d_%s' % (W, strat)] = dict(rank_ms=times, max_ms=max(times),
                                                 model_ms=model, arena_pad=pad,
                                                 arena_mb=W * max(nb) / 2 ** 20)
            print('W=%d %-9s max %7.2f ms  ranks [%s]  model max %6.1f  arena %7.1f MB pad %5.1f%%'
                  '  (%.0f s)' % (W, strat, max(times), ' '.join('%.1f' % t for t in times),
                                  max(model), W * max(nb) / 2 ** 20, 100 * pad, time.time() - t0),
                  flush=True)
    # random subsets for the fit
    rng = random.Random(0)
    allsizes = [n for a, g in L for n in (a, g)]
    for k in range(16):
        s = rng.sample(allsizes, rng.randint(2, 40))
        data.append((s, solve_ms(s, dev, reps)))
        print('subset %2d  n_max %5d  count %3d  %.2f ms' % (k, max(s), len(s), data[-1][1]),
              flush=True)
    X = np.array([[max(s), sum(float(n) ** 3 for n in s), sum(float(n) ** 2 for n in s), len(s)]
                  for s, _ in data])
    y = np.array([ms for _, ms in data])
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    pred = X @ coef
    old = np.array([P.batched_cost(s) for s, _ in data])
    print('fit (a, b3, b2, b0) = (%.4g, %.4g, %.4g, %.4g)' % tuple(coef))
    print('fit rel err: max %.1f%%  mean %.1f%%;  current table: max %.1f%%  mean %.1f%%' % (
        100 * np.max(np.abs(pred - y) / y), 100 * np.mean(np.abs(pred - y) / y),
        100 * np.max(np.abs(old - y) / y), 100 * np.mean(np.abs(old - y) / y)))
    report['fit'] = list(map(float, coef))
    print(json.dumps(report))


if __name__ == '__main__':
    main()
