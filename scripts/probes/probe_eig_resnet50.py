"""Probe: wall time of one full ResNet-50 inverse update (symeig_many over every
A and G factor size of the 54 K-FAC layers, random SPD matrices) under eigensolver
scheduling variants: size-class batching vs concurrent single-matrix jobs for
the big classes (SPLIT_N), worker streams, tridiag threshold."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402


def sizes():
    m = resnet.resnet50()
    out = []
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            out += [mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1] +
                    (mod.bias is not None), mod.out_channels]
        elif isinstance(mod, torch.nn.Linear):
            out += [mod.in_features + 1, mod.out_features]
    return out


def main():
    dev = torch.device('cuda')
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    ns = sizes()
    g = torch.Generator(device=dev).manual_seed(0)
    mats = []
    for n in ns:
        x = torch.randn(n, max(64, n // 2), device=dev, generator=g)
        mats.append(x @ x.t() / x.shape[1] + 1e-3 * torch.eye(n, device=dev))
    print('factors', len(ns), 'sum n^3 %.3g' % sum(float(n) ** 3 for n in ns), flush=True)
    variants = [('default', {}), ('fs1', {'FS': 1}), ('fs3', {'FS': 3}),
                ('only_big', {'SEL': 'big'}), ('only_rest', {'SEL': 'rest'}),
                ('only_big_fs1', {'SEL': 'big', 'FS': 1}), ('only_rest_fs1', {'SEL': 'rest', 'FS': 1})]
    if len(sys.argv) > 1:
        variants = [v for v in variants if v[0] in sys.argv[1:]]
    res = {}
    base = dict(FS=eigen.FUSED_STREAMS)
    for name, cfg in variants:
        eigen.FUSED_STREAMS = cfg.get('FS', base['FS'])
        nmax = max(A.shape[0] for A in mats)
        sel = cfg.get('SEL')
        run_mats = mats if sel is None else [A for A in mats if (2 * A.shape[0] > nmax) == (sel == 'big')]
        eigen.symeig_many(run_mats)       # warm: buffers, graphs
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            outs = eigen.symeig_many(run_mats)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        eigen.check_solver_status()
        err = 0.0
        orth = 0.0
        for A, (Q, d) in zip(run_mats, outs):
            err = max(err, float((A @ Q - Q * d).norm() / A.norm()))
            orth = max(orth, float((Q.t() @ Q - torch.eye(Q.shape[0], device=Q.device)).abs().max()))
        res[name] = {'ms': min(ts), 'all_ms': ts, 'resid': err, 'orth': orth}
        print('%-14s %8.2f ms  (runs %s)  resid %.1e  orth %.1e' % (name, min(ts),
              ' '.join('%.1f' % t for t in ts), err, orth), flush=True)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
