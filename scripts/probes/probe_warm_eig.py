"""Probe: how far do ResNet-50 K-FAC factors move between two inverse updates?

Trains the bench model (ResNet-50, batch 32, bf16 autocast, K-FAC COMM_OPT,
factors every 10 steps, eigendecompositions every 100) eagerly for 201 steps.
The eigendata of step 100 and the factors of step 200 (10 EMA updates later)
are kept; for every factor it reports, in fp64:

  * the production solver's accuracy at step 200 (off-diagonal of Q^T A Q),
  * the mixing band of the old eigenbasis: U = Q100^T Q_ref(200); for each
    eigenvector above the noise floor, how far (in sorted index) its weight
    spreads (|U_ij| > 1e-2 / 1e-4),
  * iterations of the warm-started refinement (scripts/probes/eig_warm.refine_reference)
    to reach the tolerance, per window size.

    python scripts/probes/probe_warm_eig.py [--fixed] [--steps 201] [--min-n 256]
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
import eig_warm  # noqa: E402  (scripts/probes/eig_warm.py)


def train(args, dev):
    torch.manual_seed(0)
    model = resnet.get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5)
    pre = kfac.KFAC(model, damping=1e-3, factor_decay=0.95, factor_update_freq=10,
                    inv_update_freq=100, kl_clip=1e-3, lr=0.0125,
                    comm_method=kfac.CommMethod.COMM_OPT, distribute_layer_factors=False,
                    precond_precision='bf16x6')
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(32, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device=dev, generator=g)
    snaps = {}
    t0 = time.time()
    for step in range(args.steps):
        if not args.fixed:
            x.normal_(generator=g)
            y.random_(0, 1000, generator=g)
        opt.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
        loss.backward()
        pre.step()
        opt.step()
        if step in (args.steps - 101, args.steps - 1):
            s = {}
            for i, layer in enumerate(pre.layers):
                st = layer.state
                s[i] = {k: st[k].detach().float().clone() for k in ('A', 'G', 'QA', 'QG', 'dA', 'dG')
                        if st.get(k) is not None}
            snaps[step] = s
        if step % 50 == 0:
            print('step', step, 'loss %.4f' % float(loss), '%.1fs' % (time.time() - t0), flush=True)
    return snaps


def band(U, keep, thr):
    """For each kept column j of U: max |i - j| over rows with |U_ij| > thr."""
    n = U.shape[0]
    idx = torch.arange(n, device=U.device)
    big = U.abs() > thr
    dist = (idx[:, None] - idx[None, :]).abs()
    b = torch.where(big, dist, torch.zeros_like(dist)).max(dim=0).values
    b = b[keep]
    if b.numel() == 0:
        return (0, 0, 0)
    q = torch.quantile(b.double(), torch.tensor([0.5, 0.9], dtype=torch.float64, device=U.device))
    return int(q[0]), int(q[1]), int(b.max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fixed', action='store_true', help='one fixed batch (the bench) instead of '
                    'a fresh random batch per step')
    ap.add_argument('--steps', type=int, default=201)
    ap.add_argument('--min-n', type=int, default=256)
    ap.add_argument('--windows', default='64,128,256')
    ap.add_argument('--max-iter', type=int, default=8)
    ap.add_argument('--tol', type=float, default=1e-7)
    args = ap.parse_args()
    dev = torch.device('cuda')
    snaps = train(args, dev)
    s0, s1 = snaps[args.steps - 101], snaps[args.steps - 1]
    windows = [int(w) for w in args.windows.split(',')]
    print('mode', 'fixed batch' if args.fixed else 'fresh batches', flush=True)
    print('factor n | solver off | band p50/p90/max @1e-2 | band @1e-4 | iters per window ' +
          ' '.join(str(w) for w in windows) + ' | off per iteration (best window)', flush=True)
    seen = 0
    for i in sorted(s1, key=lambda i: -s1[i]['A'].shape[0]):
        for kind in ('A', 'G'):
            F1 = s1[i][kind].double()
            n = F1.shape[0]
            if n < args.min_n:
                continue
            Q0 = s0[i]['Q' + kind].double()
            Qs = s1[i]['Q' + kind].double()
            d_ref, Q_ref = torch.linalg.eigh(F1)
            scale = float(d_ref.abs().max())
            Ss = Qs.t() @ F1 @ Qs
            solver_off = float((Ss - torch.diag(Ss.diagonal())).abs().max()) / scale
            U = Q0.t() @ Q_ref
            keep = d_ref > args.tol * scale
            b2 = band(U, keep, 1e-2)
            b4 = band(U, keep, 1e-4)
            its, best = [], None
            for w in windows:
                X, d, hist = eig_warm.refine_reference(F1, Q0, window=w, max_iter=args.max_iter,
                                                       tol=args.tol)
                its.append(len(hist) - 1 if hist[-1] <= args.tol else -1)
                if best is None or (its[-1] >= 0 and (best[0] < 0 or its[-1] < best[0])):
                    best = (its[-1], hist)
            print('L%02d %s %5d | %.1e | %d/%d/%d | %d/%d/%d | %s | %s' % (
                i, kind, n, solver_off, b2[0], b2[1], b2[2], b4[0], b4[1], b4[2],
                ' '.join(str(t) for t in its), ' '.join('%.0e' % h for h in best[1])), flush=True)
            seen += 1
    print('factors', seen)


if __name__ == '__main__':
    main()
