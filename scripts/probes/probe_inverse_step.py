"""Probe: where the wall time of a ResNet-50 inverse-update step goes (the
bench config: batch 32, bf16 autocast, COMM_OPT, bf16x6 preconditioning,
channels_last, fused BN).  Every K-FAC sub-phase of the eager update is
wrapped with a device sync on both sides, so the numbers add up to the step
(syncs serialise what would overlap; the solver itself runs as in the bench).

    python scripts/probes/probe_inverse_step.py [reps]
"""
import collections
import functools
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402

T = collections.defaultdict(list)


def timed(name, fn):
    @functools.wraps(fn)
    def run(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn(*a, **k)
        torch.cuda.synchronize()
        T[name].append((time.perf_counter() - t) * 1e3)
        return out
    return run


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5,
                          fused=True)
    pre = kfac.KFAC(model, damping=1e-3, factor_decay=0.95, factor_update_freq=1,
                    inv_update_freq=1, kl_clip=1e-3, lr=0.0125,
                    distribute_layer_factors=False, precond_precision='bf16x6',
                    assignment_strategy='batched', use_hip_graphs=False)
    x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device=dev)
    for name in ('compute_inverses', 'broadcast_inverses', '_eigendata_updated',
                 'compute_preconditioned_gradients', 'update_gradients', 'allreduce_factors',
                 '_store_inverses', '_solve_inverses'):
        setattr(pre, name, timed(name, getattr(pre, name)))
    eigen.symeig_many = timed('symeig_many', eigen.symeig_many)
    eigen.check_solver_status = timed('check_solver_status', eigen.check_solver_status)
    fwdbwd = timed('forward_backward', lambda: (
        F.cross_entropy(model(x), y, label_smoothing=0.1)).backward())
    step = timed('kfac_step', pre.step)
    ostep = timed('opt_step', opt.step)
    for i in range(reps + 2):
        if i == 2:
            T.clear()
        opt.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            fwdbwd()
        step()
        ostep()
    torch.cuda.synchronize()
    for k, v in sorted(T.items(), key=lambda kv: -sum(kv[1])):
        print('%-34s %8.2f ms/step  (calls %d)' % (k, sum(v) / reps, len(v)))


if __name__ == '__main__':
    main()
