"""Stage times of the one-stage eigensolver on ResNet-50's largest size class
alone (3 x 4608, or the sizes given): tridiagonal reduction, divide and
conquer, back-transformation -- device events between the stages
(eigen.STAGE_EVENTS).  Run under `rocprofv3 --kernel-trace --stats` for the
per-kernel split.

    python scripts/probes/probe_eig_stages_4608.py [n ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402


def main():
    ns = [int(a) for a in sys.argv[1:]] or [4608] * 3
    dev = torch.device('cuda', torch.cuda.current_device())
    torch.cuda.set_stream(torch.cuda.Stream())
    g = torch.Generator(device=dev).manual_seed(0)
    mats = []
    for n in ns:
        x = torch.randn(n, n // 2, device=dev, generator=g)
        mats.append(x @ x.t() / x.shape[1] + 1e-3 * torch.eye(n, device=dev))
    for rep in range(4):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        eigen.STAGE_EVENTS = []
        outs = eigen.symeig_many(mats)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        stages, eigen.STAGE_EVENTS = eigen.STAGE_EVENTS, None
        torch.cuda.synchronize()
        eigen.check_solver_status()
        prev = 0.0
        parts = []
        for slot, stage, e in stages:
            t = e0.elapsed_time(e)
            parts.append('%s %.2f' % (stage, t - prev))
            prev = t
        print('run %d: total %.2f ms | %s' % (rep, e0.elapsed_time(e1), ', '.join(parts)),
              flush=True)
    A, (Q, d) = mats[0], outs[0]
    print('resid %.2e' % float((A @ Q - Q * d).norm() / A.norm()))


if __name__ == '__main__':
    main()
