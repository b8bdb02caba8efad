"""When each eigensolver stream finishes its share of a ResNet-50 inverse
update (symeig_many over the 108 factor sizes): device events recorded on the
caller's stream and on every side stream right after the call is enqueued,
timed from an event before it.  Shows which group is the critical path and how
long the back-transformations / copies after each reduction take.

    python scripts/probes/probe_eig_stream_ends.py
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402
from probe_eig_resnet50 import sizes  # noqa: E402


def main():
    dev = torch.device('cuda', torch.cuda.current_device())
    torch.cuda.set_stream(torch.cuda.Stream())
    ns = sizes()
    # KFAC_PROBE_MIN_N: drop the factors below this size (what they cost the rest)
    ns = [n for n in ns if n >= int(os.environ.get('KFAC_PROBE_MIN_N', '0'))]
    g = torch.Generator(device=dev).manual_seed(0)
    mats = []
    for n in ns:
        x = torch.randn(n, max(64, n // 2), device=dev, generator=g)
        mats.append(x @ x.t() / x.shape[1] + 1e-3 * torch.eye(n, device=dev))
    groups = eigen._fused_groups(mats)
    for gi, grp in enumerate(groups):
        sz = sorted({mats[i].shape[0] for i in grp}, reverse=True)
        print('group %d: %d factors, sizes %s' % (gi, len(grp), sz))
    for rep in range(4):
        cur = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        eigen.STAGE_EVENTS = []
        eigen.symeig_many(mats)
        stages, eigen.STAGE_EVENTS = eigen.STAGE_EVENTS, None
        ends = []
        for s in [cur] + eigen.side_streams(dev):
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ends.append(e)
        torch.cuda.synchronize()
        eigen.check_solver_status()
        print('run %d: stream ends (ms) %s' % (rep, ' '.join('%.2f' % e0.elapsed_time(e)
                                                            for e in ends)), flush=True)
        if rep == 3:
            for slot, stage, e in stages:
                print('  group %d %-8s done at %8.2f ms' % (slot, stage, e0.elapsed_time(e)))


if __name__ == '__main__':
    main()
