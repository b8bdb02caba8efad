"""Graphed factor-step cost on ResNet-50 (bf16 autocast, channels_last, batch 32,
one GPU): factors computed in KFAC.step() (single-segment graphs, the one-rank
bench path) vs inside the backward's captured hooks (compute_factor_in_hook,
segmented graphs: the multi-rank path).  Replays only -- no Python hooks run
in either -- so the difference is GPU time.  Median over replays of each kind.

    python scripts/probes/probe_hook_factors_graphed.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd import graphs  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402


def build(in_hook):
    torch.manual_seed(0)
    m = resnet.resnet50().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
    pre = kfac.KFAC(m, factor_update_freq=10, inv_update_freq=100, lr=0.01,
                    compute_factor_in_hook=in_hook, precond_precision='bf16x6')
    x = torch.randn(32, 3, 224, 224, device='cuda').contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device='cuda')

    def fb():
        opt.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        return loss

    def update():
        pre.step()
        opt.step()

    def whole():
        loss = fb()
        update()
        return loss

    if in_hook:
        step = graphs.GraphedTrainStep(None, pre, [opt], forward_backward=fb, update=update)
    else:
        step = graphs.GraphedTrainStep(whole, pre, [opt])
    return pre, step


def time_kind(pre, step, s, reps=10):
    p = pre.param_groups[0]
    ts = []
    for _ in range(reps):
        p['step'] = s
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        step()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    res = {}
    for name, in_hook in (('in_step', False), ('in_hook', True)):
        pre, step = build(in_hook)
        for _ in range(3):
            step()
        step.prepare()
        plain = time_kind(pre, step, 11)
        factor = time_kind(pre, step, 20)
        res[name] = (plain, factor)
        print('%-8s plain %.3f ms  factor %.3f ms  factor - plain %.3f ms  (replays %d)' % (
            name, plain, factor, factor - plain, step.replays), flush=True)
        del pre, step
        torch.cuda.empty_cache()
    d = (res['in_hook'][1] - res['in_hook'][0]) - (res['in_step'][1] - res['in_step'][0])
    print('in-hook factor overhead vs in-step: %+.3f ms' % d)


if __name__ == '__main__':
    main()
