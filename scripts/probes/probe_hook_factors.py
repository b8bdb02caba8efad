"""Factor-step cost on ResNet-50 (bf16 autocast, channels_last, batch 32):
forward + backward + factor update, with the factors computed
  grouped   in KFAC.step()'s grouped launches (one rank, the bench default)
  hooks     compute_factor_in_hook=True (the multi-rank segmented-graph mode):
            grouped launches from the backward's last gradient hook
  hooks_layer  the same mode with per-layer launches inside every hook
Eager (no graphs), CUDA events around the step, median of 10."""
import os
import sys
import statistics

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402


def run(mode):
    torch.manual_seed(0)
    m = resnet.resnet50().cuda().to(memory_format=torch.channels_last)
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=10 ** 6, lr=0.1,
                    compute_factor_in_hook=mode.startswith('hooks'), use_hip_graphs=False)
    if mode == 'hooks_layer':
        pre.grouped_factors = False     # round-2 behaviour: per-layer launches in every hook
    x = torch.randn(32, 3, 224, 224, device='cuda').contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device='cuda')
    times = []
    for i in range(14):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        m.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        p = pre.param_groups[0]
        if mode == 'grouped':
            pre.compute_factors(alpha=p['factor_decay'])
        p['step'] += 1
        b.record()
        torch.cuda.synchronize()
        if i >= 4:
            times.append(a.elapsed_time(b))
    return statistics.median(times)


def run_fb():
    torch.manual_seed(0)
    m = resnet.resnet50().cuda().to(memory_format=torch.channels_last)
    x = torch.randn(32, 3, 224, 224, device='cuda').contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device='cuda')
    times = []
    for i in range(14):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        m.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        b.record()
        torch.cuda.synchronize()
        if i >= 4:
            times.append(a.elapsed_time(b))
    return statistics.median(times)


if __name__ == '__main__':
    fb = run_fb()
    print('forward+backward alone      %.3f ms' % fb, flush=True)
    for mode in ('grouped', 'hooks', 'hooks_layer'):
        t = run(mode)
        print('%-8s factor step %.3f ms  (factors %.3f ms)' % (mode, t, t - fb), flush=True)
