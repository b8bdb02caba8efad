"""Probe: grouped factor SYRK + EMA time on ResNet-50 (B=32) vs the row-split size."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import resnet
from distributed_kfac_pytorch_amd.ops import factors

dev = torch.device('cuda:0')
torch.manual_seed(0)
m = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=10 ** 6)
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
with torch.autocast('cuda', dtype=torch.bfloat16):
    loss = F.cross_entropy(m(x), y)
loss.backward()
items, refs = [], []
for layer in pre.layers:
    for which in ('A', 'G'):
        job = layer.take_factor_job(which)
        if job is not None:
            items.append((layer.state[which], job[0], job[1]))
flops = 0.0
for _, srcs, _ in items:
    for s in srcs:
        n = s.ncols
        flops += s.rows[0] * n * (n + 1)   # upper triangle, 2 flops per MAC
print('factors: %d, SYRK %.1f GFLOP (upper triangle)' % (len(items), flops / 1e9))
outs = factors.update_factors_grouped(items, 0.95)
items = [(o, s, d) for o, (_, s, d) in zip(outs, items)]

def timeit(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n

for split in [int(v) for v in os.environ.get('PROBE_SPLITS', '512,1024,2048,4096,8192').split(',')]:
    factors.SPLIT_ROWS = split
    t = timeit(lambda: factors.update_factors_grouped(items, 0.95))
    print('SPLIT_ROWS %5d (wide tiles from n >= %d): %.3f ms per factor step (%.0f TFLOP/s)' % (
        split, factors.WIDE_MIN, t, flops / t / 1e9), flush=True)
