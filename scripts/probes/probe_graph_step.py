"""Probe: is the B=32 ResNet-50 step CPU-launch bound? eager vs whole-step hipGraph."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import resnet

dev = torch.device('cuda:0')
torch.backends.cudnn.benchmark = True
B = int(os.environ.get('B', 32))

def build(use_kfac):
    torch.manual_seed(0)
    m = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-5)
    pre = kfac.KFAC(m, factor_update_freq=10**9, inv_update_freq=10**9, lr=0.01) if use_kfac else None
    return m, opt, pre

x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (B,), device=dev)

def make_step(m, opt, pre):
    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y, label_smoothing=0.1)
        loss.backward()
        if pre is not None:
            pre.step()
        opt.step()
        return loss
    return step

def bench(fn, n=50):
    for _ in range(5): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n * 1e3

for use_kfac in (False, True):
    m, opt, pre = build(use_kfac)
    step = make_step(m, opt, pre)
    if pre is not None:
        step()  # step 0 = factor + inverse step (eager); later steps are plain
        pre.use_hip_graphs = True
    e = bench(step)
    # whole-step capture
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3): step()
    torch.cuda.current_stream().wait_stream(s)
    if pre is not None:
        pre.use_hip_graphs = False   # the outer graph already covers the tail
    g = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=False)
    with torch.cuda.graph(g):
        step()
    gt = bench(g.replay)
    print('kfac' if use_kfac else 'sgd ', 'B=%d eager %.2f ms  graphed %.2f ms' % (B, e, gt), flush=True)
