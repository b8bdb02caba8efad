"""GPU probe: baseline costs of the pieces a K-FAC step is made of on MI355X.

Measures (1) ResNet-50 fwd+bwd+SGD at per-GPU batch 32, bf16 autocast, NCHW vs
channels_last; (2) torch.linalg.eigh (rocSOLVER) for the ResNet-50 factor sizes;
(3) fp32 GEMM rate for the preconditioning shapes. Writes gpurun_out/probe.json.
"""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.models.resnet import resnet50

out = {}
dev = torch.device('cuda:0')
print('device', torch.cuda.get_device_name(0), flush=True)

def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters

for bs in (32, 128):
    for fmt in ('nchw', 'nhwc'):
        torch.manual_seed(0)
        m = resnet50().to(dev)
        mf = torch.channels_last if fmt == 'nhwc' else torch.contiguous_format
        m = m.to(memory_format=mf)
        opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
        x = torch.randn(bs, 3, 224, 224, device=dev).to(memory_format=mf)
        y = torch.randint(0, 1000, (bs,), device=dev)
        lossf = torch.nn.CrossEntropyLoss()
        def step():
            opt.zero_grad(set_to_none=False)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = lossf(m(x), y)
            loss.backward()
            opt.step()
        t = timeit(step, iters=10, warm=5)
        out['resnet50_b%d_%s_ms' % (bs, fmt)] = t * 1e3
        print('resnet50', bs, fmt, '%.2f ms  %.0f img/s' % (t * 1e3, bs / t), flush=True)
        del m, opt, x

for n in (64, 128, 256, 512, 576, 1024, 1152, 2048, 2304, 4608):
    torch.manual_seed(0)
    a = torch.randn(n, 4 * n, device=dev)
    A = a @ a.t() / (4 * n) + 1e-3 * torch.eye(n, device=dev)
    try:
        t = timeit(lambda: torch.linalg.eigh(A), iters=3, warm=1)
    except Exception as e:
        t = float('nan'); print('eigh fail', n, e)
    out['eigh_%d_ms' % n] = t * 1e3
    t2 = timeit(lambda: torch.cholesky_inverse(torch.linalg.cholesky(A)), iters=3, warm=1)
    out['cholinv_%d_ms' % n] = t2 * 1e3
    print('eigh n=%d %.2f ms, cholinv %.2f ms' % (n, t * 1e3, t2 * 1e3), flush=True)

for (m_, k_, n_) in ((512, 4608, 4608), (2048, 2048, 2048), (4096, 4096, 4096), (256, 2304, 2304)):
    a = torch.randn(m_, k_, device=dev); b = torch.randn(k_, n_, device=dev)
    t = timeit(lambda: a @ b, iters=20, warm=3)
    out['sgemm_%dx%dx%d_tflops' % (m_, k_, n_)] = 2 * m_ * k_ * n_ / t / 1e12
    ab = a.bfloat16(); bb = b.bfloat16()
    t = timeit(lambda: ab @ bb, iters=20, warm=3)
    out['bgemm_%dx%dx%d_tflops' % (m_, k_, n_)] = 2 * m_ * k_ * n_ / t / 1e12
    print('gemm', m_, k_, n_, out['sgemm_%dx%dx%d_tflops' % (m_, k_, n_)], out['bgemm_%dx%dx%d_tflops' % (m_, k_, n_)], flush=True)

os.makedirs('gpurun_out', exist_ok=True)
json.dump(out, open('gpurun_out/probe.json', 'w'), indent=1)
print(json.dumps(out))
