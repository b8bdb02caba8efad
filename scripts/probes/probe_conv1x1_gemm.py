"""ResNet-50's stride-1 1x1 convolutions (batch 32, bf16, channels_last):
MIOpen (F.conv2d, cudnn.benchmark) against the same layer as plain GEMMs
(forward X W^T, backward dY W and dY^T X through torch.matmul = hipBLASLt),
forward + backward (input and weight gradients) replayed from a hipGraph.

    python scripts/probes/probe_conv1x1_gemm.py
"""
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
N = 32
# (cin, cout, hw, count per ResNet-50 step)
SHAPES = [(64, 64, 56, 1), (64, 256, 56, 4), (256, 64, 56, 2), (256, 128, 56, 1),
          (128, 512, 28, 4), (512, 128, 28, 3), (512, 256, 28, 1), (256, 1024, 14, 6),
          (1024, 256, 14, 5), (1024, 512, 14, 1), (512, 2048, 7, 3), (2048, 512, 7, 2)]


def conv_miopen(x, w):
    return F.conv2d(x, w)


def conv_gemm(x, w):
    n, c, h, wd = x.shape
    xm = x.permute(0, 2, 3, 1).reshape(-1, c)          # channels_last: a view
    y = xm @ w.view(w.shape[0], c).t()
    return y.view(n, h, wd, -1).permute(0, 3, 1, 2)


def timed(fn, x, w, gy, reps=20):
    def body():
        x.grad = None
        w.grad = None
        y = fn(x, w)
        y.backward(gy)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    x.grad = None
    w.grad = None
    with torch.cuda.graph(g):
        for _ in range(reps):
            y = fn(x, w)
            gx, gw = torch.autograd.grad(y, (x, w), gy)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps), gx, gw


def main():
    tot_m = tot_g = 0.0
    print('%5s %5s %3s %3s  %9s %9s  %s' % ('cin', 'cout', 'hw', 'n', 'miopen', 'gemm', 'max rel diff'))
    for cin, cout, hw, cnt in SHAPES:
        g = torch.Generator(device='cuda').manual_seed(0)
        x = torch.randn(N, cin, hw, hw, device='cuda', generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
        w = (torch.randn(cout, cin, 1, 1, device='cuda', generator=g) / cin ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
        gy = torch.randn(N, cout, hw, hw, device='cuda', generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        tm, gxm, gwm = timed(conv_miopen, x, w, gy)
        tg, gxg, gwg = timed(conv_gemm, x, w, gy)
        d = max(((gxm.float() - gxg.float()).norm() / gxm.float().norm()).item(),
                ((gwm.float() - gwg.float()).norm() / gwm.float().norm()).item())
        tot_m += cnt * tm
        tot_g += cnt * tg
        print('%5d %5d %3d %3d  %9.4f %9.4f  %.2e' % (cin, cout, hw, cnt, tm, tg, d), flush=True)
    print('per ResNet-50 step (stride-1 1x1 convs, fwd+bwd): miopen %.3f ms, gemm %.3f ms'
          % (tot_m, tot_g))


if __name__ == '__main__':
    main()
