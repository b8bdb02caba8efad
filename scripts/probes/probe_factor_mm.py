"""Factor products as library GEMMs: ResNet-50 (batch 32, 224^2) A/G factor
shapes as explicit bf16 [rows][cols] matrices, X^T X with fp32 output through
torch.mm(out_dtype=float32) (hipBLASLt), plus the explicit im2col (unfold) of
the k>1 convolutions, against the grouped implicit-im2col SYRK's measured
3.3 ms per factor update.

    python scripts/probes/probe_factor_mm.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from distributed_kfac_pytorch_amd.models.resnet import resnet50  # noqa: E402


def shapes():
    m = resnet50().cuda().to(memory_format=torch.channels_last)
    out = []

    def hook(mod, inp, outp):
        x = inp[0]
        if isinstance(mod, nn.Conv2d):
            rows = outp.shape[0] * outp.shape[2] * outp.shape[3]
            k = mod.kernel_size[0] * mod.kernel_size[1]
            out.append((rows, mod.in_channels * k + (mod.bias is not None), mod.out_channels,
                        k, tuple(x.shape), mod))
        elif isinstance(mod, nn.Linear):
            out.append((x.shape[0], mod.in_features + 1, mod.out_features, 1, tuple(x.shape), mod))
    for mod in m.modules():
        if isinstance(mod, (nn.Conv2d, nn.Linear)):
            mod.register_forward_hook(hook)
    with torch.no_grad():
        m(torch.randn(32, 3, 224, 224, device='cuda').contiguous(memory_format=torch.channels_last))
    return out


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    sh = shapes()
    mats = []
    for rows, na, ng, k, xs, mod in sh:
        mats.append(torch.randn(rows, na, device='cuda').to(torch.bfloat16))
        mats.append(torch.randn(rows, ng, device='cuda').to(torch.bfloat16))

    def mm_only():
        for x in mats:
            torch.mm(x.t(), x, out_dtype=torch.float32)
    flops = sum(2.0 * x.shape[0] * x.shape[1] ** 2 for x in mats)
    t = timeit(mm_only)
    print('library GEMM X^T X over %d factors: %.3f ms (%.1f TFLOP/s full-square, %.1f GFLOP)' % (
        len(mats), t, flops / t / 1e9, flops / 1e9))
    # per-factor breakdown of the 12 most expensive
    per = []
    for x in mats:
        per.append((timeit(lambda: torch.mm(x.t(), x, out_dtype=torch.float32), 10), tuple(x.shape)))
    per.sort(reverse=True)
    for t1, s in per[:12]:
        print('  %8.3f ms  %s  %.0f TFLOP/s' % (t1, s, 2.0 * s[0] * s[1] ** 2 / t1 / 1e9))
    # explicit im2col of the k>1 convolutions (bf16 NHWC input)
    ins = []
    for rows, na, ng, k, xs, mod in sh:
        if isinstance(mod, nn.Conv2d) and k > 1:
            ins.append((torch.randn(*xs, device='cuda').to(torch.bfloat16)
                        .contiguous(memory_format=torch.channels_last), mod))

    def unfold_all():
        for x, mod in ins:
            torch.nn.functional.unfold(x, mod.kernel_size, padding=mod.padding,
                                       stride=mod.stride).transpose(1, 2).contiguous()
    print('explicit im2col (unfold + transpose) of %d convolutions: %.3f ms' % (
        len(ins), timeit(unfold_all)))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mm_only()
    print('library GEMMs graphed: %.3f ms' % timeit(g.replay))


if __name__ == '__main__':
    main()
