"""Roofline model of ResNet-50's factor products (batch 32, 224x224): every
Conv2d / Linear A (implicit im2col P^T P) and G (g^T g) factor, as the grouped
SYRK computes them (upper 128 x 128 tiles over all rows).

Per problem (M rows, n columns, nt = ceil(n / 128) tiles per side):
  MFMA flops     = nt (nt + 1) / 2 * 2 * M * 128^2   (tiles are computed whole)
  useful flops   = M * n * (n + 1)                    (the upper triangle)
  operand bytes  = nt (nt + 1) / 2 * 2 * M * 128 * 2  (each tile streams its two
                   128-column bf16 panels over all M rows: L2 / MALL traffic)
  unique bytes   = M * n_src * 2                      (the activation / gradient
                   itself, read once: HBM)
Floors: MFMA at 2.5 PFLOP/s (dense bf16), operand traffic at an assumed
L2 + MALL rate, unique bytes at 6 TB/s.  Prints the per-problem class totals
and the sum of per-problem maxima (launch overlap ignored).

    python scripts/probes/syrk_roofline_model.py [L2_TBps]
"""
import sys

import torch

sys.path.insert(0, '.')
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402

L2 = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0   # TB/s, operand traffic
PEAK = 2.5e15
HBM = 6e12


def problems(batch=32, size=224):
    m = resnet.resnet50()
    out = []
    hooks = []

    def hook(mod, inp, outp):
        x = inp[0]
        if isinstance(mod, torch.nn.Conv2d):
            kh, kw = mod.kernel_size
            rows = outp.shape[0] * outp.shape[2] * outp.shape[3]
            out.append(('A', mod, rows, mod.in_channels * kh * kw, x.numel()))
            out.append(('G', mod, rows, mod.out_channels, outp.numel()))
        elif isinstance(mod, torch.nn.Linear):
            out.append(('A', mod, x.shape[0], mod.in_features + 1, x.numel()))
            out.append(('G', mod, x.shape[0], mod.out_features, outp.numel()))

    for mod in m.modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear)):
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(batch, 3, size, size))
    return out


def main():
    tot = dict(mfma=0.0, useful=0.0, opb=0.0, uniq=0.0, t_floor=0.0, t_mfma=0.0, t_op=0.0)
    rows = []
    for kind, mod, M, n, src in problems():
        nt = (n + 127) // 128
        tiles = nt * (nt + 1) // 2
        mf = tiles * 2.0 * M * 128 * 128
        uf = float(M) * n * (n + 1)
        opb = tiles * 2.0 * M * 128 * 2
        ub = src * 2.0
        tm, to, tu = mf / PEAK, opb / (L2 * 1e12), ub / HBM
        tot['mfma'] += mf
        tot['useful'] += uf
        tot['opb'] += opb
        tot['uniq'] += ub
        tot['t_mfma'] += tm
        tot['t_op'] += to
        tot['t_floor'] += max(tm, to, tu)
        rows.append((max(tm, to, tu), kind, M, n, tm, to, tu))
    rows.sort(reverse=True)
    print('problems %d  MFMA flops %.1f G (useful %.1f G)  operand traffic %.2f GB  unique %.1f MB'
          % (len(rows), tot['mfma'] / 1e9, tot['useful'] / 1e9, tot['opb'] / 1e9, tot['uniq'] / 1e6))
    print('floors (ms): MFMA %.3f  operand traffic at %.0f TB/s %.3f  sum of per-problem max %.3f'
          % (tot['t_mfma'] * 1e3, L2, tot['t_op'] * 1e3, tot['t_floor'] * 1e3))
    print('largest problems (ms): floor  kind  M  n  mfma  operands  unique')
    for r in rows[:12]:
        print('  %.4f  %s  %7d  %5d  %.4f  %.4f  %.4f' % (r[0] * 1e3, r[1], r[2], r[3],
                                                         r[4] * 1e3, r[5] * 1e3, r[6] * 1e3))


if __name__ == '__main__':
    main()
