"""Probe: per-stage time / TFLOPs of the fused preconditioning chain on ResNet-50 shapes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import resnet
from distributed_kfac_pytorch_amd.ops import _lib

dev = torch.device('cuda:0')
prec = sys.argv[1] if len(sys.argv) > 1 else 'bf16x3'
torch.manual_seed(0)
m = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=1000, lr=0.01, precond_precision=prec,
                use_hip_graphs=False)
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
with torch.autocast('cuda', dtype=torch.bfloat16):
    loss = F.cross_entropy(m(x), y)
loss.backward()
pre.step()
torch.cuda.synchronize()
fz = pre.fused
L = _lib.lib()
stream = _lib.stream(dev)

def timeit(fn, n=50):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n

flops = [0.0] * 4
for b in fz.bufs:
    nG, nA = b.nG, b.nA
    flops[0] += 2.0 * nG * nA * nG
    flops[1] += 2.0 * nA * nG * nA
    flops[2] += 2.0 * nG * nA * nG
    flops[3] += 2.0 * nG * nA * nA
from distributed_kfac_pytorch_amd.ops import precond_fused as pf


def outputs():
    fz.run(damping=0.001)
    torch.cuda.synchronize()
    return [b.layer._pgrad_matrix().clone() for b in fz.bufs]


pf.TILE_CFG = None
fz._build_stage_tables()
ref = outputs()
for cfg in [int(c) for c in os.environ.get('PGEMM_CFGS', '0,3,5,6,7').split(',') if c]:
    pf.TILE_CFG = cfg
    fz._build_stage_tables()
    t = timeit(lambda: fz.run(damping=0.001))
    err = max(((o - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
              for o, r in zip(outputs(), ref))
    print('tile cfg %d %s: chain %.3f ms  max rel diff vs default %.2e' % (
        cfg, pf.TILE_SHAPES[cfg], t, err), flush=True)
pf.TILE_CFG = int(os.environ['TILE_CFG']) if 'TILE_CFG' in os.environ else None
fz._build_stage_tables()
tot = timeit(lambda: fz.run(damping=0.001))
print('%s (operands %s): full chain %.3f ms  (%.1f GFLOP real, %.1f TFLOP/s)' % (prec, pf.X6_MODE, tot, sum(flops) / 1e9, sum(flops) / tot / 1e9))
for i, launches in enumerate(fz._stage_tables):
    def stage(i=i, launches=launches):
        slot = 1
        for tile, table, count, tiles in launches:
            kl = _lib.c_vp(fz.kl_buf.data_ptr() + 8 * slot) if i == 3 else None
            prec_i = fz.prec if fz.stage_prec is None else fz.stage_prec[i]
            L.kfac_pgemm(prec_i, tile, _lib.ptr(table), count, tiles, kl, stream)
            slot += tiles
    t = timeit(stage)
    desc = ' '.join('%s:%d' % ('big' if tl else 'small', n) for tl, _, _, n in launches)
    print('  stage %d: %.3f ms  %6.1f GFLOP  %6.1f TFLOP/s  tiles %s' % (i + 1, t, flops[i] / 1e9, flops[i] / t / 1e9, desc))
recs = fz._gather_table()
t = timeit(lambda: L.kfac_gather_grad(fz.store_prec, recs, len(recs), stream))
print('  gather: %.3f ms' % t)
