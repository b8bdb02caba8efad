"""Debug: eigendecompose the real ResNet-50 K-FAC factors with rocSOLVER syevd and
with the hand-written tridiagonal path; report any non-finite / mismatching class."""
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.getcwd())
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
m = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=1000, lr=0.01)
opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
for _ in range(int(os.environ.get('STEPS', '12'))):
    m.zero_grad()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x), y)
    loss.backward()
    pre.step()
    opt.step()
torch.cuda.synchronize()
mats, names = [], []
for i, l in enumerate(pre.layers):
    for w in ('A', 'G'):
        t = l.state[w].float().contiguous()
        if t.shape[0] >= 2048:
            mats.append(t)
            names.append('%d%s n=%d' % (i, w, t.shape[0]))
print('factors', len(mats), 'finite', all(bool(torch.isfinite(t).all()) for t in mats))
eigen.LARGE_PATH = 'syevd'
ref = eigen.symeig_many(mats, clip=0.0)
eigen.LARGE_PATH = 'tridiag'
got = eigen.symeig_many(mats, clip=0.0)
torch.cuda.synchronize()
got2 = eigen.symeig_many(mats, clip=0.0)   # graph replay
torch.cuda.synchronize()
for nm, (Q1, d1), (Q2, d2) in zip(names, got, got2):
    if not (torch.isfinite(Q2).all() and torch.equal(d1, d2)):
        print('REPLAY MISMATCH', nm, bool(torch.isfinite(Q2).all()), (d1 - d2).abs().max().item())
for nm, A, (Qr, dr), (Qg, dg) in zip(names, mats, ref, got):
    fin = bool(torch.isfinite(Qg).all()) and bool(torch.isfinite(dg).all())
    A64 = A.double()
    res = ((A64 @ Qg.double() - Qg.double() * dg.double()).norm() / A64.norm()).item() if fin else float('nan')
    print(nm, 'finite', fin, 'dmax %.3e' % dr.max().item(), 'ddiff %.2e' % (dg - dr).abs().max().item(), 'resid %.1e' % res,
          'A diag min %.2e max %.2e' % (A.diagonal().min().item(), A.diagonal().max().item()), flush=True)
