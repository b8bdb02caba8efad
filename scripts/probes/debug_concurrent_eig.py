"""Debug: concurrent size classes mixing the hand-written path and rocSOLVER syevd."""
import os
import sys
import torch
sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402

mode = sys.argv[1]
dev = torch.device('cuda')


def spd(n, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn(n, 50, device=dev, generator=g)
    return X @ X.t() / 50 + 1e-3 * torch.eye(n, device=dev)


mats = [spd(n, n) for n in (300, 2048, 300, 2100)]
if mode == 'serial':
    outs = eigen.symeig_many(mats, clip=0.0, solver='serial')
elif mode == 'tri_only':
    outs = eigen.symeig_many([mats[1], mats[3]], clip=0.0)
elif mode == 'syevd_only':
    eigen.LARGE_PATH = 'syevd'
    outs = eigen.symeig_many(mats, clip=0.0)
else:
    outs = eigen.symeig_many(mats, clip=0.0)
torch.cuda.synchronize()
print(mode, 'ok', [float(d.max()) for _, d in outs], flush=True)
