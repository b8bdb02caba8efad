"""Debug: back-transformation residual per (n, batch), eager vs graph."""
import os
import sys
import torch
sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen  # noqa: E402

dev = torch.device('cuda')
side = torch.cuda.Stream()
for arg in sys.argv[1:]:
    n, b = (int(v) for v in arg.split('x'))
    g = torch.Generator(device=dev).manual_seed(n)
    X = torch.randn(b, n, n // 3 + 1, device=dev, dtype=torch.float64, generator=g)
    A64 = X @ X.transpose(1, 2) / X.shape[2] + 1e-3 * torch.eye(n, device=dev, dtype=torch.float64)
    mats = [A64[i].float() for i in range(b)]
    for ug in (False, True, True):
        side.wait_stream(torch.cuda.current_stream())
        outs = eigen._tridiag_class(mats, 0.0, side, use_graph=ug)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        res = []
        for i, (Q, d) in enumerate(outs):
            r = ((A64[i] @ Q.double() - Q.double() * d.double()).norm() / A64[i].norm()).item()
            res.append('%.1e' % r)
        print(n, b, 'graph' if ug else 'eager', res, flush=True)
