"""Probe: run the fused reduction on a CPU-generated (reproducible) factor
and dump d, e to gpurun_out/ for a host-side LAPACK dsytrd comparison.
argv: n"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import eigen, _lib  # noqa: E402


def cpu_factor(n, seed=5):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, n // 4, generator=g, dtype=torch.float64)
    X *= torch.exp(torch.randn(n, 1, generator=g, dtype=torch.float64))
    A = X @ X.t() / X.shape[1] + 0.3 * torch.eye(n, dtype=torch.float64)
    return A.float()


def main():
    n = int(sys.argv[1])
    A32 = cpu_factor(n)
    dev = torch.device('cuda')
    L = _lib.lib()
    B = eigen._tri_buffers(dev, n, 1, slot=9)
    B['A'][0, :n, :n].copy_(A32.to(dev))
    rr = (_lib.ReduceRecord * 1)()
    r = rr[0]
    r.A, r.lda, r.d = B['A'][0].data_ptr(), B['lda'], B['d'][0].data_ptr()
    r.e, r.tau = B['e'][0].data_ptr(), B['tau'][0].data_ptr()
    r.ws, r.n = B['rws'].data_ptr(), n
    _lib.check(L.kfac_reduce_batched(rr, 1, 0, _lib.stream()), 'reduce')
    torch.cuda.synchronize()
    os.makedirs('gpurun_out/r3', exist_ok=True)
    np.save('gpurun_out/r3/dump_d_%d.npy' % n, B['d'][0].cpu().numpy())
    np.save('gpurun_out/r3/dump_e_%d.npy' % n, B['e'][0].cpu().numpy())
    print('dumped', n)


if __name__ == '__main__':
    main()
