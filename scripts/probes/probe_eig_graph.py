"""Probe: hipGraph capture of rocSOLVER sytrd (the dominant part of syevd)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from distributed_kfac_pytorch_amd.ops import _lib

dev = torch.device('cuda:0')
L = _lib.lib()
for n, b in ((4608, 3), (2304, 6), (1024, 6), (512, 6)):
    torch.manual_seed(0)
    X = torch.randn(b, n, n // 2, device=dev)
    A0 = X @ X.transpose(1, 2) / (n // 2) + 1e-3 * torch.eye(n, device=dev)
    A = A0.clone()
    D = torch.empty(b, n, device=dev); E = torch.empty(b, n, device=dev)
    tau = torch.empty(b, n, device=dev)
    torch.cuda.synchronize()

    def call():
        A.copy_(A0)
        _lib.check(L.kfac_rocsolver_sytrd_batched(_lib.ptr(A), n, b, _lib.ptr(D), _lib.ptr(E), _lib.ptr(tau), 1,
                                        _lib.stream(dev)), 'sytrd')
    call(); torch.cuda.synchronize()
    t = time.perf_counter(); call(); torch.cuda.synchronize(); te = (time.perf_counter() - t) * 1e3
    D1 = D.clone()
    s = torch.cuda.Stream()
    # warm the rocblas handle + its workspace for the capture stream outside capture
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        call()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s):
            call()
    except Exception as e:
        print('n=%d x%d eager sytrd %.1f ms | capture failed: %s' % (n, b, te, str(e)[:120]), flush=True)
        break
    g.replay(); torch.cuda.synchronize()
    t = time.perf_counter(); g.replay(); torch.cuda.synchronize(); tg = (time.perf_counter() - t) * 1e3
    print('n=%d x%d eager sytrd %.1f ms | graph %.1f ms | same d: %s' % (
        n, b, te, tg, torch.allclose(D, D1)), flush=True)
