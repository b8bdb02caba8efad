"""Probe: per-tick phase times of one stage-2 (band -> tridiagonal) workgroup
(csrc/eig_sb2st.hip debug stamps) on a random n = 4608 band, plus the
kernel's wall time; and stage-1 / Q2 wall times of the same matrix."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import _lib, eig2s  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4608
    wg = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    L = _lib.lib()
    g = torch.Generator(device='cuda').manual_seed(0)
    A = torch.randn(n, n, device='cuda', generator=g)
    A = A + A.t()
    band0 = eig2s.pack_band(A)
    buf = torch.zeros(512 * 8, dtype=torch.int64, device='cuda')
    for rep in range(3):
        band = band0.clone()
        if rep == 2:
            _lib.check(L.kfac_sb2st_stamps(buf.data_ptr(), wg), 'stamps')
        torch.cuda.synchronize()
        t = time.perf_counter()
        eig2s.sb2st([band])
        torch.cuda.synchronize()
        print('sb2st n=%d  %.2f ms' % (n, (time.perf_counter() - t) * 1e3), flush=True)
    _lib.check(L.kfac_sb2st_stamps(None, 0), 'stamps off')
    st = buf.view(512, 8).cpu().numpy().astype(np.float64)
    ok = st[:, 0] > 0
    st = st[ok]
    d = np.diff(st[:, :5], axis=1) * 10.0      # 100 MHz -> ns
    tick = np.diff(st[:, 0]) * 10.0
    print('workgroup %d: %d ticks stamped' % (wg, len(st)))
    print('mean ns: issue %.0f  tasks+bar %.0f  commit+bar %.0f  retire %.0f  | tick %.0f (median %.0f)' % (
        d[:, 0].mean(), d[:, 1].mean(), d[:, 2].mean(), d[:, 3].mean(), tick.mean(), np.median(tick)))
    print('first ticks (ns):', ' '.join('%.0f' % x for x in tick[:20]))


if __name__ == '__main__':
    main()
