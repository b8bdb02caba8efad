"""Chain A (4000 dependent one-workgroup launches, one hipGraph) beside
  (1) nothing, (2) an identical chain B on another stream, (3) ONE persistent
  kernel on another stream that runs the same number of phases separated by
  grid barriers (256 / 64 workgroups).
Per-launch time of A in each case, and the persistent kernel's time per
barrier.  Build first (in-tree, on the CPU):

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/probes/persistent_vs_chain.so \\
        scripts/probes/persistent_vs_chain.hip
    python scripts/probes/probe_persistent_vs_chain.py [N]
"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    torch.cuda.init()
    lib = ctypes.CDLL(os.path.join(HERE, 'persistent_vs_chain.so'))
    vp = ctypes.c_void_p
    lib.pvc_chain.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    lib.pvc_persistent.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    assert lib.pvc_init() == 0
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

    def run(chain_a, chain_b, pers_grid, sleep=1):
        cur = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        ends = {}
        if chain_a:
            s1.wait_event(e0)
            assert lib.pvc_chain(vp(s1.cuda_stream), n, 0) == 0
            ends['A'] = torch.cuda.Event(enable_timing=True)
            ends['A'].record(s1)
        if chain_b:
            s2.wait_event(e0)
            assert lib.pvc_chain(vp(s2.cuda_stream), n, 1) == 0
            ends['B'] = torch.cuda.Event(enable_timing=True)
            ends['B'].record(s2)
        if pers_grid:
            s3.wait_event(e0)
            assert lib.pvc_persistent(vp(s3.cuda_stream), n, pers_grid, sleep) == 0
            ends['P'] = torch.cuda.Event(enable_timing=True)
            ends['P'].record(s3)
        torch.cuda.synchronize()
        err = lib.pvc_err() if pers_grid else 0
        return {k: e0.elapsed_time(e) for k, e in ends.items()}, err

    cases = [('A alone', (1, 0, 0, 1)), ('A + chain B', (1, 1, 0, 1))]
    for grid in (256, 64, 16):
        for sl in (1, 8, 32):
            cases += [('persistent %d sleep %d alone' % (grid, sl), (0, 0, grid, sl)),
                      ('A + persistent %d sleep %d' % (grid, sl), (1, 0, grid, sl))]
    for rep in range(3):
        for name, (a, b, p, sl) in cases:
            t, err = run(a, b, p, sl)
            if rep == 2:
                print('%-32s %s%s' % (name, '  '.join(
                    '%s %.2f ms (%.2f us/step)' % (k, v, 1e3 * v / n) for k, v in sorted(t.items())),
                    '  ERR %d' % err if err else ''), flush=True)
            if err:
                print('persistent kernel barrier timed out; stopping', flush=True)
                return


if __name__ == '__main__':
    main()
