"""Collective micro-benchmark (reference: tests/communication.py + launch_communication.sh).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        scripts/comm_bench.py [--sizes-mb 1 4 16 64 256] [--iters 20]

1. The reference's sweep: grouped all-reduce SUM of a 100x100 fp32 tensor for
   every group size that divides the world (groups of consecutive ranks).
2. The MI355X sweep that chooses K-FAC's factor bucket size: all-reduce and
   per-root broadcast bandwidth for message sizes 1-256 MB on RCCL over xGMI
   (bus bandwidth = 2 (W-1)/W * bytes / time for the all-reduce ring).
Timing uses device events around `iters` back-to-back calls after a warm-up,
max over ranks; rank 0 prints one JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_kfac_pytorch_amd.parallel import launch  # noqa: E402


def timed(fn, iters, device):
    for _ in range(3):
        fn()
    if device.type == 'cuda':
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if device.type == 'cuda':
        torch.cuda.synchronize()
    dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=device)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes-mb', nargs='+', type=float, default=[1, 4, 16, 64, 256])
    ap.add_argument('--iters', type=int, default=20)
    args = ap.parse_args()
    device = launch.init_distributed()
    if not dist.is_initialized():
        print('run under torch.distributed.run with WORLD_SIZE > 1', file=sys.stderr)
        return
    world, rank = dist.get_world_size(), dist.get_rank()

    def out(rec):
        if rank == 0:
            print(json.dumps(rec), flush=True)

    # 1. reference sweep: grouped all-reduce of 100 x 100 fp32
    x = torch.ones(100, 100, device=device)
    for gs in [g for g in range(1, world + 1) if world % g == 0]:
        groups = [dist.new_group(list(range(s, s + gs))) for s in range(0, world, gs)]
        mine = groups[rank // gs]
        t = timed(lambda: dist.all_reduce(x, group=mine), args.iters, device)
        out({'bench': 'grouped_allreduce_100x100', 'group_size': gs, 'ms': t * 1e3})

    # 2. bucket sweep
    for mb in args.sizes_mb:
        n = int(mb * 2 ** 20 / 4)
        buf = torch.ones(n, device=device)
        t = timed(lambda: dist.all_reduce(buf), args.iters, device)
        busbw = 2 * (world - 1) / world * n * 4 / t / 1e9
        out({'bench': 'allreduce', 'mb': mb, 'ms': t * 1e3, 'busbw_GBps': busbw})
        t = timed(lambda: dist.broadcast(buf, src=0), args.iters, device)
        out({'bench': 'broadcast', 'mb': mb, 'ms': t * 1e3, 'algbw_GBps': n * 4 / t / 1e9})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
