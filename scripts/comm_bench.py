"""Collective micro-benchmark (reference: tests/communication.py + launch_communication.sh).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        scripts/comm_bench.py [--sizes-mb 1 4 16 64 256] [--iters 20]

1. The reference's sweep: grouped all-reduce SUM of a 100x100 fp32 tensor for
   every group size that divides the world (groups of consecutive ranks).
2. Raw bandwidth: all-reduce and per-root broadcast for message sizes 1-256 MB
   on RCCL over xGMI (bus bandwidth = 2 (W-1)/W * bytes / time for the ring).
3. The collectives the library itself issues, on ITS communicator
   (comm.backend: the dedicated K-FAC process group):
   * `allgather_into_tensor` -- the eigendata / gradient broadcasts
     (parallel/collectives.py broadcast_eigendata / broadcast_gradients) --
     for total arena sizes 4-256 MB;
   * the factor all-reduce (parallel/collectives.FactorAllreduce) on the
     ResNet-50 factor set (108 triu-packed fp32 factors, ~300 MB), swept over
     bucket_cap_mb 4..256: pack + bucketed async all-reduce + join + unpack,
     i.e. what KFAC(bucket_cap_mb=...) pays per factor step.
Timing: wall clock around `iters` back-to-back calls after a warm-up (device
synchronised), max over ranks; rank 0 prints one JSON line per measurement.
`--skip-raw` runs only section 3.
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
    ap.add_argument('--buckets-mb', nargs='+', type=float, default=[4, 8, 16, 32, 64, 128, 256])
    ap.add_argument('--skip-raw', action='store_true')
    args = ap.parse_args()
    device = launch.init_distributed()
    if not dist.is_initialized():
        print('run under torch.distributed.run with WORLD_SIZE > 1', file=sys.stderr)
        return
    world, rank = dist.get_world_size(), dist.get_rank()

    def out(rec):
        if rank == 0:
            print(json.dumps(rec), flush=True)

    if not args.skip_raw:
        raw_sweeps(args, device, world, rank, out)
    library_sweeps(args, device, world, rank, out)
    dist.barrier()
    dist.destroy_process_group()


def raw_sweeps(args, device, world, rank, out):
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


def resnet50_factor_sizes():
    from distributed_kfac_pytorch_amd.models import resnet
    out = []
    for mod in resnet.resnet50().modules():
        if isinstance(mod, torch.nn.Conv2d):
            out.append((mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1] +
                        (mod.bias is not None), mod.out_channels))
        elif isinstance(mod, torch.nn.Linear):
            out.append((mod.in_features + 1, mod.out_features))
    return out


class _FakeLayer(object):
    def __init__(self, na, ng, device):
        self.state = {'A': torch.eye(na, device=device), 'G': torch.eye(ng, device=device)}


def library_sweeps(args, device, world, rank, out):
    from distributed_kfac_pytorch_amd import comm
    from distributed_kfac_pytorch_amd.parallel import collectives
    comm.init_comm_backend()
    be = comm.backend
    out({'bench': 'kfac_communicator', 'world': be.size(), 'built_by': list(comm.build_log)})
    # 3a. all_gather_into_tensor on the K-FAC communicator (one slot per rank)
    for mb in args.sizes_mb:
        per = max(1, int(mb * 2 ** 20 / 4) // world)
        arena = torch.ones(per * world, device=device)
        mine = arena[rank * per:(rank + 1) * per]
        t = timed(lambda: be.sync(be.allgather_into(arena, mine)), args.iters, device)
        nbytes = per * world * 4
        out({'bench': 'kfac_allgather_into', 'mb': nbytes / 2 ** 20, 'ms': t * 1e3,
             'busbw_GBps': (world - 1) / world * nbytes / t / 1e9})
    # 3b. factor all-reduce of the ResNet-50 factor set per bucket size
    layers = [_FakeLayer(a, g, device) for a, g in resnet50_factor_sizes()]
    for cap in args.buckets_mb:
        fa = collectives.FactorAllreduce(layers, bucket_cap_mb=cap)
        t = timed(fa, max(3, args.iters // 4), device)
        nbytes = sum(a.numel() * a.element_size() for a in fa.arenas.values())
        out({'bench': 'kfac_factor_allreduce', 'model': 'resnet50', 'bucket_cap_mb': cap,
             'buckets': len(fa.buckets), 'mb': nbytes / 2 ** 20, 'ms': t * 1e3,
             'busbw_GBps': 2 * (world - 1) / world * nbytes / t / 1e9})


if __name__ == '__main__':
    main()
