"""One rank on RCCL (torch.distributed 'nccl' on ROCm), world size 1, run as
a child process by tests/test_gpu_rccl.py.

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one
device), so this drives the K-FAC communication layer's own calls through a
real RCCL communicator at world size 1: the bucketed factor arena
(pack_triu -> SUM all-reduce -> unpack_triu, fp32 and bf16, the X1 path of
parallel/collectives.py), the in-place all-gather of the eigendata / gradient
arenas (X3 / X5), broadcast, the dedicated K-FAC world group and a sub-group
from new_group, then a few K-FAC steps of a small CNN with the process group
up.  Prints RCCL_W1_OK and the backend counters on success.
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='env://', rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == 'nccl'
    from distributed_kfac_pytorch_amd import comm
    from distributed_kfac_pytorch_amd.ops import comm_pack
    comm.reset_comm_backend()
    b = comm.init_comm_backend()
    assert isinstance(b, comm.TorchBackend), type(b)

    g = torch.Generator(device=dev).manual_seed(0)
    # X1: triu-packed factor arena, SUM all-reduce, unpack with 1/world
    for dtype in (torch.float32, torch.bfloat16):
        n = 300
        x = torch.randn(n, n, device=dev, generator=g)
        A = (x @ x.t()).to(dtype)
        arena = torch.empty(comm_pack.triu_numel(n), device=dev, dtype=dtype)
        comm_pack.pack_triu(A, arena)
        h = b.allreduce(arena, op=comm.Ops.Sum)
        b.wait(h)
        B = torch.zeros_like(A)
        comm_pack.unpack_triu(arena, B, divisor=b.size())
        assert torch.equal(A, B), dtype
    # Average divides by the group size inside wait()
    v = torch.randn(4096, device=dev, generator=g)
    w = v.clone()
    b.sync(b.allreduce(w, op=comm.Ops.Average))
    assert torch.equal(v, w)
    # X3 / X5: in-place all-gather into the arena (this rank's slot is the arena)
    arena = torch.randn(1 << 20, device=dev, generator=g)
    ref = arena.clone()
    b.sync(b.allgather_into(arena, arena[:arena.numel()]))
    assert torch.equal(arena, ref)
    # broadcast from rank 0 over the K-FAC world / a one-rank sub-group
    t = torch.randn(1000, device=dev, generator=g)
    tr = t.clone()
    b.sync(b.broadcast(t, src=0))
    assert torch.equal(t, tr)
    grp = comm.CommGroup([0])
    assert b.allreduce(t, group=grp) is None          # one-rank group: no collective
    b.barrier()
    torch.cuda.synchronize()

    # K-FAC steps with the RCCL process group up (COMM_OPT; at world size 1
    # the plan issues no collective, the backend stays the torch one)
    import distributed_kfac_pytorch_amd as kfac
    torch.manual_seed(0)
    model = torch.nn.Sequential(
        torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.Flatten(),
        torch.nn.Linear(8 * 8 * 8, 10)).to(dev)
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2, use_hip_graphs=False)
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    for _ in range(4):
        x = torch.randn(16, 3, 8, 8, device=dev)
        y = torch.randint(0, 10, (16,), device=dev)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        opt.step()
    torch.cuda.synchronize()
    assert all(bool(torch.isfinite(p).all()) for p in model.parameters())
    print('counters', b.counters())
    print('RCCL_W1_OK', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
