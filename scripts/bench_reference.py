"""Baseline: the READ-ONLY reference K-FAC (MLHPC/Distributed_KFAC_Pytorch) on MI355X.

BASELINE.md asks for the reference itself, run on PyTorch-ROCm with the one
shim it needs on torch 2.x (torch.symeig -> torch.linalg.eigh, SURVEY.md
section 0), on the headline config: ResNet-50, per-GPU batch 32, synthetic
224x224 images, COMM_OPT, factors every 10 steps, eigendecompositions every
100, damping 1e-3, kl_clip 1e-3, SGD momentum 0.9 -- timed exactly like
bench.py (W warmup steps, the K-FAC step counter reset so the K-step window
opens with an inverse step, device synchronize on both sides).

The model is this framework's ResNet-50 with stock BatchNorm modules
(KFAC_FUSED_BN=0: torchvision is not in the image; the layer inventory is
torchvision's), wrapped in torch DDP like the reference example
(examples/torch_imagenet_resnet.py:141-151), eager (the reference has no
graph capture).  The reference sources are never copied into this
repository: locally they are read from /root/reference; on the GPU box from
a tar of that tree passed with --ref-tar (git-ignored, extracted to /tmp).

    python scripts/bench_reference.py --steps 20 --warmup 5 [--autocast bf16|none]
"""
import argparse
import json
import os
import sys
import tarfile
import time

sys.dont_write_bytecode = True
os.environ.setdefault('KFAC_FUSED_BN', '0')

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _symeig(t, eigenvectors=True):
    d, Q = torch.linalg.eigh(t)
    return d, Q.contiguous()


def _cholesky(t, upper=False):
    return torch.linalg.cholesky(t, upper=upper)


def import_reference(ref_dir, ref_tar):
    if ref_tar:
        dst = '/tmp/kfac_reference_src'
        if not os.path.isdir(os.path.join(dst, 'kfac')):
            with tarfile.open(ref_tar) as tf:
                tf.extractall(dst)
        ref_dir = dst
    torch.symeig = _symeig
    torch.cholesky = _cholesky
    sys.path.insert(0, ref_dir)
    import kfac as refkfac
    assert os.path.abspath(refkfac.__file__).startswith(os.path.abspath(ref_dir)), refkfac.__file__
    return refkfac


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch-size', type=int, default=32)
    ap.add_argument('--autocast', default='bf16', choices=['bf16', 'none'])
    ap.add_argument('--no-kfac', action='store_true')
    ap.add_argument('--channels-last', type=int, default=0,
                    help='the reference reshapes activations with .view(), which needs NCHW')
    ap.add_argument('--ref-dir', default=os.environ.get('KFAC_REFERENCE', '/root/reference'))
    ap.add_argument('--ref-tar', default=None)
    args = ap.parse_args()

    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl')
    world = dist.get_world_size()
    refkfac = import_reference(args.ref_dir, args.ref_tar)
    refkfac.comm.init_comm_backend()
    from distributed_kfac_pytorch_amd.models import resnet

    torch.manual_seed(1234)
    torch.backends.cudnn.benchmark = True
    mf = torch.channels_last if args.channels_last else torch.contiguous_format
    model = resnet.resnet50().to(dev).to(memory_format=mf)
    model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    base_lr = 0.0125 * world
    opt = torch.optim.SGD(model.parameters(), lr=base_lr, momentum=0.9, weight_decay=5e-5)
    pre = None
    if not args.no_kfac:
        pre = refkfac.KFAC(model, damping=0.001, factor_decay=0.95, factor_update_freq=10,
                           inv_update_freq=100, kl_clip=0.001, lr=base_lr,
                           comm_method=refkfac.CommMethod.COMM_OPT,
                           distribute_layer_factors=False)
    B = args.batch_size
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 3, 224, 224, device=dev, generator=g).to(memory_format=mf)
    y = torch.randint(0, 1000, (B,), device=dev, generator=g)

    def step():
        opt.zero_grad(set_to_none=True)
        if args.autocast == 'bf16':
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
        else:
            loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
        loss.backward()
        if pre is not None:
            pre.step()
        opt.step()
        return loss

    for i in range(args.warmup):
        step()
        print('warmup', i, flush=True)
    if pre is not None:
        pre.param_groups[0]['step'] = 0
    kinds, evs = [], []
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        kinds.append(('inverse' if i % 100 == 0 else 'factor' if i % 10 == 0 else 'plain')
                     if pre is not None else 'plain')
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append(e)
        loss = step()
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    evs.append(e)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    per = {}
    for k, a, b in zip(kinds, evs[:-1], evs[1:]):
        per.setdefault(k, []).append(a.elapsed_time(b))
    rec = {'metric': 'images/sec (whole node) ResNet-50 K-FAC+SGD, REFERENCE implementation'
                     if pre is not None else 'images/sec ResNet-50 SGD-only, stock modules, eager',
           'value': round(B * world * args.steps / el, 2), 'unit': 'images/s', 'n_gpus': world,
           'steps': args.steps, 'warmup': args.warmup,
           'ms_per_step': round(el / args.steps * 1e3, 3),
           'autocast': args.autocast, 'channels_last': bool(args.channels_last), 'final_loss': round(float(loss.item()), 4),
           'step_ms_by_kind': {k: round(sum(v) / len(v), 3) for k, v in per.items()},
           'steps_by_kind': {k: len(v) for k, v in per.items()},
           'implementation': 'reference kfac (torch.symeig shim: linalg.eigh), torch DDP, '
                             'stock BatchNorm, eager',
           'data': 'synthetic'}
    if dist.get_rank() == 0:
        print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
