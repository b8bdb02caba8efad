"""Shared driver of the CIFAR-10 and ImageNet examples (one process per GPU).

Launch: `python -m torch.distributed.run --nproc-per-node 8 --master-addr
127.0.0.1 examples/torch_imagenet_resnet.py ...` (or a single process).
Flow per the reference (examples/torch_cifar10_resnet.py:110-194,
examples/torch_imagenet_resnet.py:117-210): init RCCL process group ->
model -> DDP -> SGD + K-FAC + schedulers -> resume from the newest checkpoint
(rank 0 decides, broadcast) -> train/test per epoch -> checkpoint every
`--checkpoint-freq` epochs on rank 0.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from distributed_kfac_pytorch_amd import models  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import launch  # noqa: E402
from examples.cnn_utils import datasets, engine, optimizers  # noqa: E402
from examples.utils import (LabelSmoothLoss, latest_checkpoint_epoch, load_checkpoint,  # noqa: E402
                            save_checkpoint)


def run(args, dataset):
    device = launch.init_distributed(backend=args.backend, no_cuda=args.no_cuda)
    import torch.distributed as dist
    args.world_size = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    args.verbose = args.verbose and rank == 0
    torch.manual_seed(args.seed)
    if args.cuda:
        torch.backends.cudnn.benchmark = not getattr(args, 'deterministic', False)
        torch.backends.cudnn.deterministic = bool(getattr(args, 'deterministic', False))

    if dataset == 'cifar':
        (train_sampler, train_loader), (_, val_loader) = datasets.get_cifar(args)
    else:
        (train_sampler, train_loader), (_, val_loader) = datasets.get_imagenet(args)

    if dataset == 'cifar' and args.model.lower() not in models.resnet_cifar._MODELS:
        model = models.get_model(args.model, num_classes=10)   # an ImageNet-style net on CIFAR
    else:
        model = models.get_model(args.model)
    model = model.to(device)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    if args.verbose:
        print(model)
    # --graphs: the bench's fast path (no eager DDP: a flat-arena all-reduce
    # between graph replays), micro-batching and fp16 + GradScaler included
    # (amp.CapturableGradScaler: the overflow skip stays on the device);
    # otherwise the reference's eager DDP loop
    args.graphed = bool(getattr(args, 'graphs', 0))
    grad_sync = None
    if args.graphed and args.world_size > 1:
        from distributed_kfac_pytorch_amd.parallel import grad_sync as grad_sync_mod
        grad_sync = grad_sync_mod.GradientAllreduce(model)
    elif not args.graphed:
        model = launch.wrap_ddp(model, device)

    # LR scales with the number of workers and micro-batches (reference)
    args.base_lr = args.base_lr * args.world_size * args.batches_per_allreduce
    if args.fp16 and args.cuda:
        # a GradScaler (the eager loop uses its standard API) whose unscale /
        # step / update the graphed loop can capture
        from distributed_kfac_pytorch_amd.amp import CapturableGradScaler
        args.grad_scaler = CapturableGradScaler('cuda')
    optimizer, preconditioner, lr_schedules = optimizers.get_optimizer(model, args)
    loss_func = LabelSmoothLoss(args.label_smoothing) if args.label_smoothing > 0 \
        else torch.nn.CrossEntropyLoss()

    os.makedirs(args.log_dir, exist_ok=True)
    fmt = os.path.join(args.log_dir, args.checkpoint_format)
    resume = latest_checkpoint_epoch(fmt, args.epochs)
    if resume > 0:
        load_checkpoint(fmt.format(epoch=resume), model, optimizer, preconditioner,
                        lr_schedules, device)
        if args.verbose:
            print('resumed from epoch', resume)

    trainer = engine.GraphedTrainer(model, optimizer, preconditioner, loss_func, args,
                                    grad_sync) if args.graphed else None
    history = []
    start = time.time()
    for epoch in range(resume, args.epochs):
        tr = engine.train(epoch, model, optimizer, preconditioner, loss_func, train_sampler,
                          train_loader, args, trainer=trainer)
        if trainer is not None:
            trainer.sync_buffers()
        va = engine.test(epoch, model, loss_func, val_loader, args)
        for s in lr_schedules:
            s.step()
        history.append({'epoch': epoch + 1, 'train': tr, 'val': va})
        if rank == 0:
            print(json.dumps(history[-1]), flush=True)
        if args.checkpoint_freq > 0 and (epoch + 1) % args.checkpoint_freq == 0 and rank == 0:
            save_checkpoint(model, optimizer, preconditioner, lr_schedules,
                            fmt.format(epoch=epoch + 1))
    if rank == 0 and args.verbose:
        print('Training time: {:.1f} s'.format(time.time() - start))
    return history
