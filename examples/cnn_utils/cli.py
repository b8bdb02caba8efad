"""Shared CLI of the CNN examples (reference flags: SURVEY.md Appendix B)."""
import argparse

__all__ = ['base_parser', 'finalize']


def base_parser(desc, d):
    """d: per-example defaults (batch_size, epochs, base_lr, lr_decay, ...)."""
    p = argparse.ArgumentParser(description=desc,
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--data-dir', default=None, help='dataset root (synthetic data if absent)')
    p.add_argument('--log-dir', default='./logs')
    p.add_argument('--checkpoint-format', default='checkpoint_{epoch}.pth.tar')
    p.add_argument('--no-cuda', action='store_true')
    p.add_argument('--seed', type=int, default=42)
    p.add_argument('--fp16', action='store_true', help='fp16 autocast + GradScaler')
    p.add_argument('--no-bf16', action='store_true', help='disable bf16 autocast on the GPU')
    p.add_argument('--channels-last', type=int, default=1)
    p.add_argument('--model', default=d['model'])
    p.add_argument('--batch-size', type=int, default=d['batch_size'])
    p.add_argument('--val-batch-size', type=int, default=d['batch_size'])
    p.add_argument('--batches-per-allreduce', type=int, default=1)
    p.add_argument('--epochs', type=int, default=d['epochs'])
    p.add_argument('--base-lr', type=float, default=d['base_lr'])
    p.add_argument('--lr-decay', nargs='+', type=int, default=d['lr_decay'])
    p.add_argument('--warmup-epochs', type=float, default=5)
    p.add_argument('--momentum', type=float, default=0.9)
    p.add_argument('--weight-decay', type=float, default=d['weight_decay'])
    p.add_argument('--label-smoothing', type=float, default=d.get('label_smoothing', 0.0))
    p.add_argument('--checkpoint-freq', type=int, default=d['checkpoint_freq'])
    p.add_argument('--synthetic-size', type=int, default=d['synthetic_size'],
                   help='samples per epoch of the synthetic dataset')
    p.add_argument('--image-size', type=int, default=d.get('image_size', 32))
    p.add_argument('--workers', type=int, default=0)
    p.add_argument('--verbose', action='store_true')
    # K-FAC
    p.add_argument('--kfac-update-freq', type=int, default=d['kfac_update_freq'],
                   help='iterations between inverse updates (0 disables K-FAC)')
    p.add_argument('--kfac-cov-update-freq', type=int, default=d['kfac_cov_update_freq'])
    p.add_argument('--kfac-update-freq-alpha', type=float, default=10)
    p.add_argument('--kfac-update-freq-decay', nargs='+', type=int, default=None)
    p.add_argument('--use-inv-kfac', action='store_true', help='inverse instead of eigen path')
    p.add_argument('--stat-decay', type=float, default=0.95)
    p.add_argument('--damping', type=float, default=d['damping'])
    p.add_argument('--damping-alpha', type=float, default=0.5)
    p.add_argument('--damping-decay', nargs='+', type=int, default=None)
    p.add_argument('--kl-clip', type=float, default=0.001)
    p.add_argument('--skip-layers', nargs='+', type=str, default=[])
    p.add_argument('--coallocate-layer-factors', type=int, default=1,
                   help='A and G of a layer on one rank (the reference flag could not be '
                        'turned off: it was store_true with default True)')
    p.add_argument('--kfac-comm-method', default='comm-opt',
                   choices=['comm-opt', 'mem-opt', 'hybrid-opt'])
    p.add_argument('--kfac-grad-worker-fraction', type=float, default=0.25)
    p.add_argument('--precond-precision', default='bf16x6', choices=['fp32', 'bf16x3', 'bf16x6'],
                   help='fused preconditioning GEMMs: fp32 (exact-f32 MFMA), bf16x6 (three bf16 '
                        'planes, fp32-level error at the bf16 MFMA rate; the bench default) or '
                        'bf16x3 (~1e-5 relative error)')
    p.add_argument('--graphs', type=int, default=0,
                   help='MI355X fast path (1): the whole training step replayed as hipGraphs '
                        '(graphs.GraphedTrainStep), the data-parallel gradient all-reduce as one '
                        'flat-arena RCCL call between graph replays (parallel/grad_sync.py) '
                        'instead of eager DDP, K-FAC factors computed inside the captured hooks; '
                        'micro-batches (--batches-per-allreduce) are captured in the one '
                        'forward/backward graph, --fp16 uses amp.CapturableGradScaler '
                        '(overflow skip on the device)')
    p.add_argument('--deterministic', action='store_true',
                   help='deterministic MIOpen algorithms (cudnn.deterministic, no autotuning)')
    p.add_argument('--backend', default=None, help='torch.distributed backend (nccl = RCCL)')
    p.add_argument('--local_rank', '--local-rank', type=int, default=None)
    return p


def finalize(args):
    import torch
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    args.bf16 = not args.no_bf16
    args.channels_last = bool(args.channels_last) and args.cuda
    args.coallocate_layer_factors = bool(args.coallocate_layer_factors)
    return args
