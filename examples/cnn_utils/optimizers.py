"""SGD + K-FAC + schedulers from the example CLI (reference: examples/cnn_utils/optimizers.py:1-74).

The preconditioner is built with the framework's MI355X options
(`--precond-precision`, hipGraph tail) and the same KFACParamScheduler /
LambdaLR wiring as the reference: one LambdaLR for the optimizer, one for the
K-FAC `lr` that feeds the KL clip, and the K-FAC damping/frequency scheduler.
"""
import torch.optim as optim

import distributed_kfac_pytorch_amd as kfac

from examples.utils import create_lr_schedule

__all__ = ['get_optimizer']

COMM = {'comm-opt': kfac.CommMethod.COMM_OPT, 'mem-opt': kfac.CommMethod.MEM_OPT,
        'hybrid-opt': kfac.CommMethod.HYBRID_OPT}


def get_optimizer(model, args, batch_first=True):
    use_kfac = args.kfac_update_freq > 0
    # (not the fused SGD with fp16: on this ROCm build its GradScaler inf skip
    # let non-finite updates through -- scripts/probes/probe_fp16_example.py;
    # the graphed loop skips overflowed steps itself, engine.GraphedTrainer)
    optimizer = optim.SGD(model.parameters(), lr=args.base_lr, momentum=args.momentum,
                          weight_decay=args.weight_decay)
    preconditioner = None
    if use_kfac:
        if args.kfac_comm_method not in COMM:
            raise ValueError('Unknown KFAC Comm Method: {}'.format(args.kfac_comm_method))
        preconditioner = kfac.KFAC(
            model,
            damping=args.damping,
            factor_decay=args.stat_decay,
            factor_update_freq=args.kfac_cov_update_freq,
            inv_update_freq=args.kfac_update_freq,
            kl_clip=args.kl_clip,
            lr=args.base_lr,
            batch_first=batch_first,
            comm_method=COMM[args.kfac_comm_method],
            distribute_layer_factors=not args.coallocate_layer_factors,
            grad_scaler=getattr(args, 'grad_scaler', None),
            grad_worker_fraction=args.kfac_grad_worker_fraction,
            skip_layers=args.skip_layers,
            use_eigen_decomp=not args.use_inv_kfac,
            precond_precision=getattr(args, 'precond_precision', 'fp32'),
            # graphed multi-rank loop: a replayed forward/backward runs no Python
            # hooks, so the factors are computed inside the captured hooks
            compute_factor_in_hook=bool(getattr(args, 'graphed', False)) and
            getattr(args, 'world_size', 1) > 1,
            verbose=getattr(args, 'verbose', False))
        kfac_scheduler = kfac.KFACParamScheduler(
            preconditioner,
            damping_alpha=args.damping_alpha,
            damping_schedule=args.damping_decay,
            update_freq_alpha=args.kfac_update_freq_alpha,
            update_freq_schedule=args.kfac_update_freq_decay)
    lrs = create_lr_schedule(args.world_size, args.warmup_epochs, args.lr_decay)
    lr_scheduler = [optim.lr_scheduler.LambdaLR(optimizer, lrs)]
    if use_kfac:
        lr_scheduler.append(optim.lr_scheduler.LambdaLR(preconditioner, lrs))
        lr_scheduler.append(kfac_scheduler)
    return optimizer, preconditioner, lr_scheduler
