"""Example utilities: metrics, checkpoints, label smoothing, LR schedule.

Reference behaviour: examples/utils.py:1-61.  MI355X-specific change: the
`Metric` accumulates on the device and reduces across ranks only when the
average is read (the reference did a blocking all-reduce + .cpu() on every
update, twice per iteration: SURVEY.md X9).
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

__all__ = ['accuracy', 'save_checkpoint', 'load_checkpoint', 'LabelSmoothLoss', 'Metric',
           'create_lr_schedule', 'latest_checkpoint_epoch']


def accuracy(output, target):
    pred = output.argmax(1)
    return (pred == target).float().mean()


def save_checkpoint(model, optimizer, preconditioner, schedulers, filepath):
    """{'model','optimizer','preconditioner','schedulers'} (reference layout)."""
    m = model.module if hasattr(model, 'module') else model
    state = {
        'model': m.state_dict(),
        'optimizer': optimizer.state_dict(),
        'preconditioner': preconditioner.state_dict() if preconditioner is not None else None,
        'schedulers': [s.state_dict() for s in schedulers] if isinstance(schedulers, list)
        else None,
    }
    tmp = filepath + '.tmp'
    torch.save(state, tmp)
    os.replace(tmp, filepath)


def load_checkpoint(filepath, model, optimizer, preconditioner, schedulers, device):
    """Counterpart of save_checkpoint; loads tensors only (weights_only)."""
    state = torch.load(filepath, map_location=device, weights_only=True)
    m = model.module if hasattr(model, 'module') else model
    m.load_state_dict(state['model'])
    optimizer.load_state_dict(state['optimizer'])
    if preconditioner is not None and state.get('preconditioner') is not None:
        preconditioner.load_state_dict(state['preconditioner'])
    if state.get('schedulers') is not None and isinstance(schedulers, list):
        for s, sd in zip(schedulers, state['schedulers']):
            s.load_state_dict(sd)


def latest_checkpoint_epoch(fmt, max_epochs):
    """Newest epoch with a checkpoint file, decided on rank 0 and broadcast so
    every rank resumes from the same epoch (the reference let each rank scan
    the filesystem on its own: SURVEY.md section 5.3)."""
    epoch = 0
    if not dist.is_initialized() or dist.get_rank() == 0:
        for e in range(max_epochs, 0, -1):
            if os.path.exists(fmt.format(epoch=e)):
                epoch = e
                break
    if dist.is_initialized():
        t = torch.tensor([epoch])
        if dist.get_backend() == 'nccl':
            t = t.cuda()
        dist.broadcast(t, 0)
        epoch = int(t.item())
    return epoch


class LabelSmoothLoss(torch.nn.Module):
    def __init__(self, smoothing=0.0):
        super().__init__()
        self.smoothing = smoothing

    def forward(self, input, target):
        log_prob = F.log_softmax(input, dim=-1)
        weight = input.new_full(input.size(), self.smoothing / (input.size(-1) - 1.0))
        weight.scatter_(-1, target.unsqueeze(-1), 1.0 - self.smoothing)
        return (-weight * log_prob).sum(dim=-1).mean()


class Metric(object):
    """Running mean kept on the device; cross-rank average on read."""

    def __init__(self, name):
        self.name = name
        self.total = None
        self.n = 0

    def update(self, val, n=1):
        val = val.detach().float()
        self.total = val * n if self.total is None else self.total + val * n
        self.n += n

    @property
    def avg(self):
        if self.total is None:
            return torch.tensor(0.0)
        t = torch.stack([self.total.reshape(()), self.total.new_tensor(float(self.n))])
        if dist.is_initialized():
            dist.all_reduce(t)
        return (t[0] / t[1]).cpu()


def create_lr_schedule(workers, warmup_epochs, decay_schedule, alpha=0.1):
    """Linear warm-up from 1/workers to 1 over warmup_epochs, then x alpha at
    every epoch in decay_schedule (reference examples/utils.py:50-61)."""
    decay = sorted(decay_schedule, reverse=True)

    def lr_schedule(epoch):
        if epoch < warmup_epochs:
            return 1.0 / workers * (epoch * (workers - 1) / warmup_epochs + 1)
        adj = 1.0
        for e in decay:
            if epoch >= e:
                adj *= alpha
        return adj
    return lr_schedule
