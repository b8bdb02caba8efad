"""Train / test loops for the CNN examples (reference: examples/cnn_utils/engine.py:1-125).

Per loader batch: `batches_per_allreduce` micro-batches, all but the last
under `model.no_sync()` (DDP), optional mixed precision (bf16 autocast on the
GPU; fp16 + GradScaler when `--fp16`), then `preconditioner.step()` between
the gradient all-reduce and `optimizer.step()`.  Metrics stay on the device
(examples/utils.Metric) and are reduced once per epoch.

`--graphs 1` (GraphedTrainer): the MI355X fast path of bench.py in the
examples -- each batch is copied into static input buffers and the step
replays as hipGraphs (graphs.GraphedTrainStep: forward, backward, K-FAC
factor SYRKs in the captured hooks, the fused preconditioning chain, SGD);
at world size > 1 the gradient all-reduce is one flat-arena RCCL call between
the forward/backward graph and the update graph (parallel/grad_sync.py), the
K-FAC factor all-reduce is issued eagerly and joined at the next factor step.
A batch of another shape (the last, ragged one) runs the same step eagerly.
The fast path covers the reference's other two training modes too
(examples/cnn_utils/engine.py:33-82 of the reference):
  * `--batches-per-allreduce k`: the k micro-batches' forward/backward passes
    are captured in the ONE forward/backward graph (gradients accumulate; the
    graphed loop has no DDP, so the single all-reduce after it is the
    reference's no_sync behaviour);
  * `--fp16`: the loss is scaled by the GradScaler's device scale inside the
    graph, and the update is unscale -> K-FAC -> SGD step -> scale update with
    every overflow decision on the device (distributed_kfac_pytorch_amd/amp.py
    CapturableGradScaler: op for op GradScaler + SGD, a skipped step selected
    away with torch.where).
"""
import contextlib
import time

import torch

from examples.utils import Metric, accuracy

__all__ = ['train', 'test', 'GraphedTrainer']

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def _autocast(args):
    if not args.cuda:
        return contextlib.nullcontext()
    if getattr(args, 'fp16', False):
        return torch.autocast('cuda', dtype=torch.float16)
    if getattr(args, 'bf16', True):
        return torch.autocast('cuda', dtype=torch.bfloat16)
    return contextlib.nullcontext()


class GraphedTrainer(object):
    """One training step over static input buffers, replayed as hipGraphs."""

    def __init__(self, model, optimizer, preconditioner, loss_func, args, grad_sync=None):
        from distributed_kfac_pytorch_amd import graphs
        self.model, self.optimizer, self.pre = model, optimizer, preconditioner
        self.loss_func, self.args, self.grad_sync = loss_func, args, grad_sync
        self.micro = max(1, int(getattr(args, 'batches_per_allreduce', 1)))
        self.scaler = getattr(args, 'grad_scaler', None)
        if self.scaler is not None and not hasattr(self.scaler, 'step_graphable'):
            raise TypeError('the graphed loop needs amp.CapturableGradScaler')
        self.x = self.y = None
        if grad_sync is not None:
            # (a phased update would run optimizer.step() without the scaler:
            # with fp16 a kind whose update communicates runs it eagerly)
            self.step = graphs.GraphedTrainStep(None, preconditioner, [optimizer],
                                                enabled=args.cuda,
                                                forward_backward=self._forward_backward,
                                                communicate=grad_sync, update=self._update,
                                                phased_update=self.scaler is None)
        else:
            # forward_backward / update too: inverse steps replay a forward/
            # backward graph with the factors in its hooks (bench.py's one-GPU path)
            self.step = graphs.GraphedTrainStep(self._train_step, preconditioner, [optimizer],
                                                enabled=args.cuda,
                                                forward_backward=self._forward_backward,
                                                update=self._update)

    def _forward_backward(self, ragged=False):
        if self.grad_sync is not None:
            self.grad_sync.zero_grad()
        else:
            self.optimizer.zero_grad(set_to_none=False)
        k = self.micro
        mb = self.x.shape[0] // k
        if ragged:
            # a batch that does not split into k equal micro-batches (eager):
            # micro-batches of args.batch_size and a shorter last one, like the
            # reference's data[i:i + batch_size] loop (examples/cnn_utils/engine.py:33-48)
            mb = int(getattr(self.args, 'batch_size', 0)) or -(-self.x.shape[0] // k)
            k = -(-self.x.shape[0] // mb)
        losses, outs = [], []
        # factors in the captured hooks (multi-rank): all but the last
        # micro-batch only save hook data, so the factors come from the last
        # micro-batch with one EMA update, as in the eager loop and the
        # reference (KFAC.defer_hook_factors)
        defer = self.pre is not None and getattr(self.pre, 'compute_factor_in_hook', False)
        for i in range(k):
            xb, yb = (self.x, self.y) if k == 1 else \
                (self.x[i * mb:(i + 1) * mb], self.y[i * mb:(i + 1) * mb])
            ctx = self.pre.defer_hook_factors() if (defer and i < k - 1) else \
                contextlib.nullcontext()
            with ctx:
                with _autocast(self.args):
                    out = self.model(xb)
                    loss = self.loss_func(out, yb) / k
                if self.scaler is not None:
                    self.scaler.scale(loss).backward()
                else:
                    loss.backward()
            losses.append(loss.detach())
            outs.append(out.detach())
        if k == 1:
            return losses[0], outs[0]
        return torch.stack(losses).sum(), torch.cat(outs)

    def _update(self):
        sc = self.scaler
        if sc is not None:
            sc.unscale_graphable(self.optimizer)
        if self.pre is not None:
            self.pre.step()
        if sc is not None:
            sc.step_graphable(self.optimizer)
            sc.update_graphable()
        else:
            self.optimizer.step()

    def _train_step(self):
        res = self._forward_backward()
        self._update()
        return res

    def _eager(self, data, target):
        x, y = self.x, self.y
        self.x, self.y = data, target
        try:
            loss, out = self._forward_backward(ragged=data.shape[0] % self.micro != 0)
            if self.grad_sync is not None:
                self.grad_sync()
            self._update()
        finally:
            self.x, self.y = x, y
        return loss, out

    def sync_buffers(self):
        """Rank 0's BatchNorm running statistics to every rank before an
        evaluation: what the reference's DDP(broadcast_buffers=True) leaves
        on every rank at eval time (the graphed loop has no DDP wrapper)."""
        import torch.distributed as dist
        if self.grad_sync is None or not dist.is_initialized():
            return
        for b in self.model.buffers():
            if b.is_floating_point() or b.dtype in (torch.int64, torch.int32):
                dist.broadcast(b.data, src=0)

    def __call__(self, data, target):
        if data.shape[0] % self.micro:
            return self._eager(data, target)       # ragged batch: no equal micro-batches
        if self.x is None:
            self.x, self.y = data.clone(), target.clone()
        elif data.shape != self.x.shape or data.stride() != self.x.stride() or \
                target.shape != self.y.shape:
            return self._eager(data, target)
        else:
            self.x.copy_(data)
            self.y.copy_(target)
        return self.step()


def train(epoch, model, optimizer, preconditioner, loss_func, train_sampler, train_loader, args,
          log_writer=None, trainer=None):
    model.train()
    train_sampler.set_epoch(epoch)
    train_loss, train_acc = Metric('train_loss'), Metric('train_accuracy')
    scaler = getattr(args, 'grad_scaler', None)
    bar = None
    if tqdm is not None and getattr(args, 'verbose', False):
        bar = tqdm(total=len(train_loader), desc='Epoch {:3d}/{:3d}'.format(epoch, args.epochs),
                   bar_format='{l_bar}{bar:10}{r_bar}')
    t0 = time.time()
    for data, target in train_loader:
        if args.cuda:
            data, target = data.cuda(non_blocking=True), target.cuda(non_blocking=True)
            if getattr(args, 'channels_last', False):
                data = data.contiguous(memory_format=torch.channels_last)
        if trainer is not None:
            loss, out = trainer(data, target)
            train_loss.update(loss)
            train_acc.update(accuracy(out, target))
            if bar is not None:
                bar.update(1)
            continue
        optimizer.zero_grad(set_to_none=False)
        starts = list(range(0, len(data), args.batch_size))
        for i in starts:
            xb, yb = data[i:i + args.batch_size], target[i:i + args.batch_size]
            sync = i == starts[-1] or not hasattr(model, 'no_sync')
            ctx = contextlib.nullcontext() if sync else model.no_sync()
            with ctx:
                with _autocast(args):
                    out = model(xb)
                    loss = loss_func(out, yb) / len(starts)
                with torch.no_grad():
                    train_loss.update(loss * len(starts))
                    train_acc.update(accuracy(out, yb))
                if scaler is not None:
                    scaler.scale(loss).backward()
                else:
                    loss.backward()
        if preconditioner is not None:
            if scaler is not None:
                scaler.unscale_(optimizer)
            preconditioner.step()
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        if bar is not None:
            bar.update(1)
    if bar is not None:
        bar.close()
    loss_avg, acc_avg = train_loss.avg, train_acc.avg
    if log_writer is not None:
        log_writer.add_scalar('train/loss', loss_avg, epoch)
        log_writer.add_scalar('train/accuracy', acc_avg, epoch)
        log_writer.add_scalar('train/lr', optimizer.param_groups[0]['lr'], epoch)
    return {'loss': float(loss_avg), 'accuracy': float(acc_avg), 'time': time.time() - t0}


def test(epoch, model, loss_func, val_loader, args, log_writer=None):
    model.eval()
    val_loss, val_acc = Metric('val_loss'), Metric('val_accuracy')
    with torch.no_grad():
        for data, target in val_loader:
            if args.cuda:
                data, target = data.cuda(non_blocking=True), target.cuda(non_blocking=True)
                if getattr(args, 'channels_last', False):
                    data = data.contiguous(memory_format=torch.channels_last)
            with _autocast(args):
                out = model(data)
            val_loss.update(loss_func(out.float(), target))
            val_acc.update(accuracy(out, target))
    loss_avg, acc_avg = val_loss.avg, val_acc.avg
    if log_writer is not None:
        log_writer.add_scalar('val/loss', loss_avg, epoch)
        log_writer.add_scalar('val/accuracy', acc_avg, epoch)
    return {'loss': float(loss_avg), 'accuracy': float(acc_avg)}
