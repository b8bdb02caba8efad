"""Flat-arena data-parallel gradient averaging (the graph-friendly DDP replacement).

`GradientAllreduce(model)` makes every parameter's `.grad` a view into ONE
contiguous buffer per dtype (with the parameter's own strides, so
channels_last conv weights stay channels_last) and averages the whole buffer
with a single RCCL all-reduce per call -- one large message, which is what a
ring over the point-to-point xGMI links (7 x ~153 GB/s per MI355X) moves at
full per-link bandwidth, instead of DDP's ~25 MB buckets.  It has no autograd
hooks, so a forward+backward segment can be captured into a hipGraph and the
all-reduce issued between graph replays (graphs.GraphedTrainStep, segmented
mode); DDP's reducer, whose hooks run during backward, cannot.

Overlap with backward: `start()` issues the all-reduce asynchronously (RCCL's
stream, joined later by `finish()`), so with a backward split into graph
segments (parallel/overlap.py) the all-reduce of the gradients a segment
completed runs while the next segment replays -- one GradientAllreduce per
segment's parameters (`params=`).
On construction parameters and buffers are broadcast from rank 0 (what DDP
does), so ranks may initialise their models independently.

Reference counterpart: the DDP / Horovod gradient all-reduce of the examples
(examples/torch_imagenet_resnet.py:151-152).
"""
import torch
import torch.distributed as dist

__all__ = ['GradientAllreduce']


class GradientAllreduce(object):
    def __init__(self, model, group=None, broadcast_from=0, average=True, params=None):
        self.group = group
        self.average = average
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if params is None:
            params = model.parameters()
        params = [p for p in params if p.requires_grad]
        by_dtype = {}
        for p in params:
            by_dtype.setdefault(p.dtype, []).append(p)
        self.arenas = []
        self.views = []      # (param, arena view)
        for dtype, ps in by_dtype.items():
            total = sum(p.numel() for p in ps)
            arena = torch.zeros(total, dtype=dtype, device=ps[0].device)
            off = 0
            for p in ps:
                n = p.numel()
                if not _dense_strides(p):
                    raise ValueError('parameter with non-dense strides {}'.format(p.stride()))
                view = torch.as_strided(arena, p.shape, p.stride(), off)
                p.grad = view
                self.views.append((p, view))
                off += n
            self.arenas.append(arena)
        if self.world > 1 and broadcast_from is not None:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, src=broadcast_from, group=group)

    @staticmethod
    def broadcast_model(model, group=None, src=0):
        """Broadcast every parameter and buffer of `model` from rank `src`
        (what construction does with broadcast_from=src), e.g. before fp32
        masters are derived from the weights (ops/mixed.BF16Weights)."""
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, src=src, group=group)

    def zero_grad(self):
        """One fill per arena instead of one per parameter."""
        for arena in self.arenas:
            arena.zero_()

    def check_views(self):
        """True while every .grad is still the arena view it was bound to (an
        optimizer `zero_grad(set_to_none=True)` or a user assigning .grad
        breaks this: the next backward allocates gradients outside the arena,
        which an all-reduce of the arena would silently skip)."""
        for p, view in self.views:
            g = p.grad
            if g is None or g.data_ptr() != view.data_ptr() or g.stride() != view.stride():
                return False
        return True

    def rebind(self):
        """Point every .grad back at its arena view, copying a gradient that
        backward produced elsewhere into the arena (None -> zeros)."""
        with torch.no_grad():
            for p, view in self.views:
                g = p.grad
                if g is not None and g.data_ptr() == view.data_ptr() and \
                        g.stride() == view.stride():
                    continue
                if g is None:
                    view.zero_()
                else:
                    view.copy_(g)
                p.grad = view

    def start(self):
        """Issue the all-reduce of every arena asynchronously -> handles."""
        if not self.check_views():
            self.rebind()
        if self.world <= 1:
            return []
        # SUM + scale (ReduceOp.AVG needs ncclAvg support in the RCCL build)
        return [(dist.all_reduce(arena, op=dist.ReduceOp.SUM, group=self.group, async_op=True),
                 arena) for arena in self.arenas]

    def finish(self, handles):
        """Order the current stream behind the all-reduces; average."""
        for work, arena in handles:
            work.wait()
            if self.average:
                arena.mul_(1.0 / self.world)

    def __call__(self):
        self.finish(self.start())


def _dense_strides(t):
    """The strides are a permutation of a contiguous layout (no gaps/overlap)."""
    dims = sorted(((s, n) for s, n in zip(t.stride(), t.shape) if n != 1))
    expect = 1
    for s, n in dims:
        if s != expect:
            return False
        expect *= n
    return True
