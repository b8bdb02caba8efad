"""Gradient all-reduce overlapped with backward, hipGraph-compatible.

DDP overlaps its bucketed all-reduce with backward through autograd hooks,
which a captured forward/backward graph never runs.  Here the backward is cut
in two at an activation boundary instead (`model.forward_bottom` /
`forward_top`, e.g. ResNet's layer2 / layer3 seam):

  segment 0  forward of both halves with the boundary activation detached,
             loss.backward() through the TOP half only: the top half's
             parameter gradients (~90% of ResNet-50's bytes) are complete
  comm 0     the top half's all-reduce is ISSUED (async, RCCL's stream)
  segment 1  backward of the bottom half from the boundary gradient -- runs
             on the compute stream WHILE the top all-reduce moves over xGMI
  comm 1     the bottom half's all-reduce; both joined

Each segment is a separate graph of graphs.GraphedTrainStep (a list of
forward_backward / communicate callables); collectives are never captured.
The split changes no arithmetic: the gradients equal a single backward's.
Reference counterpart: DDP's overlapped reducer in the examples
(examples/torch_imagenet_resnet.py:151-152).
"""
import torch

from .grad_sync import GradientAllreduce

__all__ = ['SplitBackward']


class SplitBackward(object):
    """forward_backward / communicate segment lists for GraphedTrainStep.

    model: has forward_bottom, forward_top and split_parameters().
    loss_fn(out) -> scalar loss; `inputs` is a callable returning the (static)
    input tensor; autocast: dtype or None.
    """

    def __init__(self, model, loss_fn, inputs, autocast=None, group=None, weights=None,
                 broadcast_from=0):
        self.model = model
        self.loss_fn = loss_fn
        self.inputs = inputs
        self.autocast = autocast
        bottom, top = model.split_parameters()
        # bf16-stored weights (ops/mixed.BF16Weights): each segment widens its
        # bf16 weight gradients into the fp32 masters, and the masters' .grad
        # are what the arenas all-reduce (fp32, as with autocast)
        self.w_top = weights.subset(top) if weights is not None else None
        self.w_bottom = weights.subset(bottom) if weights is not None else None
        if weights is not None:
            top = [weights.master_of(p) for p in top]
            bottom = [weights.master_of(p) for p in bottom]
        # top first: rank 0's parameters / buffers are broadcast once
        self.sync_top = GradientAllreduce(model, group=group, params=top,
                                          broadcast_from=broadcast_from)
        self.sync_bottom = GradientAllreduce(model, group=group, params=bottom,
                                             broadcast_from=None)
        self._mid = None
        self._mid_in = None
        self._handles = []

    def zero_grad(self):
        self.sync_top.zero_grad()
        self.sync_bottom.zero_grad()
        for w in (self.w_top, self.w_bottom):
            if w is not None:
                w.zero_model_grads()

    def segment_top(self):
        self.zero_grad()
        x = self.inputs()
        dev = x.device.type
        with torch.autocast(device_type=dev, dtype=self.autocast or torch.float32,
                            enabled=self.autocast is not None):
            mid = self.model.forward_bottom(x)
            mid_in = mid.detach().requires_grad_(True)
            loss = self.loss_fn(self.model.forward_top(mid_in))
        loss.backward()
        if self.w_top is not None:
            self.w_top.grads_to_master()
        self._mid, self._mid_in = mid, mid_in
        return loss

    def segment_bottom(self):
        self._mid.backward(self._mid_in.grad)
        if self.w_bottom is not None:
            self.w_bottom.grads_to_master()
        return None

    def comm_top(self):
        self._handles = self.sync_top.start()

    def comm_bottom(self):
        handles = self.sync_bottom.start()
        self.sync_top.finish(self._handles)
        self.sync_bottom.finish(handles)
        self._handles = []

    @property
    def segments(self):
        return [self.segment_top, self.segment_bottom]

    @property
    def communicate(self):
        return [self.comm_top, self.comm_bottom]
