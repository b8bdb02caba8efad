"""Static execution plan: owners, rank groups and flat communication arenas.

Built once, the first time `KFAC.step()` has factor shapes (the reference
assigns workers at the same point: kfac/preconditioner.py:499-504,616-659).
Everything the per-step collectives need is laid out here so that each
collective is ONE call on ONE contiguous buffer:

  grad arena   f32, every layer's (nG x nA) preconditioned gradient, ordered
               by the inverse group ("block") of the layer's owner.  In
               MEM_OPT / HYBRID_OPT the gradient broadcast of block b inside
               gradient group k is a single broadcast of a contiguous range
               from rank b*gw + k -- no packing.
  eigen arena  inv_dtype, the QA/QG/dGdA (or dA, dG / A_inv, G_inv) of every
               layer whose owner sits in this rank's inverse group, ordered
               by owner.  COMM_OPT / HYBRID_OPT eigendata distribution is one
               broadcast per owner rank (W roots drive their xGMI links
               concurrently) instead of 2-3 broadcasts per layer.
Layer tensors (`layer.pgrad_buffer`, `layer.state['QA']`, ...) become views
into these arenas.
"""
import torch

from ..utils.distribution import WorkerAllocator

__all__ = ['ExecutionPlan']


def _eig_items(layer, use_eigen, prediv):
    """[(key, shape, factor)] eigendata items of a layer; factor in {'A','G'}."""
    nA = layer.state['A'].shape[0]
    nG = layer.state['G'].shape[0]
    if not use_eigen:
        return [('A_inv', (nA, nA), 'A'), ('G_inv', (nG, nG), 'G')]
    items = [('QA', (nA, nA), 'A'), ('QG', (nG, nG), 'G')]
    if prediv:
        items.append(('dGdA', (nG, nA), 'A'))
    else:
        items += [('dA', (nA,), 'A'), ('dG', (nG,), 'G')]
    return items


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


class ExecutionPlan(object):
    def __init__(self, layers, world, rank, a_locs, g_locs, allocator, use_eigen, prediv,
                 inv_dtype, build_eig_arena, device):
        self.layers = layers
        self.world = world
        self.rank = rank
        self.a_locs = list(a_locs)
        self.g_locs = list(g_locs)
        self.allocator = allocator
        self.gw = allocator.grad_workers
        self.use_eigen = use_eigen
        self.prediv = prediv
        self.inv_dtype = inv_dtype
        self.device = device
        self._build_grad_arena()
        self.eig_arena = None
        self.eig_regions = {}
        if build_eig_arena:
            self._build_eig_arena()

    # ---------------------------------------------------------------- grads
    def _build_grad_arena(self):
        nblocks = self.world // self.gw
        order = sorted(range(len(self.layers)), key=lambda i: (self.a_locs[i] // self.gw, i))
        total = sum(_numel(self.layers[i].grad_shape) for i in order)
        self.grad_arena = torch.zeros(max(total, 1), dtype=torch.float32, device=self.device)
        self.grad_blocks = [[0, 0] for _ in range(nblocks)]
        off = 0
        cur_block = None
        for i in order:
            layer = self.layers[i]
            b = self.a_locs[i] // self.gw
            if b != cur_block:
                self.grad_blocks[b][0] = off
                cur_block = b
            n = _numel(layer.grad_shape)
            layer.pgrad_buffer = self.grad_arena[off:off + n].view(*layer.grad_shape)
            off += n
            self.grad_blocks[b][1] = off
        self.grad_group_index = self.rank % self.gw
        self.grad_group = self.allocator.get_grad_group(self.rank)

    def grad_block_src(self, b):
        return b * self.gw + self.grad_group_index

    # ------------------------------------------------------------ eigendata
    def _build_eig_arena(self):
        my_group = set(self.allocator.get_inv_ranks(self.rank))
        per_owner = {}
        for i, layer in enumerate(self.layers):
            for key, shape, factor in _eig_items(layer, self.use_eigen, self.prediv):
                owner = self.a_locs[i] if factor == 'A' else self.g_locs[i]
                if owner in my_group:
                    per_owner.setdefault(owner, []).append((layer, key, shape))
        total = sum(_numel(s) for items in per_owner.values() for _, _, s in items)
        self.eig_arena = torch.zeros(max(total, 1), dtype=self.inv_dtype, device=self.device)
        off = 0
        for owner in sorted(per_owner):
            start = off
            for layer, key, shape in per_owner[owner]:
                n = _numel(shape)
                view = self.eig_arena[off:off + n].view(*shape)
                old = layer.state.get(key)
                if old is not None and old.shape == view.shape:
                    view.copy_(old)
                layer.state[key] = view
                off += n
            self.eig_regions[owner] = (start, off)

    def eig_group(self, owner):
        return self.allocator.get_inv_group(owner)

    def describe(self):
        lines = ['ExecutionPlan(world={}, grad_workers={}, layers={})'.format(
            self.world, self.gw, len(self.layers))]
        lines.append('  grad arena: {:.1f} MB, blocks {}'.format(
            self.grad_arena.numel() * 4 / 2 ** 20, self.grad_blocks))
        if self.eig_arena is not None:
            lines.append('  eigen arena: {:.1f} MB, owners {}'.format(
                self.eig_arena.numel() * self.eig_arena.element_size() / 2 ** 20,
                sorted(self.eig_regions)))
        return '\n'.join(lines)


def make_allocator(world, fraction):
    return WorkerAllocator(world, fraction)
