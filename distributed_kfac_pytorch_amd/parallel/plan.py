"""Static execution plan: owners, rank groups and flat communication arenas.

Built once, the first time `KFAC.step()` has factor shapes (the reference
assigns workers at the same point: kfac/preconditioner.py:499-504,616-659).
Everything the per-step collectives need is laid out here so that each
collective is ONE call on ONE contiguous buffer:

  grad arena   f32, every layer's (nG x nA) preconditioned gradient, ordered
               by the inverse group ("block") of the layer's owner, each block
               in an equal, padded slot.  In MEM_OPT / HYBRID_OPT the gradient
               distribution inside gradient group k (ranks b*gw + k, b = block)
               is ONE in-place all-gather of the slots: block b's rank
               contributes slot b.
  eigen arena  inv_dtype, the QA/QG/dGdA (or dA, dG / A_inv, G_inv) of every
               layer whose owner sits in this rank's inverse group, one equal
               padded slot per group rank (LPT balances the slots).  COMM_OPT
               / HYBRID_OPT eigendata distribution is ONE in-place all-gather
               over the inverse group (every rank's xGMI links busy at once)
               instead of one broadcast per owner or 2-3 per layer.
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
        self.eig_empty = True
        if build_eig_arena:
            self._build_eig_arena()

    # ---------------------------------------------------------------- grads
    def _build_grad_arena(self):
        nblocks = self.world // self.gw
        order = sorted(range(len(self.layers)), key=lambda i: (self.a_locs[i] // self.gw, i))
        sizes = [0] * nblocks
        for i in order:
            sizes[self.a_locs[i] // self.gw] += _numel(self.layers[i].grad_shape)
        # equal slots (64-element aligned): the distribution is one all-gather
        self.grad_slot = max(1, (max(sizes) + 63) // 64 * 64)
        self.grad_arena = torch.zeros(nblocks * self.grad_slot, dtype=torch.float32,
                                      device=self.device)
        self.grad_blocks = [[b * self.grad_slot, b * self.grad_slot] for b in range(nblocks)]
        for i in order:
            layer = self.layers[i]
            b = self.a_locs[i] // self.gw
            off = self.grad_blocks[b][1]
            n = _numel(layer.grad_shape)
            layer.pgrad_buffer = self.grad_arena[off:off + n].view(*layer.grad_shape)
            self.grad_blocks[b][1] = off + n
        self.grad_group_index = self.rank % self.gw
        self.grad_group = self.allocator.get_grad_group(self.rank)

    def grad_block_src(self, b):
        return b * self.gw + self.grad_group_index

    # ------------------------------------------------------------ eigendata
    def _build_eig_arena(self):
        self.eig_ranks = sorted(self.allocator.get_inv_ranks(self.rank))
        my_group = set(self.eig_ranks)
        per_owner = {}
        for i, layer in enumerate(self.layers):
            for key, shape, factor in _eig_items(layer, self.use_eigen, self.prediv):
                owner = self.a_locs[i] if factor == 'A' else self.g_locs[i]
                if owner in my_group:
                    per_owner.setdefault(owner, []).append((layer, key, shape))
        sizes = [sum(_numel(s) for _, _, s in per_owner.get(o, [])) for o in self.eig_ranks]
        # one equal, 64-element aligned slot per group rank (group-rank order =
        # sorted global ranks): the distribution is one in-place all-gather
        self.eig_slot = max(1, (max(sizes) + 63) // 64 * 64)
        # a group that owns no factor (more groups than layers) has nothing to
        # distribute: broadcast_eigendata issues no collective for it
        self.eig_empty = max(sizes) == 0
        self.eig_arena = torch.zeros(len(self.eig_ranks) * self.eig_slot, dtype=self.inv_dtype,
                                     device=self.device)
        for gi, owner in enumerate(self.eig_ranks):
            off = start = gi * self.eig_slot
            self.eig_regions[owner] = (start, start)
            for layer, key, shape in per_owner.get(owner, []):
                n = _numel(shape)
                view = self.eig_arena[off:off + n].view(*shape)
                old = layer.state.get(key)
                if old is not None and old.shape == view.shape:
                    view.copy_(old)
                layer.state[key] = view
                off += n
            self.eig_regions[owner] = (start, off)

    def eig_slot_of(self, rank):
        """(start, end) of `rank`'s slot in the eigen arena."""
        gi = self.eig_ranks.index(rank)
        return gi * self.eig_slot, (gi + 1) * self.eig_slot

    def grad_slot_of(self, block):
        return block * self.grad_slot, (block + 1) * self.grad_slot

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
