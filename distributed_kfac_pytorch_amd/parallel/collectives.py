"""Bucketed K-FAC collectives over RCCL (xGMI) / gloo.

FactorAllreduce   X1+X2: the upper triangles of every
                  A and G factor are packed (K12 kernel) into one flat arena
                  per dtype, all-reduced (SUM) in buckets of whole factors of
                  about `bucket_cap_mb`, and unpacked with the 1/world
                  averaging folded into the unpack kernel.  Halves the bytes
                  on the wire and turns 2 x #layers NCCL calls into a handful.
                  Split in two: `start()` packs and issues every bucket
                  asynchronously on the K-FAC communicator's stream and
                  returns; `finish()` joins (a device-side stream wait, no
                  host sync on RCCL) and unpacks.  KFAC calls finish() only
                  where the averaged factors are consumed -- the next EMA
                  update, the next inverse update, a state_dict -- so the
                  all-reduce of a factor step runs under the rest of that
                  step and the following plain steps (reference: issued and
                  waited inside step(), kfac/preconditioner.py:525-533).
broadcast_eigendata  X3/X4: ONE in-place all-gather of the plan's eigen arena
                  (equal per-owner slots) over this rank's inverse group:
                  every owner's region reaches every member in one RCCL call
                  with all ranks' xGMI links busy, instead of one broadcast
                  per owner (round 1) or per layer (reference,
                  kfac/layers/base.py:129-196).
broadcast_gradients  X5: ONE in-place all-gather of the grad arena's block
                  slots over this rank's gradient group (MEM_OPT /
                  HYBRID_OPT; reference kfac/layers/base.py:160-196).
All calls are asynchronous collectives whose completion only orders the
current HIP stream behind RCCL's stream: no host synchronisation.
"""
import torch

from .. import comm
from ..ops import comm_pack

__all__ = ['FactorAllreduce', 'broadcast_eigendata', 'broadcast_gradients']


class _Entry(object):
    __slots__ = ('layer', 'key', 'n', 'off', 'numel')

    def __init__(self, layer, key, n, off):
        self.layer, self.key, self.n, self.off = layer, key, n, off
        self.numel = comm_pack.triu_numel(n)


class FactorAllreduce(object):
    def __init__(self, layers, bucket_cap_mb=64.0, symmetric=True):
        self.layers = layers
        self.bucket_cap = int(bucket_cap_mb * 2 ** 20)
        self.symmetric = symmetric
        self._signature = None
        self.arenas = {}    # dtype -> flat tensor
        self.buckets = []   # (dtype, start, end, [entries])
        self._pending = None    # in-flight buckets: [(handle, dtype, entries)]
        self.waits = 0          # finish() calls that joined an in-flight all-reduce (tests)

    def _current_signature(self):
        sig = []
        for layer in self.layers:
            for key in ('A', 'G'):
                t = layer.state.get(key)
                sig.append(None if t is None else (tuple(t.shape), t.dtype, str(t.device)))
        return tuple(sig)

    def _build(self):
        by_dtype = {}
        device = None
        for layer in self.layers:
            for key in ('A', 'G'):
                t = layer.state.get(key)
                if t is None:
                    continue
                device = t.device
                by_dtype.setdefault(t.dtype, []).append((layer, key, t.shape[0]))
        self.arenas, self.buckets = {}, []
        for dtype, items in by_dtype.items():
            # reverse registration order: the last layers' factors are the
            # first complete in backward, so they open the first bucket
            items = list(reversed(items))
            off, entries = 0, []
            for layer, key, n in items:
                e = _Entry(layer, key, n, off)
                entries.append(e)
                off += e.numel if self.symmetric else n * n
            esize = torch.tensor([], dtype=dtype).element_size()
            self.arenas[dtype] = torch.empty(max(off, 1), dtype=dtype, device=device)
            cur, start, size = [], 0, 0
            for e in entries:
                nbytes = (e.numel if self.symmetric else e.n * e.n) * esize
                if cur and size + nbytes > self.bucket_cap:
                    self.buckets.append((dtype, start, e.off, cur))
                    cur, start, size = [], e.off, 0
                cur.append(e)
                size += nbytes
            if cur:
                self.buckets.append((dtype, start, off, cur))
        self._signature = self._current_signature()

    @property
    def pending(self):
        return self._pending is not None

    def __call__(self):
        self.start()
        self.finish()

    def start(self):
        """Pack every factor and issue the bucketed SUM all-reduce; returns
        without waiting.  A previous all-reduce still in flight is joined
        first (its arena is about to be overwritten)."""
        backend = comm.backend
        if backend.size() == 1:
            return
        self.finish()
        if self._signature != self._current_signature():
            self._build()
        for dtype, arena in self.arenas.items():
            for b_dtype, s, e, entries in self.buckets:
                if b_dtype != dtype:
                    continue
                for ent in entries:
                    self._pack(ent, arena)
        pending = []
        for dtype, s, e, entries in self.buckets:
            h = backend.allreduce(self.arenas[dtype][s:e], op=comm.Ops.Sum)
            pending.append((h, dtype, entries))
        self._pending = pending

    def finish(self):
        """Join the in-flight all-reduce and write the averaged factors back
        (1/world folded into the unpack).  No-op when nothing is in flight."""
        pending, self._pending = self._pending, None
        if pending is None:
            return
        backend = comm.backend
        world = backend.size()
        self.waits += 1
        for h, dtype, entries in pending:
            backend.wait(h)
            arena = self.arenas[dtype]
            for ent in entries:
                self._unpack(ent, arena, world)

    def _pack(self, ent, arena):
        t = ent.layer.state[ent.key]
        if self.symmetric:
            comm_pack.pack_triu(t, arena[ent.off:ent.off + ent.numel])
        else:
            arena[ent.off:ent.off + ent.n * ent.n].copy_(t.reshape(-1))

    def _unpack(self, ent, arena, world):
        t = ent.layer.state[ent.key]
        if self.symmetric:
            comm_pack.unpack_triu(arena[ent.off:ent.off + ent.numel], t, divisor=world)
        else:
            t.view(-1).copy_(arena[ent.off:ent.off + ent.n * ent.n])
            t /= world


def broadcast_eigendata(plan):
    backend = comm.backend
    if backend.size() == 1 or plan.eig_arena is None or len(plan.eig_ranks) <= 1 or \
            plan.eig_empty:
        return
    s, e = plan.eig_slot_of(plan.rank)
    backend.sync(backend.allgather_into(plan.eig_arena, plan.eig_arena[s:e],
                                        group=plan.eig_group(plan.rank)))


def broadcast_gradients(plan):
    backend = comm.backend
    if backend.size() == 1 or plan.grad_group.size <= 1:
        return
    s, e = plan.grad_slot_of(plan.rank // plan.gw)
    backend.sync(backend.allgather_into(plan.grad_arena, plan.grad_arena[s:e],
                                        group=plan.grad_group))
