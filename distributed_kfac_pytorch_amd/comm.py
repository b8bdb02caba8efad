"""Communication backends for K-FAC traffic.

API parity with the reference (kfac/comm.py:1-275): a module-global
`backend`, `init_comm_backend()`, `CommGroup(ranks)`, `Ops.{Average,Sum}`
and `backend.{size,rank,local_rank,allreduce,broadcast,reduce,barrier,
sync,wait}`.

Differences by design (SURVEY.md section 7.4 defects #6/#7):
  * No Horovod.  Selection is torch.distributed (RCCL on ROCm, gloo on CPU)
    > null single-process backend.
  * AVERAGE over a sub-group divides by the *group* size, and the post-wait
    division is carried by each handle (the reference inspected only
    `handles[0]`).
  * `local_rank()` returns an int.
  * K-FAC traffic has a communicator of its own (`TorchBackend.kfac_world`),
    created once when the backend is selected: with RCCL and a process group
    bound to its GPU it is split off the default communicator
    (`dist.split_group` -> ncclCommSplit), otherwise a plain `new_group`.
    Its collectives run on that communicator's own HIP stream, so the
    factor all-reduce and the eigendata / gradient all-gathers never queue
    behind the data-parallel gradient all-reduce on the default group, and
    are ordered against the compute stream by events only (SURVEY.md
    5.8.1; reference: one torch group per layer collective,
    kfac/comm.py:53-64,194-275).
  * Sub-communicators (HYBRID_OPT / MEM_OPT inverse and gradient groups) are
    created per PARTITION of the world (`CommGroup.partition`): one
    ncclCommSplit of the K-FAC world for the whole partition on RCCL, one
    `new_group` per member group otherwise; every rank creates them in the
    same order (the execution plan does so once, at build time).

The bulk K-FAC traffic does not go through these per-tensor calls on the
fast path: parallel/collectives.py packs factors, eigendata and gradients
into flat arenas and issues one collective per bucket / per root.
"""
import enum
import os

import torch
import torch.distributed as dist

__all__ = ['Ops', 'CommGroup', 'CommBackend', 'TorchBackend', 'Handle',
           'init_comm_backend', 'reset_comm_backend', 'backend', 'build_log']

backend = None
# every communicator construction, in program order (identical on every rank;
# bench.py reports it so a multi-GPU run says how its groups were built)
build_log = []


def _record(what, method, ranks):
    build_log.append({'what': what, 'method': method,
                      'ranks': [list(r) for r in ranks] if ranks and
                      isinstance(ranks[0], (list, tuple)) else list(ranks)})


class Ops(enum.Enum):
    Average = 'average'
    Sum = 'sum'


def init_comm_backend():
    """Select the backend once: torch.distributed if initialised, else null."""
    global backend
    if backend is None:
        backend = TorchBackend() if _dist_ready() else CommBackend()
    return backend


def reset_comm_backend():
    """Forget the selected backend and cached groups (tests / re-init)."""
    global backend
    backend = None
    del build_log[:]
    CommGroup._cache.clear()
    CommGroup._partitions.clear()


def _can_split():
    """ncclCommSplit is requested (KFAC_COMM_SPLIT=1) and available: RCCL/NCCL
    default group bound to a device (init_process_group(device_id=...),
    parallel/launch.py) and a torch with dist.split_group.  Identical on every
    rank.  Off by default: the split path has run only on gloo with a
    recorded split_group (tests/test_distributed.py); plain new_group
    communicators are the path every torch / RCCL build exercises."""
    if not (_dist_ready() and hasattr(dist, 'split_group')):
        return False
    if os.environ.get('KFAC_COMM_SPLIT', '0') != '1':
        return False
    if dist.get_backend() != 'nccl':
        return False
    pg = dist.distributed_c10d._get_default_group()
    return getattr(pg, 'bound_device_id', None) is not None


def _new_world_group():
    world = dist.get_world_size()
    if world <= 1:
        return None
    ranks = list(range(world))
    if _can_split():
        try:
            g = dist.split_group(split_ranks=[ranks], group_desc='kfac_world')
            _record('kfac_world', 'split_group', ranks)
            return g
        except Exception as e:   # pragma: no cover - depends on the RCCL build
            # an API-level refusal is the same on every rank: all fall back
            import warnings
            warnings.warn('ncclCommSplit of the K-FAC world failed ({}); using new_group'
                          .format(e))
    _record('kfac_world', 'new_group', ranks)
    return dist.new_group(ranks)


def _dist_ready():
    return dist.is_available() and dist.is_initialized()


class CommGroup(object):
    """A set of ranks plus its communicator.

    `group` is None when the ranks are the whole world (collectives use the
    K-FAC world communicator) or a single rank (collectives are no-ops).
    """
    _cache = {}
    _partitions = {}

    def __init__(self, ranks, group=None, create=True):
        self.ranks = sorted(int(r) for r in ranks)
        key = tuple(self.ranks)
        self.group = group
        # create=False: bookkeeping for a group this rank is not in whose
        # communicator came from a collective split (new_group is collective
        # over the world: calling it on some ranks only would mismatch)
        if group is None and create and _dist_ready():
            world = dist.get_world_size()
            if 1 < len(self.ranks) < world:
                if key not in CommGroup._cache:
                    _record('group', 'new_group', self.ranks)
                    CommGroup._cache[key] = dist.new_group(self.ranks)
                self.group = CommGroup._cache[key]

    @classmethod
    def partition(cls, rank_lists):
        """CommGroups for a partition of the world (disjoint rank lists
        covering every rank), created collectively: on RCCL one
        ncclCommSplit of the K-FAC world for the whole partition (this
        rank's group is a real communicator, the others are bookkeeping),
        else one new_group per list.  Cached by the partition."""
        lists = [sorted(int(r) for r in g) for g in rank_lists]
        key = tuple(tuple(g) for g in lists)
        if key in cls._partitions:
            return cls._partitions[key]
        if not _dist_ready():
            out = [cls(g) for g in lists]
        else:
            world = dist.get_world_size()
            cover = sorted(r for g in lists for r in g)
            if cover != list(range(world)):
                raise ValueError('not a partition of the world: {}'.format(lists))
            multi = [g for g in lists if 1 < len(g) < world]
            if multi and _can_split() and isinstance(backend, TorchBackend) and \
                    backend.kfac_world is not None:
                me = dist.get_rank()
                # split_ranks are ranks of the parent (the K-FAC world spans
                # every rank in order: parent rank == global rank)
                mine = dist.split_group(parent_pg=backend.kfac_world, split_ranks=multi,
                                        group_desc='kfac_sub')
                _record('partition', 'split_group', multi)
                out = [cls(g, group=mine if (me in g and 1 < len(g) < world) else None,
                           create=False) for g in lists]
            else:
                out = [cls(g) for g in lists]
        cls._partitions[key] = out
        return out

    @property
    def size(self):
        return len(self.ranks)

    def __contains__(self, rank):
        return rank in self.ranks

    def __repr__(self):
        return 'CommGroup({})'.format(self.ranks)


class Handle(object):
    """Async work handle; `wait()` finishes the op including any averaging."""
    __slots__ = ('work', 'tensor', 'divisor')

    def __init__(self, work, tensor=None, divisor=None):
        self.work, self.tensor, self.divisor = work, tensor, divisor

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        if self.divisor is not None:
            self.tensor.div_(self.divisor)
            self.divisor = None


class CommBackend(object):
    """Single-process backend: size 1, every collective is a no-op."""
    Average = Ops.Average
    Sum = Ops.Sum

    def size(self):
        return 1

    def rank(self):
        return 0

    def local_rank(self):
        return 0

    def allreduce(self, tensor, op=Ops.Average, group=None, async_op=True):
        return None

    def broadcast(self, tensor, src, group=None, async_op=True):
        return None

    def reduce(self, tensor, dst, op=Ops.Average, group=None, async_op=True):
        return None

    def allgather(self, outputs, tensor, group=None, async_op=True):
        for o in outputs:
            o.copy_(tensor)
        return None

    def allgather_into(self, output, tensor, group=None, async_op=True):
        """output = concat of every group rank's `tensor` (group-rank order);
        `tensor` may be this rank's slice of `output` (in place)."""
        if tensor.data_ptr() != output.data_ptr() or tensor.numel() != output.numel():
            output.view(-1)[:tensor.numel()].copy_(tensor.view(-1))
        return None

    def barrier(self):
        return None

    def counters(self):
        return {}

    def sync(self, handles):
        if handles is None:
            return
        if not isinstance(handles, (list, tuple)):
            handles = [handles]
        for h in handles:
            self.wait(h)

    def wait(self, handle):
        if handle is not None:
            handle.wait()


class TorchBackend(CommBackend):
    """torch.distributed backend (RCCL over xGMI on MI355X, gloo on CPU).

    `kfac_world`: the dedicated K-FAC communicator over all ranks (None at
    world size 1), created here -- every rank selects the backend at the
    same program point (KFAC construction / parallel.launch.init_distributed).
    """

    def __init__(self):
        self.kfac_world = _new_world_group()
        self.stats = {}     # op -> [calls, bytes] issued by this rank

    def _count(self, op, tensor):
        st = self.stats.setdefault(op, [0, 0])
        st[0] += 1
        st[1] += tensor.numel() * tensor.element_size()

    def counters(self):
        """{op: (calls, bytes)} of every collective this backend issued."""
        return {k: tuple(v) for k, v in self.stats.items()}

    def size(self):
        return dist.get_world_size()

    def rank(self):
        return dist.get_rank()

    def local_rank(self):
        v = os.environ.get('LOCAL_RANK')
        if v is None:
            raise RuntimeError('LOCAL_RANK must be set in the environment '
                               'when using torch.distributed')
        return int(v)

    def _resolve(self, group):
        """-> (skip, kwargs, group_size).  None / a world-sized group -> the
        K-FAC world communicator."""
        world_kw = {'group': self.kfac_world} if self.kfac_world is not None else {}
        if group is None:
            return False, world_kw, dist.get_world_size()
        if group.size <= 1:
            return True, {}, 1
        kw = {'group': group.group} if group.group is not None else world_kw
        return False, kw, group.size

    def allreduce(self, tensor, op=Ops.Average, group=None, async_op=True):
        skip, kw, gsize = self._resolve(group)
        if skip:
            return None
        divisor = gsize if op == Ops.Average else None
        self._count('all_reduce', tensor)
        work = dist.all_reduce(tensor, async_op=async_op, **kw)
        h = Handle(work if async_op else None, tensor, divisor)
        if not async_op:
            h.wait()
            return None
        return h

    def broadcast(self, tensor, src, group=None, async_op=True):
        skip, kw, _ = self._resolve(group)
        if skip:
            return None
        self._count('broadcast', tensor)
        work = dist.broadcast(tensor, src=src, async_op=async_op, **kw)
        return Handle(work) if async_op else None

    def reduce(self, tensor, dst, op=Ops.Average, group=None, async_op=True):
        skip, kw, gsize = self._resolve(group)
        if skip:
            return None
        self._count('reduce', tensor)
        work = dist.reduce(tensor, dst=dst, async_op=async_op, **kw)
        divisor = gsize if (op == Ops.Average and self.rank() == dst) else None
        h = Handle(work if async_op else None, tensor, divisor)
        if not async_op:
            h.wait()
            return None
        return h

    def allgather(self, outputs, tensor, group=None, async_op=True):
        skip, kw, _ = self._resolve(group)
        if skip:
            outputs[0].copy_(tensor)
            return None
        self._count('all_gather', tensor)
        work = dist.all_gather(outputs, tensor, async_op=async_op, **kw)
        return Handle(work) if async_op else None

    def allgather_into(self, output, tensor, group=None, async_op=True):
        skip, kw, _ = self._resolve(group)
        if skip:
            return super().allgather_into(output, tensor)
        self._count('all_gather_into_tensor', output)
        work = dist.all_gather_into_tensor(output, tensor, async_op=async_op, **kw)
        return Handle(work) if async_op else None

    def barrier(self):
        if self.kfac_world is not None:
            dist.barrier(group=self.kfac_world)
        else:
            dist.barrier()
