"""Cross-rank consistency checks for K-FAC communication (debug mode).

SURVEY.md section 5.2 lists the reference's silent-corruption hazards: a
broadcast of a non-contiguous eigenvector buffer corrupts receivers without an
error (reference kfac/layers/base.py:143-159 with kfac/layers/utils.py:45-74),
`TorchBackend.sync` decides "average or not" from the first handle only
(reference kfac/comm.py:254-271), and a rank-order mismatch of sub-group
creation deadlocks (reference kfac/comm.py:58).  The reference has no way to
detect the first two.  This module is the detector: after each collective
phase of `KFAC.step()` every rank checksums the buffers that must now be
bitwise identical across ranks and compares the checksums with MAX and MIN
all-reduces of small fp64 vectors.  A mismatch raises
`CommConsistencyError` naming the offending layer buffers.

Enabled by `KFAC(..., comm_check=True)` or the environment variable
`KFAC_COMM_CHECK=1`.  It synchronises the device and costs four small
all-reduces per checked phase, so it is a debugging aid, not a production
default.

What must agree, per phase (section 3.5 of SURVEY.md):
  * after the factor all-reduce: A and G of every layer, on every rank
  * after the eigendata broadcast (COMM_OPT): QA, QG and dGdA (or dA, dG),
    or A_inv and G_inv, of every layer, on every rank
  * after the gradient broadcast (MEM_OPT): every layer's preconditioned
    gradient, on every rank
"""
import torch
import torch.distributed as dist

__all__ = ['CommConsistencyError', 'checksums', 'assert_consistent']

_NAN_SENTINEL = 1.0e300


class CommConsistencyError(RuntimeError):
    """Buffers that must be identical across ranks differ after a collective."""


def checksums(tensors):
    """fp64 [len(tensors), 2]: plain sum and position-weighted sum per tensor
    (the weighted sum catches permutations, e.g. a transposed eigenvector
    matrix, which a plain sum misses).  NaN/inf map to fixed sentinels so the
    MIN/MAX comparison stays meaningful."""
    if not tensors:
        return torch.zeros(0, 2, dtype=torch.float64)
    dev = tensors[0].device
    rows = []
    for t in tensors:
        x = t.detach().reshape(-1).to(torch.float64)
        w = 1.0 + (torch.arange(x.numel(), device=dev, dtype=torch.float64) % 7)
        s = torch.stack([x.sum(), (x * w).sum()])
        rows.append(torch.nan_to_num(s, nan=_NAN_SENTINEL, posinf=2 * _NAN_SENTINEL,
                                     neginf=-2 * _NAN_SENTINEL))
    return torch.stack(rows)


def assert_consistent(named_tensors, phase, group=None):
    """Raise CommConsistencyError unless every (name, tensor) pair is bitwise
    identical (by checksum) on every rank of `group`.  Collective: every rank
    must call it with the same names in the same order."""
    if not dist.is_available() or not dist.is_initialized():
        return
    if dist.get_world_size(group) <= 1:
        return
    names = [n for n, _ in named_tensors]
    c = checksums([t for _, t in named_tensors])
    # the reduction runs on the process group's device (gloo: CPU, RCCL: GPU)
    backend = dist.get_backend(group)
    dev = torch.device('cuda', torch.cuda.current_device()) \
        if backend == 'nccl' else torch.device('cpu')
    c = c.to(dev)
    # the buffer lists must agree first (a rank-order mismatch of layers, or a
    # buffer one rank lacks); a differently sized checksum all-reduce would be
    # a collective mismatch, so the list signature travels on its own
    sig = torch.tensor([float(len(names)), float(sum(len(n) for n in names))],
                       dtype=torch.float64, device=dev)
    shi, slo = sig.clone(), sig.clone()
    dist.all_reduce(shi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(slo, op=dist.ReduceOp.MIN, group=group)
    if not torch.equal(shi, slo):
        raise CommConsistencyError('{}: ranks disagree on the checked buffer list '
                                   '(rank {}: {} buffers)'.format(phase, dist.get_rank(),
                                                                  len(names)))
    hi, lo = c.reshape(-1).clone(), c.reshape(-1).clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    if bool(torch.equal(hi, lo)):
        return
    diff = (hi != lo).reshape(-1, 2).any(dim=1).cpu().tolist()
    bad = [n for n, d in zip(names, diff) if d]
    raise CommConsistencyError('{}: {} buffer(s) differ across ranks (rank {}): {}'.format(
        phase, len(bad), dist.get_rank(), ', '.join(bad[:16]) + (' ...' if len(bad) > 16 else '')))
