"""`kfac.utils` surface: work distribution, tracing and small helpers."""
from .distribution import (load_balance, balance_batched, partition_grad_ranks, partition_inv_ranks,
                           WorkerAllocator, get_block_boundary, try_contiguous)
from .tracing import trace, get_trace, print_trace, clear_trace, PhaseTimer

__all__ = ['load_balance', 'balance_batched', 'partition_grad_ranks', 'partition_inv_ranks',
           'WorkerAllocator', 'get_block_boundary', 'try_contiguous',
           'trace', 'get_trace', 'print_trace', 'clear_trace', 'PhaseTimer']
