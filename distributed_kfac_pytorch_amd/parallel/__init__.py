"""Distributed execution: static plan + bucketed RCCL collectives + DDP helpers."""
from .plan import ExecutionPlan
from .collectives import FactorAllreduce, broadcast_eigendata, broadcast_gradients
from .launch import init_distributed, wrap_ddp, get_local_device

__all__ = ['ExecutionPlan', 'FactorAllreduce', 'broadcast_eigendata', 'broadcast_gradients',
           'init_distributed', 'wrap_ddp', 'get_local_device']
