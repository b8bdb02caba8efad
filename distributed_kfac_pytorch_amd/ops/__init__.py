"""gfx950 HIP kernels (csrc/) bound through ctypes, plus their CPU twins.

_lib       library loader (fails loudly on GPU tensors when not built)
factors    implicit-im2col MFMA SYRK + fused EMA (K1-K5)
eigen      batched Jacobi eigensolver (K6) / Cholesky inverse (K9)
precond    eigenbasis preconditioning, grouped KL-dot + apply (K7, K8, K10, K11)
comm_pack  triu pack/unpack for the factor all-reduce arena (K12)
"""
from . import _lib, factors, eigen, precond, comm_pack

__all__ = ['_lib', 'factors', 'eigen', 'precond', 'comm_pack', 'native_available']


def native_available():
    return _lib.available()
