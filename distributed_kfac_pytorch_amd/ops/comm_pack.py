"""Symmetric-factor packing for communication (K12).

pack_triu:   n x n symmetric -> n(n+1)/2 upper triangle (row-major) into `out`
unpack_triu: packed -> full symmetric matrix divided by `divisor` (folds the
             1/world of an AVERAGE all-reduce into the unpack)
GPU: csrc/factors.hip triu kernels (LDS-tiled transpose for the mirror).
CPU: index gather/scatter with cached triu indices.
Reference analogue: get_triu / fill_triu (kfac/layers/utils.py:126-162),
which the reference never enabled for communication.
"""
import torch

from . import _lib

__all__ = ['triu_numel', 'pack_triu', 'unpack_triu']

_idx_cache = {}


def triu_numel(n):
    return n * (n + 1) // 2


def _triu_idx(n, device):
    key = (n, str(device))
    idx = _idx_cache.get(key)
    if idx is None:
        r, c = torch.triu_indices(n, n, device=device)
        idx = (r * n + c, c * n + r)
        _idx_cache[key] = idx
    return idx


def pack_triu(mat, out):
    n = mat.shape[0]
    if _lib.use_native(mat):
        if mat.dtype != out.dtype or not mat.is_contiguous():
            raise ValueError('pack_triu expects a contiguous matrix of the arena dtype')
        _lib.check(_lib.lib().kfac_triu_pack(_lib.DTYPE_CODE[mat.dtype], _lib.ptr(mat),
                                             _lib.ptr(out), n, _lib.stream(mat.device)),
                   'kfac_triu_pack')
        return out
    up, _ = _triu_idx(n, mat.device)
    torch.index_select(mat.reshape(-1), 0, up, out=out)
    return out


def unpack_triu(packed, mat, divisor=1):
    """mat <- sym(packed) / divisor."""
    n = mat.shape[0]
    if _lib.use_native(mat):
        _lib.check(_lib.lib().kfac_triu_unpack(_lib.DTYPE_CODE[mat.dtype], _lib.ptr(packed),
                                               _lib.ptr(mat), n, 1.0 / float(divisor),
                                               _lib.stream(mat.device)), 'kfac_triu_unpack')
        return mat
    up, low = _triu_idx(n, mat.device)
    vals = packed / divisor if divisor != 1 else packed
    flat = mat.view(-1)
    flat[up] = vals
    flat[low] = vals
    return mat
