"""ctypes binding to the in-tree gfx950 kernel library (`_native/libkfac_hip.so`).

The library exposes a plain C ABI (csrc/*.hip, `KFAC_API` functions); every
entry point takes raw device pointers plus the hipStream_t of torch's
current stream, so kernels are stream-ordered with PyTorch work and can be
captured into hipGraphs.  On a GPU process the library is REQUIRED: the
ops fail loudly instead of silently falling back (the CPU plumbing path is
used only for CPU tensors).
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_HERE, '_native', 'libkfac_hip.so')

_lock = threading.Lock()
_lib = None
_load_error = None

DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}

c_vp = ctypes.c_void_p
c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_f = ctypes.c_float
c_d = ctypes.c_double


class MatRecord(ctypes.Structure):
    _fields_ = [('v', c_vp), ('g', c_vp), ('ldv', c_ll), ('rows', c_ll), ('cols', c_ll),
                ('gdtype', c_ll), ('gs0', c_ll), ('gs1', c_ll), ('gs2', c_ll), ('gs3', c_ll),
                ('kk', c_ll), ('kw', c_ll)]


class EigRecord(ctypes.Structure):
    _fields_ = [('A', c_vp), ('Q', c_vp), ('d', c_vp), ('Vt', c_vp), ('n', c_ll)]


class ReduceRecord(ctypes.Structure):
    # csrc/eig_reduce.hip KfacReduceRecord
    _fields_ = [('A', c_vp), ('lda', c_ll), ('d', c_vp), ('e', c_vp), ('tau', c_vp),
                ('ws', c_vp), ('n', c_ll)]


class CholRecord(ctypes.Structure):
    """Mirror of csrc/chol.hip KfacCholRecord."""
    _fields_ = [('F', ctypes.c_void_p), ('ldf', ctypes.c_longlong), ('out', ctypes.c_void_p),
                ('ldo', ctypes.c_longlong), ('ws', ctypes.c_void_p), ('n', ctypes.c_longlong)]


class DcRecord(ctypes.Structure):
    # csrc/eig_dc.hip KfacDcRecord
    _fields_ = [('d', c_vp), ('e', c_vp), ('dout', c_vp), ('Zout', c_vp), ('ldz', c_ll),
                ('ws', c_vp), ('n', c_ll)]


class Sy2sbRecord(ctypes.Structure):
    # csrc/eig_sy2sb.hip KfacSy2sbRecord
    _fields_ = [('A', c_vp), ('lda', c_ll), ('tau', c_vp), ('band', c_vp), ('ws', c_vp),
                ('n', c_ll)]


class Sb2stRecord(ctypes.Structure):
    # csrc/eig_sb2st.hip KfacSb2stRecord
    _fields_ = [('band_in', c_vp), ('band', c_vp), ('v2', c_vp), ('d', c_vp), ('e', c_vp),
                ('ldv2', c_ll), ('n', c_ll), ('status', c_vp)]


class Q2Record(ctypes.Structure):
    # csrc/eig_q2.hip KfacQ2Record
    _fields_ = [('Z', c_vp), ('v2', c_vp), ('ldz', c_ll), ('ldv2', c_ll), ('n', c_ll)]


_SIGS = {
    'kfac_sy2sb_batched': [ctypes.POINTER(Sy2sbRecord), c_int, c_int, c_vp],
    'kfac_sy2sb_ws_floats': [c_ll],
    'kfac_sy2sb_nmax': [],
    'kfac_sb2st_batched': [ctypes.POINTER(Sb2stRecord), c_int, c_int, c_vp],
    'kfac_backtransform_slabs': [c_int],
    'kfac_backtransform_block': [],
    'kfac_event_create': [],
    'kfac_event_destroy': [c_vp],
    'kfac_event_record_external': [c_vp, c_vp],
    'kfac_stream_wait_external': [c_vp, c_vp],
    'kfac_sb2st_debug_stamps': [ctypes.POINTER(ctypes.c_longlong), c_int],
    'kfac_sb2st_debug_phases': [ctypes.POINTER(ctypes.c_longlong)],
    'kfac_q2_batched': [ctypes.POINTER(Q2Record), c_int, c_int, c_vp],
    'kfac_q2_nmax': [],
    'kfac_band_backtransform': [c_vp, c_int, c_ll, c_vp, c_vp, c_int, c_ll, c_int, c_int,
                                c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp],
    'kfac_syrk_patch': [c_int, c_vp, c_ll, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_vp, c_int,
                        c_int, c_vp, c_vp, c_vp],
    'kfac_factor_ema': [c_int, c_vp, c_vp, c_int, c_int, c_f, c_int, c_vp, c_vp],
    'kfac_syrk_vec': [c_int, c_vp, c_ll, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_vp, c_int,
                      c_int, c_vp, c_vp, c_vp],
    'kfac_syrk_splits': [c_int, c_ll, c_int, c_int],
    'kfac_chol_inverse_batched': [c_vp, c_int, c_f, c_int, c_vp],
    'kfac_chol_ws_bytes': [c_int],
    'kfac_chol_info_offset': [c_int],
    'kfac_syrk_problem_set_part': [c_vp, c_vp],
    'kfac_syrk_problem_set_dscale': [c_vp, c_vp],
    'kfac_red_job_size': [],
    'kfac_red_max_contrib': [],
    'kfac_tile_reduce': [c_vp, c_int, c_vp],
    'kfac_syrk_problem_size': [],
    'kfac_ema_job_size': [],
    'kfac_syrk_problem_init': [c_vp, c_int, c_int, c_vp, c_ll, c_ll, c_ll, c_ll, c_int, c_int,
                               c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_int, c_f, c_vp, c_int, c_ll, c_int],
    'kfac_syrk_grouped': [c_vp, c_int, c_int, c_vp],
    'kfac_ema_grouped': [c_vp, c_int, c_vp],
    'kfac_split_f16': [c_vp, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_vp, c_vp,
                       c_vp, c_vp],
    'kfac_split_blocks': [],
    'kfac_factor_ema_perm': [c_int, c_vp, c_vp, c_int, c_int, c_f, c_int, c_int, c_int, c_int,
                             c_vp, c_vp],
    'kfac_triu_pack': [c_int, c_vp, c_vp, c_int, c_vp],
    'kfac_triu_unpack': [c_int, c_vp, c_vp, c_int, c_f, c_vp],
    'kfac_grouped_kl_dot': [ctypes.POINTER(MatRecord), c_int, c_vp, c_vp],
    'kfac_grouped_apply': [ctypes.POINTER(MatRecord), c_int, c_vp, c_d, c_d, c_int, c_vp],
    'kfac_outer_recip': [c_vp, c_vp, c_vp, c_int, c_int, c_f, c_vp],
    'kfac_hadamard': [c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_f, c_int, c_vp],
    'kfac_eig_jacobi_small': [ctypes.POINTER(EigRecord), c_int, c_int, c_f, c_int, c_f, c_vp],
    'kfac_max_small_eig_n': [],
    'kfac_tridiag_backtransform': [c_vp, c_int, c_ll, c_vp, c_vp, c_int, c_ll, c_int, c_int,
                                   c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
    'kfac_backtransform_prepare': [c_vp, c_int, c_ll, c_vp, c_vp, c_int, c_ll, c_int, c_int,
                                   c_vp, c_vp, c_vp, c_vp],
    'kfac_pgemm': [c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp],
    'kfac_kl_finalize': [c_vp, c_int, c_vp, c_vp],
    'kfac_kl_elems_per_block': [],
    'kfac_gather_grad': [c_int, c_vp, c_int, c_vp],
    'kfac_split_copy': [c_int, c_vp, c_int, c_int, c_vp],
    'kfac_pgemm_record_size': [],
    'kfac_gather_record_size': [],
    'kfac_split_record_size': [],
    'kfac_graph_fix_memsets': [c_vp, c_int, ctypes.POINTER(c_ll)],
    'kfac_dc_batched': [ctypes.POINTER(DcRecord), c_int, c_int, c_vp],
    'kfac_cast_grouped': [c_vp, c_int, c_int, c_vp],
    'kfac_reduce_batched': [ctypes.POINTER(ReduceRecord), c_int, c_int, c_vp],
    'kfac_reduce_prepare': [ctypes.POINTER(ReduceRecord), c_int],
    'kfac_reduce_ws_floats': [c_int],
    'kfac_reduce_set_tail': [c_int],
    'kfac_reduce_stamps': [c_vp],
    'kfac_dc_prepare': [ctypes.POINTER(DcRecord), c_int],
    'kfac_dc_ws_bytes': [c_int],
    'kfac_dc_set_fast_scan': [c_int],
    'kfac_dc_info_offset': [c_int],
    'kfac_bn_ws_floats': [c_ll, c_int],
    'kfac_bn_forward': [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll,
                        c_int, ctypes.c_float, ctypes.c_float, c_int, c_vp],
    'kfac_bn_backward': [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll,
                         c_int, c_int, c_vp],
}


_RESTYPES = {'kfac_dc_ws_bytes': c_ll, 'kfac_sy2sb_ws_floats': c_ll,
             'kfac_reduce_ws_floats': c_ll, 'kfac_syrk_splits': c_ll,
             'kfac_chol_ws_bytes': c_ll, 'kfac_chol_info_offset': c_ll,
             'kfac_syrk_problem_set_part': None, 'kfac_syrk_problem_set_dscale': None,
             'kfac_bn_ws_floats': c_ll, 'kfac_event_create': c_vp}


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None or _load_error is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            _load_error = 'native library not built: {} (run `python csrc/build.py`)'.format(LIB_PATH)
            return None
        try:
            lib = ctypes.CDLL(LIB_PATH)
            for name, argt in _SIGS.items():
                if name in OPTIONAL and not hasattr(lib, name):
                    continue          # built only with KFAC_BUILD_TWO_STAGE=1
                fn = getattr(lib, name)
                fn.argtypes = argt
                fn.restype = _RESTYPES.get(name, c_int)
            _lib = lib
        except OSError as e:
            _load_error = str(e)
        return _lib


# entry points of the opt-in two-stage solver (csrc/build.py TWO_STAGE_SOURCES)
OPTIONAL = frozenset(['kfac_sy2sb_batched', 'kfac_sy2sb_ws_floats', 'kfac_sy2sb_nmax',
                      'kfac_sb2st_batched', 'kfac_sb2st_debug_stamps', 'kfac_sb2st_debug_phases',
                      'kfac_q2_batched', 'kfac_q2_nmax'])


def has(name):
    """True when the loaded library exports `name` (optional entry points)."""
    l = _load()
    return l is not None and hasattr(l, name)


def available():
    return _load() is not None


def lib():
    """The loaded library; raises (never falls back) when it is missing."""
    l = _load()
    if l is None:
        raise RuntimeError('distributed_kfac_pytorch_amd native kernels unavailable: ' +
                           str(_load_error))
    return l


def use_native(t):
    """True when tensor `t` must go through the HIP kernels."""
    if t is None or not t.is_cuda:
        return False
    lib()  # loud failure on a GPU tensor without the library
    return True


def stream(device=None):
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return c_vp(t.data_ptr())


def check(err, name):
    if err != 0:
        raise RuntimeError('{} failed with HIP error {}'.format(name, err))


# The grouped MFMA GEMM (csrc/precond_gemm.hip) addresses every operand with
# 32-bit offsets: a factor dimension n (padded row length <= n + 63) must keep
# n x ld x 4 bytes below 4 GiB.
PGEMM_MAX_N = 32704


def check_pgemm_extent(n, what='factor'):
    if n > PGEMM_MAX_N:
        raise ValueError('{} dimension {} exceeds the native kernels\' limit of {} '
                         '(32-bit operand offsets)'.format(what, n, PGEMM_MAX_N))


# Replace captured memset nodes by fill kernels (csrc/graph_fix.hip); 0 = keep
# them (A/B runs of the ROCm 7.2 memset-node issue)
FIX_GRAPH_MEMSETS = os.environ.get('KFAC_GRAPH_FIX_MEMSETS', '1') != '0'
graph_memset_stats = {'graphs': 0, 'memsets': 0, 'bytes': 0, 'replaced': 0}


def new_graph():
    """A torch.cuda.CUDAGraph that keeps its hipGraph after capture, so that
    finalize_graph() can rewrite it before it is instantiated."""
    return torch.cuda.CUDAGraph(keep_graph=True)


def finalize_graph(g):
    """Rewrite the memset nodes of a graph captured with new_graph() into
    kernel nodes (captured memset nodes do not reliably clear their target on
    replay with this ROCm runtime: csrc/graph_fix.hip), then instantiate it."""
    stats = (c_ll * 3)()
    check(lib().kfac_graph_fix_memsets(c_vp(g.raw_cuda_graph()), int(FIX_GRAPH_MEMSETS), stats),
          'kfac_graph_fix_memsets')
    st = graph_memset_stats
    st['graphs'] += 1
    st['memsets'] += stats[0]
    st['bytes'] += stats[1]
    st['replaced'] += stats[2]
    g.instantiate()
    return g


_ws = {}
_retired = []


def workspace(device, numel, dtype=torch.float32, tag='main'):
    """A grow-only scratch buffer per (device, tag, dtype); stream-ordered reuse.

    A buffer that is outgrown is retired but never freed: a hipGraph captured
    earlier may still address it, and freeing it would let the allocator hand
    that memory to another tensor while the graph keeps writing into it."""
    key = (str(device), tag, dtype)
    buf = _ws.get(key)
    if buf is None or buf.numel() < numel:
        if buf is not None:
            _retired.append(buf)
        buf = torch.empty(max(numel, 1), dtype=dtype, device=device)
        _ws[key] = buf
    return buf[:numel]
