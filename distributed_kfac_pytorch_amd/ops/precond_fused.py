"""Grouped, fused eigenbasis preconditioning for every layer of a rank (K7/K8/K10).

`FusedPreconditioner` owns per-layer MFMA operand buffers and runs the chain

    gather(.grad)  ->  S1 QG^T Grad  ->  S2 ((.) QA) (.) D  ->  S3 QG (.)  ->  S4 (.) QA^T  + KL dot

as 5 launches for ALL layers (csrc/precond_gemm.hip) instead of 4 library
GEMMs + a Hadamard launch per layer (reference kfac/layers/base.py:321-362,459-470
does the per-layer form).  The preconditioned gradient lands in the plan's
gradient arena (`layer.pgrad_buffer`), and <v, g> summed over all layers lands
in a device f64 scalar for the KL clip (reference kfac/preconditioner.py:661-682),
so `KFAC.step()` needs no host synchronisation.

Precision (`precision=`):
  'bf16x3'  operands kept as bf16 (hi, lo) pairs, three bf16 MFMAs per
            product, fp32 accumulation: ~1e-5 relative error on the
            preconditioned gradient (tests/test_gpu_precond_fused.py),
            ~5x the fp32 MFMA rate.
  'bf16x6'  operands as three bf16 planes (hi, mid, lo = the fp32
            significand), six bf16 MFMAs per product (every term above 2^-24
            relative), fp32 accumulation: fp32-level error at the bf16 rate.
            The eigenvector operands are stored as planes (split once per
            inverse update); the per-step operands stay fp32 and are split
            while the kernel stages them into LDS (PREC_BF16X6A / _B): half
            the k-loop split work of splitting both (PREC_BF16X6F,
            KFAC_X6_MODE=fp32); KFAC_X6_MODE=planes keeps the round-2
            all-planes kernel.  All three give bitwise-equal results.
  'fp32'    fp32 operands on the exact f32 MFMA (the reference's fp32 math).

Static GEMM tables (all pointers are arena/buffer pointers that never move)
are uploaded once; the .grad gather table is passed by value in the kernel
arguments and rebuilt on the host whenever a `.grad` tensor moved (e.g.
`zero_grad(set_to_none=True)`), so graph-captured and eager launches never
share a mutable table.
"""
import ctypes

import os

import torch

from . import _lib

__all__ = ['FusedPreconditioner', 'PRECISIONS']

PRECISIONS = {'fp32': 0, 'bf16x3': 1, 'bf16x6': 2, 'fp16x3': 6}
PLANES = {'fp32': 1, 'bf16x3': 2, 'bf16x6': 3, 'fp16x3': 1}
# Low-plane mixed modes (csrc/pgemm.h): the eigenvector operands stored once per
# inverse update as 16-bit planes, the per-step operands fp32 and converted
# while staged; fp16 operands carry a power-of-two scale (eigenvectors 2^14,
# the per-step operand from the max |x| its producer recorded).
#   'fp16x3'  fp16 hi / lo planes, 3 MFMAs per product (22 significand bits)
#   'bf16x1' / 'fp16x1'  one plane, one MFMA: KFAC(inv_dtype=bfloat16 / float16)
# name -> (stage prec with the planes as A, as B, split store mode, planes,
#          plane dtype, scaled)
LP_CFG = {'fp16x3': (6, 7, 20, 2, torch.float16, True),
          'bf16x1': (8, 9, 21, 1, torch.bfloat16, False),
          'fp16x1': (10, 11, 22, 1, torch.float16, True)}
LP_QSCALE = 2.0 ** 14          # csrc/pgemm.h LP_QEXP
# the chain precision KFAC(inv_dtype=...) runs on when it is not float32
INV_DTYPE_PRECISION = {torch.bfloat16: 'bf16x1', torch.float16: 'fp16x1'}
PREC_BF16X6F = 3   # csrc/pgemm.h: bf16x6 products on fp32 operands, planes split into LDS
PREC_BF16X6A, PREC_BF16X6B = 4, 5   # one operand (A / B) stored as planes, the other fp32
# bf16x6 operand storage (same products, same order, bitwise-equal results):
#   'mixed'  (default) the eigenvector operands QG^T, QA^T, QG, QA as three
#            bf16 planes, split once per inverse update; the per-step operands
#            (gathered gradient, intermediates) fp32, split while staged
#   'fp32'   every operand fp32, split while staged (PREC_BF16X6F, round 3-4)
#   'planes' every operand as planes (the round-2 kernel)
# KFAC_X6_MODE selects; KFAC_X6_PLANES=1 is the old spelling of 'planes'
X6_MODE = os.environ.get('KFAC_X6_MODE') or \
    ('planes' if os.environ.get('KFAC_X6_PLANES') == '1' else 'mixed')
X6_PLANES = X6_MODE == 'planes'
X6_BIG = int(os.environ['KFAC_X6_BIG']) if os.environ.get('KFAC_X6_BIG') else None
LP_BIG = int(os.environ['KFAC_LP_BIG']) if os.environ.get('KFAC_LP_BIG') else None
EPI_STORE, EPI_HADAMARD, EPI_HADAMARD_VEC, EPI_FINAL = 0, 1, 2, 3
TILE = 128        # small tile class (csrc/precond_gemm.hip)
BIG_TILE = 256    # big tile class: half the operand traffic per FLOP


BIG_TILES = False  # measured 2.7x slower on ResNet-50 (profiles/r1_pgemm_variants.log)
# kernel tile configurations of csrc/precond_gemm.hip: id -> (BM, BN)
TILE_SHAPES = {0: (128, 128), 1: (256, 256), 2: (64, 64), 3: (128, 128), 4: (128, 64),
               5: (128, 128), 6: (256, 128), 7: (128, 256), 8: (128, 128), 9: (128, 128),
               10: (128, 128), 11: (128, 128)}
# tile configuration of every problem not in the big class, per precision.
# Round 2 (branch-free operand loads, record in scalar registers; the k-step
# loads now really stay in flight under the MFMAs): 128 x 128 with 4 waves is
# best in both modes, ResNet-50 chain bf16x3 1.55 ms (8 waves 1.99, round 1
# best 1.61), fp32 2.98 ms (16 waves 3.35); profiles/r2_pgemm_sweep.log
TILE_CFG_DEFAULT = {'bf16x3': 0, 'fp32': 0, 'bf16x6': 0}
# None: per-precision default; KFAC_PGEMM_TILE_CFG=<id> forces one (experiments, tests)
TILE_CFG = int(os.environ['KFAC_PGEMM_TILE_CFG']) if os.environ.get('KFAC_PGEMM_TILE_CFG') \
    else None


def _tile_class(M, N, precision):
    """1 = 256 x 256 tiles, else the 128 x 128 configuration.  The chain is
    latency bound (few k-steps in flight per CU): 128 x 128 tiles with more
    waves per tile win over bigger tiles; the big class stays available for
    experiments."""
    if precision == 'bf16x6':
        # the instantiated configurations: 0 (2 waves / SIMD), 8 (uncapped
        # registers), 9 (two LDS images); X6_BIG (1 = 256 x 256, 6 = 256 x 128,
        # 7 = 128 x 256, fp32-operand mode only) for problems with M, N >= 256
        if X6_BIG is not None and X6_MODE == 'fp32' and M >= 256 and N >= 256:
            return X6_BIG
        return TILE_CFG if TILE_CFG in (8, 9) else 0
    if precision in LP_CFG:
        # KFAC_LP_BIG=6 / 7: 256 x 128 / 128 x 256 tiles for problems with
        # M resp. N >= 256 (experiments; 128 x 128 otherwise)
        if LP_BIG == 6 and M >= 256:
            return 6
        if LP_BIG == 7 and N >= 256:
            return 7
        return 0
    if BIG_TILES and M >= 256 and N >= 256:
        return 1
    return TILE_CFG if TILE_CFG is not None else TILE_CFG_DEFAULT[precision]


class PGemmRec(ctypes.Structure):
    _fields_ = [('a_hi', ctypes.c_void_p), ('a_lo', ctypes.c_void_p), ('lda', ctypes.c_longlong),
                ('b_hi', ctypes.c_void_p), ('b_lo', ctypes.c_void_p), ('ldb', ctypes.c_longlong),
                ('c_hi', ctypes.c_void_p), ('c_lo', ctypes.c_void_p), ('ldc', ctypes.c_longlong),
                ('dmat', ctypes.c_void_p), ('ldd', ctypes.c_longlong),
                ('vm', ctypes.c_void_p), ('vn', ctypes.c_void_p), ('damping', ctypes.c_float),
                ('g_hi', ctypes.c_void_p), ('g_lo', ctypes.c_void_p), ('ldg', ctypes.c_longlong),
                ('M', ctypes.c_int), ('N', ctypes.c_int), ('K', ctypes.c_int), ('epi', ctypes.c_int),
                ('tile_begin', ctypes.c_int), ('tiles_n', ctypes.c_int),
                ('sc_in', ctypes.c_void_p), ('sc_out', ctypes.c_void_p),
                ('sc_zero', ctypes.c_void_p), ('ea', ctypes.c_int), ('eb', ctypes.c_int)]


class GatherRec(ctypes.Structure):
    _fields_ = [('w', ctypes.c_void_p), ('bias', ctypes.c_void_p),
                ('s0', ctypes.c_longlong), ('s1', ctypes.c_longlong), ('s2', ctypes.c_longlong),
                ('s3', ctypes.c_longlong),
                ('o_hi', ctypes.c_void_p), ('o_lo', ctypes.c_void_p), ('ldo', ctypes.c_longlong),
                ('nG', ctypes.c_int), ('nA', ctypes.c_int), ('kk', ctypes.c_int), ('kw', ctypes.c_int),
                ('wdtype', ctypes.c_int), ('bdtype', ctypes.c_int),
                ('tile_begin', ctypes.c_int), ('tiles_g', ctypes.c_int),
                ('amax', ctypes.c_void_p), ('zero3', ctypes.c_void_p)]


class SplitRec(ctypes.Structure):
    _fields_ = [('src', ctypes.c_void_p), ('lds', ctypes.c_longlong),
                ('o_hi', ctypes.c_void_p), ('o_lo', ctypes.c_void_p), ('ldo', ctypes.c_longlong),
                ('rows', ctypes.c_int), ('cols', ctypes.c_int), ('trans', ctypes.c_int),
                ('tile_begin', ctypes.c_int), ('tiles_c', ctypes.c_int)]


def _pad32(n):
    """k-padding of every MFMA operand: a multiple of the kernel's TK (64)."""
    return (n + 63) // 64 * 64


def _cdiv(a, b):
    return (a + b - 1) // b


_checked = False


def _check_layouts():
    global _checked
    if _checked:
        return
    L = _lib.lib()
    for rec, fn in ((PGemmRec, L.kfac_pgemm_record_size), (GatherRec, L.kfac_gather_record_size),
                    (SplitRec, L.kfac_split_record_size)):
        fn.restype = ctypes.c_int
        if ctypes.sizeof(rec) != fn():
            raise RuntimeError('{} layout mismatch: python {} vs native {}'.format(
                rec.__name__, ctypes.sizeof(rec), fn()))
    _checked = True


def _upload(recs, device):
    raw = bytes(memoryview(recs).cast('B'))
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)


class _Operand(object):
    """rows x ld operand, k-contiguous, zero-padded along k: fp32, or 16-bit
    planes (bf16 by default; `dtype` fp16 / bf16 for the low-plane modes, any
    plane count) in ONE allocation (the kernels find plane p at hi + p (lo - hi))."""
    __slots__ = ('t', 'hi', 'lo', 'ld', 'rows', 'scale')

    def __init__(self, rows, k, planes, device, dtype=None):
        self.rows, self.ld = rows, _pad32(k)
        self.scale = LP_QSCALE if dtype == torch.float16 else 1.0
        if planes > 1 or dtype is not None:
            self.t = torch.zeros(planes, rows, self.ld, dtype=dtype or torch.bfloat16,
                                 device=device)
            self.hi = self.t[0].data_ptr()
            self.lo = self.t[1].data_ptr() if planes > 1 else self.hi
        else:
            self.t = torch.zeros(rows, self.ld, dtype=torch.float32, device=device)
            self.hi = self.lo = self.t.data_ptr()

    def value(self):
        """fp32 view of the stored matrix (tests / debugging)."""
        if self.t.dim() == 3:
            return self.t.float().sum(0) / self.scale
        return self.t.clone()


class _LayerBufs(object):
    def __init__(self, layer, planes, device, inverse=False, q_planes=None, q_dtype=None):
        self.layer = layer
        nG, nA = layer.grad_shape
        self.nG, self.nA = nG, nA
        qp = planes if q_planes is None else q_planes     # eigenvector operands
        # persistent fp32 staging copies of eigendata that is not fp32-
        # contiguous (inv_dtype 16-bit, packed triangles): the split job table
        # then keys on fixed addresses (no table per temporary)
        self.stage = {}
        # inverse path (use_eigen_decomp=False): QGt holds G_inv and QA holds
        # A_inv (both symmetric), V = (G_inv Grad) A_inv in two stages
        self.QGt = _Operand(nG, nG, qp, device, q_dtype)
        self.QA = _Operand(nA, nA, qp, device, q_dtype)
        self.Gct = _Operand(nA, nG, planes, device)
        self.T1 = _Operand(nG, nA, planes, device)
        self.prediv = layer.prediv_eigenvalues and not inverse
        if inverse:
            self.QG = self.QAt = self.T2t = self.T3 = None
            self.Dt = None
            return
        self.QG = _Operand(nG, nG, qp, device, q_dtype)
        self.QAt = _Operand(nA, nA, qp, device, q_dtype)
        self.T2t = _Operand(nA, nG, planes, device)
        self.T3 = _Operand(nG, nA, planes, device)
        self.Dt = torch.zeros(nA, nG, dtype=torch.float32, device=device) if self.prediv else None

    def staged(self, key, t):
        """`t` as an fp32 contiguous matrix at a fixed address per key."""
        if t.dtype == torch.float32 and t.is_contiguous():
            return t
        buf = self.stage.get(key)
        if buf is None or buf.shape != t.shape:
            buf = self.stage[key] = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        buf.copy_(t)
        return buf


class FusedPreconditioner(object):
    def __init__(self, layers, precision='bf16x3'):
        if precision not in PRECISIONS and precision not in LP_CFG:
            raise ValueError('precision must be one of {}'.format(sorted(PRECISIONS)))
        _check_layouts()
        self.layers = list(layers)
        self.precision = precision
        self.prec = PRECISIONS.get(precision, 0)
        self.x3 = precision == 'bf16x3'
        self.planes = PLANES.get(precision, 1)
        # precision of the stored operands: the gathered gradient (gather
        # launch) and the eigenvector operands (split launch)
        self.store_prec = self.q_store_prec = self.prec
        q_planes = None
        # kernel precision per stage: S1-S3 multiply an eigenvector operand
        # as A, S4 (and the inverse path's second stage) as B
        self.stage_prec = None
        self.lp = LP_CFG.get(precision)
        q_dtype = None
        if self.lp is not None:
            pa, pb, qstore, q_planes, q_dtype, _ = self.lp
            self.prec, self.store_prec, self.planes, self.q_store_prec = pa, 0, 1, qstore
            self.stage_prec = (pa, pa, pa, pb)
        elif precision == 'bf16x6' and X6_MODE != 'planes':
            self.prec, self.store_prec, self.planes = PREC_BF16X6F, 0, 1
            self.q_store_prec = 0
            if X6_MODE == 'mixed':
                q_planes = PLANES['bf16x6']
                self.q_store_prec = PRECISIONS['bf16x6']
                self.stage_prec = (PREC_BF16X6A, PREC_BF16X6A, PREC_BF16X6A, PREC_BF16X6B)
        self.device = self.layers[0].module.weight.device if self.layers else None
        # the damped-inverse path (K9): V = G_inv Grad A_inv, two grouped stages
        self.inverse = bool(self.layers) and not self.layers[0].use_eigen_decomp
        if self.inverse and self.stage_prec is not None:
            self.stage_prec = (self.stage_prec[0], self.stage_prec[3])
        self.bufs = [_LayerBufs(l, self.planes, self.device, self.inverse, q_planes, q_dtype)
                     for l in self.layers]
        # low-plane fp16 modes: per layer the max |x| bits of Gct, T1, T2t, T3
        # (filled by their producers, read by their consumers; see run())
        self.slots = None
        if self.lp is not None and self.lp[5] and self.layers:
            self.slots = torch.zeros(len(self.bufs), 4, dtype=torch.int32, device=self.device)
        for b in self.bufs:
            _lib.check_pgemm_extent(max(b.nG, b.nA), 'layer')
        self._gather_sig = None
        self._stage_tables = None
        # superseded device tables stay alive: a captured graph may use them
        self._retired_tables = []
        self._split_tables = {}       # refresh_eigen job tables by content
        self.damping = 0.0
        self.kl_buf = None
        self._build_stage_tables()

    # ------------------------------------------------------------- tables
    def _build_stage_tables(self):
        if self._stage_tables is not None:
            self._retired_tables.append(self._stage_tables)
        stages = []
        for stage in ((0, 3) if self.inverse else range(4)):
            probs = []
            for b in self.bufs:
                st = b.layer.state
                r = PGemmRec()
                r.epi = EPI_STORE
                if stage == 3 and self.inverse:     # V[g][a] = T1 . A_inv (+ KL dot)
                    A, B, C, M, N, K = b.T1, b.QA, None, b.nG, b.nA, b.nA
                    r.epi = EPI_FINAL
                elif stage == 0:    # T1[g][a] = QGt . Gct  (inverse path: G_inv . Gct)
                    A, B, C, M, N, K = b.QGt, b.Gct, b.T1, b.nG, b.nA, b.nG
                elif stage == 1:    # T2t[a][g] = (QAt . T1) (.) Dt
                    A, B, C, M, N, K = b.QAt, b.T1, b.T2t, b.nA, b.nG, b.nA
                    if b.prediv:
                        r.epi, r.dmat, r.ldd = EPI_HADAMARD, b.Dt.data_ptr(), b.nG
                    else:
                        r.epi = EPI_HADAMARD_VEC
                        # fp32 eigenvalues (16-bit inv_dtype: fixed-address copies,
                        # refreshed by refresh_eigen)
                        r.vm = b.staged('dA', st['dA']).data_ptr()
                        r.vn = b.staged('dG', st['dG']).data_ptr()
                        r.damping = self.damping
                elif stage == 2:    # T3[g][a] = QG . T2t
                    A, B, C, M, N, K = b.QG, b.T2t, b.T3, b.nG, b.nA, b.nG
                else:               # V[g][a] = T3 . QA  (+ KL dot)
                    A, B, C, M, N, K = b.T3, b.QA, None, b.nG, b.nA, b.nA
                    r.epi = EPI_FINAL
                r.a_hi, r.a_lo, r.lda = A.hi, A.lo, A.ld
                r.b_hi, r.b_lo, r.ldb = B.hi, B.lo, B.ld
                if C is None:
                    v = b.layer._pgrad_matrix()
                    r.c_hi = r.c_lo = v.data_ptr()
                    r.ldc = v.stride(0)
                    r.g_hi, r.g_lo, r.ldg = b.Gct.hi, b.Gct.lo, b.Gct.ld
                else:
                    r.c_hi, r.c_lo, r.ldc = C.hi, C.lo, C.ld
                r.M, r.N, r.K = M, N, K
                if self.slots is not None:
                    # slot chain: gather -> Gct (0) -> S1 -> T1 (1) -> S2 -> T2t
                    # (2) -> S3 -> T3 (3) -> S4, which frees slot 0 for the next
                    # step (the gather zeroes 1..3); inverse path: Gct (0) -> T1 (1)
                    bi = self.bufs.index(b)
                    base = self.slots.data_ptr() + 16 * bi
                    src = {0: 0, 1: 1, 2: 2, 3: 1 if self.inverse else 3}[stage]
                    r.sc_in = base + 4 * src
                    if C is not None:
                        r.sc_out = base + 4 * (stage + 1)
                    else:
                        r.sc_zero = base
                probs.append(r)
            launches = []
            classes = sorted({_tile_class(r.M, r.N, self.precision) for r in probs})
            for tile in classes:
                bm, bn = TILE_SHAPES[tile]
                sel = [r for r in probs if _tile_class(r.M, r.N, self.precision) == tile]
                if not sel:
                    continue
                # longest k-loops first: their tiles are dispatched first
                sel.sort(key=lambda r: -r.K)
                tiles = 0
                for r in sel:
                    r.tiles_n = _cdiv(r.N, bn)
                    r.tile_begin = tiles
                    tiles += _cdiv(r.M, bm) * r.tiles_n
                arr = (PGemmRec * len(sel))(*sel)
                launches.append((tile, _upload(arr, self.device), len(sel), tiles))
            stages.append(launches)
        self._stage_tables = stages
        # KL dot of the last stage: one f64 partial slot per workgroup of its
        # launches (the count depends on the tile shapes), summed in a fixed
        # order (deterministic: every rank derives the same clip scale); the
        # result is slot 0.  A grown buffer retires the old one (graphs).
        self._kl_slots = sum(tiles for _, _, _, tiles in stages[-1])
        if self.kl_buf is None or self.kl_buf.numel() < 1 + self._kl_slots:
            if self.kl_buf is not None:
                self._retired_tables.append(self.kl_buf)
            self.kl_buf = torch.zeros(1 + self._kl_slots, dtype=torch.float64, device=self.device)
            self.kl = self.kl_buf[0]

    def refresh_eigen(self):
        """Re-split QA/QG (+ transposes) and transpose dGdA after an inverse
        update (or an eigendata broadcast).  Two launches for all layers."""
        jobs, fjobs = [], []

        def add(lst, src, dst, trans):
            r = SplitRec()
            r.src, r.lds = src.data_ptr(), src.stride(0)
            r.o_hi, r.o_lo, r.ldo = dst.hi, dst.lo, dst.ld
            r.rows, r.cols, r.trans = src.shape[0], src.shape[1], int(trans)
            lst.append(r)

        class _F32Dst(object):
            def __init__(self, t):
                self.hi = self.lo = t.data_ptr()
                self.ld = t.stride(0)

        keep = []
        for b in self.bufs:
            st = b.layer.state
            if self.inverse:
                Ai, Gi = st['A_inv'], st['G_inv']
                if Ai.dim() == 1:       # symmetry-aware comm keeps packed triangles
                    from ..layers import utils as lutils
                    Ai = lutils.fill_triu((b.nA, b.nA), Ai)
                    Gi = lutils.fill_triu((b.nG, b.nG), Gi)
                Ai, Gi = b.staged('A', Ai), b.staged('G', Gi)
                add(jobs, Gi, b.QGt, False)
                add(jobs, Ai, b.QA, False)
                continue
            QA = b.staged('A', st['QA'])
            QG = b.staged('G', st['QG'])
            add(jobs, QG, b.QG, False)
            add(jobs, QG, b.QGt, True)
            add(jobs, QA, b.QA, False)
            add(jobs, QA, b.QAt, True)
            if not b.prediv:
                b.staged('dA', st['dA'])
                b.staged('dG', st['dG'])
            if b.prediv:
                D = b.staged('D', st['dGdA'])
                add(fjobs, D, _F32Dst(b.Dt), True)
        stream = _lib.stream(self.device)
        L = _lib.lib()
        for lst, prec in ((jobs, self.q_store_prec), (fjobs, 0)):
            if not lst:
                continue
            tiles = 0
            for r in lst:
                rr, cc = (r.rows, r.cols)
                r.tiles_c = _cdiv(cc, 64)
                r.tile_begin = tiles
                tiles += _cdiv(rr, 64) * r.tiles_c
            # the job tables only change when a buffer moves: uploaded once
            # per content (a host-to-device copy inside the inverse step would
            # wait behind the eigensolver's queued work on some runtimes)
            raw = bytes(memoryview((SplitRec * len(lst))(*lst)).cast('B'))
            table = self._split_tables.get(raw)
            if table is None:
                if len(self._split_tables) >= 8:
                    # split copies run only in eager inverse steps, never in a
                    # captured graph, and every table was record_stream'ed at
                    # its launch: dropping them is stream-safe (no retired list
                    # growing over a long run: ADVICE r5)
                    self._split_tables.clear()
                table = self._split_tables[raw] = _upload((SplitRec * len(lst))(*lst),
                                                          self.device)
            _lib.check(L.kfac_split_copy(prec, _lib.ptr(table), len(lst), tiles, stream),
                       'kfac_split_copy')
            keep.append(table)
        cur = torch.cuda.current_stream(self.device)
        for t in keep:
            t.record_stream(cur)

    def _gather_table(self):
        """Host-side job table for the .grad gather, rebuilt only when a .grad
        tensor moved; launched BY VALUE (no device table to go stale between
        graph-captured and eager launches)."""
        sig = []
        for b in self.bufs:
            g = b.layer._get_weight_grad()
            if g is None:
                raise RuntimeError('{} has no gradient; K-FAC needs every registered layer to '
                                   'take part in backward'.format(b.layer))
            bias = b.layer._get_bias_grad() if b.layer.has_bias else None
            sig.append((g.data_ptr(), tuple(g.stride()), g.dtype,
                        None if bias is None else (bias.data_ptr(), bias.dtype)))
        sig = tuple(sig)
        if sig == self._gather_sig:
            return self._gather
        recs = (GatherRec * len(self.bufs))()
        for r, b in zip(recs, self.bufs):
            g = b.layer._get_weight_grad()
            r.w = g.data_ptr()
            st = g.stride()
            if g.dim() == 4:
                r.s0, r.s1, r.s2, r.s3 = st
                r.kk, r.kw = g.shape[2] * g.shape[3], g.shape[3]
            elif g.dim() == 2:
                r.s0, r.s1, r.s2, r.s3 = st[0], st[1], 0, 0
                r.kk, r.kw = 1, 1
            else:
                raise ValueError('unsupported weight gradient rank {}'.format(g.dim()))
            r.wdtype = _lib.DTYPE_CODE[g.dtype]
            if b.layer.has_bias:
                bias = b.layer._get_bias_grad()
                r.bias, r.bdtype = bias.data_ptr(), _lib.DTYPE_CODE[bias.dtype]
            r.o_hi, r.o_lo, r.ldo = b.Gct.hi, b.Gct.lo, b.Gct.ld
            r.nG, r.nA = b.nG, b.nA
            if self.slots is not None:
                base = self.slots.data_ptr() + 16 * self.bufs.index(b)
                r.amax, r.zero3 = base, base + 4
        self._gather = recs
        self._gather_sig = sig
        return recs

    # ---------------------------------------------------------------- run
    def run(self, damping=0.0, with_kl=True):
        """Precondition every layer; returns the device f64 <v, g> sum (or None).

        `damping` matters only without prediv (with prediv the inverse-time
        damping is baked into dGdA, as in the reference, base.py:305-306)."""
        if not self.bufs:
            return None
        if any(not b.prediv for b in self.bufs) and float(damping) != self.damping:
            self.damping = float(damping)
            self._build_stage_tables()
        L = _lib.lib()
        stream = _lib.stream(self.device)
        recs = self._gather_table()
        _lib.check(L.kfac_gather_grad(self.store_prec, recs, len(recs), stream),
                   'kfac_gather_grad')
        final = len(self._stage_tables) - 1
        for i, launches in enumerate(self._stage_tables):
            slot = 1
            prec = self.prec if self.stage_prec is None else self.stage_prec[i]
            for tile, table, count, tiles in launches:
                kl = _lib.c_vp(self.kl_buf.data_ptr() + 8 * slot) if (with_kl and i == final) \
                    else None
                _lib.check(L.kfac_pgemm(prec, tile, _lib.ptr(table), count, tiles, kl,
                                        stream), 'kfac_pgemm')
                slot += tiles
        if with_kl:
            _lib.check(L.kfac_kl_finalize(_lib.c_vp(self.kl_buf.data_ptr() + 8), self._kl_slots,
                                          _lib.ptr(self.kl_buf), stream), 'kfac_kl_finalize')
        for b in self.bufs:
            b.layer.preconditioned_gradient = b.layer._split_pgrad(b.layer._pgrad_matrix())
        return self.kl if with_kl else None


class SplitFused(object):
    """The fused chain over a forward-order layer split, for single-rank runs
    (KFAC(overlap_precondition=True)): `top` holds the LAST layers -- the ones
    whose gradients backward produces first, and most of the chain's flops
    (ResNet-50's layer4) -- and is launched on a side stream from a gradient
    hook as soon as its gradients are accumulated, so it runs under the rest
    of the backward; run() then preconditions `bottom` on the current stream,
    joins, and adds the two KL partial dots (bottom + top, fixed order).  Same
    operands, same kernels, same math as one FusedPreconditioner."""

    def __init__(self, layers, precision, split_at):
        self.layers = list(layers)
        self.bottom = FusedPreconditioner(self.layers[:split_at], precision)
        self.top = FusedPreconditioner(self.layers[split_at:], precision)
        self.inverse = self.top.inverse
        self.device = self.top.device
        self.precision = precision
        self._side = None
        self._top_kl = None
        self._launched = None      # tag of the pending early launch, or None
        self.early_launches = 0
        self.kl_sum = torch.zeros((), dtype=torch.float64, device=self.device)

    @property
    def bufs(self):
        return self.bottom.bufs + self.top.bufs

    @property
    def kl(self):
        return self.kl_sum

    @property
    def _stage_tables(self):
        return self.top._stage_tables

    def refresh_eigen(self):
        self._join_side()
        self._launched = None      # an early result from the old eigenbasis is stale
        self.bottom.refresh_eigen()
        self.top.refresh_eigen()

    def _join_side(self):
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def launch_top(self, damping=0.0, with_kl=True, tag=None):
        """Precondition the top layers on the side stream (called from the
        hook that sees the last top-layer gradient accumulated).  `tag`
        identifies the step / eigenbasis the launch belongs to: run() reuses
        the result only under the same tag."""
        cur = torch.cuda.current_stream(self.device)
        side = self._side_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self._top_kl = self.top.run(damping=damping, with_kl=with_kl)
        self._launched = (tag, float(damping), bool(with_kl))
        self.early_launches += 1

    def run(self, damping=0.0, with_kl=True, tag=None):
        cur = torch.cuda.current_stream(self.device)
        early = self._launched
        self._launched = None
        reuse = early is not None and early == (tag, float(damping), bool(with_kl))
        if early is not None and not reuse:
            # a launch from another step (a backward without KFAC.step()) or
            # another eigenbasis: drain it, then precondition afresh
            cur.wait_stream(self._side)
        if not reuse:
            self._top_kl = self.top.run(damping=damping, with_kl=with_kl)
        klb = self.bottom.run(damping=damping, with_kl=with_kl)
        if reuse:
            cur.wait_stream(self._side)
        if not with_kl:
            return None
        torch.add(klb, self._top_kl, out=self.kl_sum)
        return self.kl_sum
