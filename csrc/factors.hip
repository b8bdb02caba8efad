// Kronecker-factor kernels for gfx950.
//
//   syrk_patch   K1+K2+K3/K4: C += scale * P^T P where P is the *implicit*
//                im2col patch matrix of a Conv2d input (rows (b,oh,ow),
//                columns (c,kh,kw) [+ a ones column for the bias]).  Linear
//                inputs and conv grad_outputs are the degenerate 1x1 case.
//                The patch matrix is never materialised: each workgroup
//                gathers a [BK rows x 128 cols] slab straight from the NCHW /
//                NHWC activation into LDS (k-contiguous) and feeds MFMA
//                (32x32x16 bf16/f16, or 32x32x2 f32 for fp32 data).  Only
//                upper-triangular 128x128 output tiles are computed (SYRK);
//                the row dimension (up to 4e5 rows) is split over
//                blockIdx.y; every (split, tile) stores its partial tile and
//                tile_reduce adds the partials in a fixed order (source,
//                split) into the workspace: bitwise-reproducible factors
//                (the f32-atomic form remains for part == nullptr).
//   factor_ema   K5: state = alpha*state + (1-alpha)*sym(ws), mirrored from
//                the upper triangle, in the factor's storage dtype.
//   triu pack/unpack K12: symmetric factors <-> packed upper triangles for
//                the bucketed RCCL all-reduce; unpack folds the 1/world
//                averaging in.
//
// Reference semantics: kfac/layers/conv.py:24-70, kfac/layers/linear.py:12-24,
// kfac/layers/utils.py:4-43,164-178 (A_conv = P^T P / (B * S^3), G_conv =
// g^T g / (B * S^3), linear: a^T a / rows).
#include "common.h"

#include <cstdlib>
#include "devtable.h"
#include <algorithm>
#include <vector>
#include <type_traits>

namespace {

struct PatchArgs {
  const void* x;          // activation base pointer
  long long sb, sc, sh, sw;  // element strides of x for (b, c, h, w)
  int B, C, H, W;
  int kh, kw, sth, stw, ph, pw, dh, dw;
  int OH, OW;
  int kcols;              // C*kh*kw
  int ncols;              // kcols + has_bias
  long long M;            // B*OH*OW rows
  long long rows_per_split;
  int ntiles;             // ceil(ncols / 128)
  float scale;
  float* ws;              // f32 workspace, row-major, leading dim ldw
  int ldw;
  float* part;            // nullptr: f32 atomics into ws; else [split][tile][BT*BT] partials
  const float* dscale;    // nullptr, or a device factor on `scale` (AMP: finite(g) / s^2;
                          // 0 drops the source without letting its NaN / Inf through)
};

constexpr int BT = 128;   // output tile
constexpr int BK = 32;    // rows per k-step

template <int DT> struct SyrkCfg;
template <> struct SyrkCfg<KDT_F32> { static constexpr int LDK = BK + 1; };   // 33 floats: conflict-free b32 reads
template <> struct SyrkCfg<KDT_BF16> { static constexpr int LDK = BK + 8; };  // 80 B rows: conflict-free b128 reads
template <> struct SyrkCfg<KDT_F16> { static constexpr int LDK = BK + 8; };

// Per-thread column descriptor for the gather: element offset of the column
// inside one patch, and its (kh, kw) displacement packed as (di << 16) | dj.
// Special values of `disp`: -1 = padding column (zero), -2 = bias column (one).
struct ColInfo { int off; int disp; };

__device__ __forceinline__ ColInfo make_col(const PatchArgs& p, int gcol) {
  ColInfo ci;
  if (gcol < p.kcols) {
    int kk = p.kh * p.kw;
    int c = gcol / kk;
    int r = gcol - c * kk;
    int i = r / p.kw;
    int j = r - i * p.kw;
    int di = i * p.dh, dj = j * p.dw;
    ci.off = (int)(c * p.sc + (long long)di * p.sh + (long long)dj * p.sw);
    ci.disp = (di << 16) | dj;
  } else if (gcol < p.ncols) {
    ci.off = 0; ci.disp = -2;
  } else {
    ci.off = 0; ci.disp = -1;
  }
  return ci;
}

template <int DT>
__device__ __forceinline__ typename DTypeTraits<DT>::raw_t gather(
    const PatchArgs& p, const typename DTypeTraits<DT>::raw_t* x, long long base,
    int hb, int wb, bool row_ok, ColInfo ci) {
  typedef typename DTypeTraits<DT>::raw_t raw_t;
  if (!row_ok || ci.disp == -1) return (raw_t)0;
  if (ci.disp == -2) return DTypeTraits<DT>::from_f32(1.0f);
  int h = hb + (ci.disp >> 16);
  int w = wb + (ci.disp & 0xffff);
  if ((unsigned)h >= (unsigned)p.H || (unsigned)w >= (unsigned)p.W) return (raw_t)0;
  return x[base + ci.off];
}

__device__ __forceinline__ void decompose_row(const PatchArgs& p, long long row,
                                              long long& base, int& hb, int& wb) {
  long long ohw = (long long)p.OH * p.OW;
  long long b = row / ohw;
  int rem = (int)(row - b * ohw);
  int oh = rem / p.OW;
  int ow = rem - oh * p.OW;
  hb = oh * p.sth - p.ph;
  wb = ow * p.stw - p.pw;
  base = b * p.sb + (long long)hb * p.sh + (long long)wb * p.sw;
}

// Epilogue of a (tile, split) work item: the scaled 128x128 partial tile
// stored whole into its slot of p.part (plain stores: tile_reduce adds the
// splits in a fixed order), or, with no partial buffer, f32 atomics into the
// upper triangle of ws.
// TW = tile width (128, or 256 for the wide grouped tiles); a wave owns MI x
// NJ 32x32 blocks at rows wr * 32 MI, columns wc * 32 NJ of the tile.
template <int TW = BT, int MI = 2, int NJ = 2>
__device__ __forceinline__ void store_tile(const PatchArgs& p, const f32x16_t (&acc)[MI][NJ],
                                           int tile, int split, int ti, int tj, bool diag, int wr,
                                           int wc, int lr, int lh) {
  const float ds = p.dscale != nullptr ? *p.dscale : 1.f;
  const float sc = p.scale * ds;
  const bool drop = (ds == 0.f);
  if (p.part != nullptr) {
    const int tp = p.ntiles * (p.ntiles + 1) / 2;
    float* dst = p.part + ((long long)split * tp + tile) * (TW * TW);
#pragma unroll
    for (int m = 0; m < MI; ++m)
#pragma unroll
      for (int n = 0; n < NJ; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lrow = wr * 32 * MI + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const int lcol = wc * 32 * NJ + n * 32 + lr;
          dst[lrow * TW + lcol] = drop ? 0.f : sc * acc[m][n][r];
        }
    return;
  }
#pragma unroll
  for (int m = 0; m < MI; ++m)
#pragma unroll
    for (int n = 0; n < NJ; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = ti * TW + wr * 32 * MI + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        int col = tj * TW + wc * 32 * NJ + n * 32 + lr;
        if (!drop && row < p.ncols && col < p.ncols && (!diag || row <= col))
          atomicAdd(p.ws + (long long)row * p.ldw + col, sc * acc[m][n][r]);
      }
}

// ws[row][col] (upper triangle, row <= col < ncols) = sum over the job's
// contributions c (in order) and their splits s (in order) of
// part_c[s][tile][local]: one workgroup per (job, tile pair).  accum = 1 adds
// the sum to ws instead (a factor with more than MAX_CONTRIB sources, e.g. an
// LSTM's per-time-step Linears, is reduced in fixed-order chained launches of
// MAX_CONTRIB contributions: still bitwise reproducible).
constexpr int MAX_CONTRIB = 8;
struct RedJob {
  float* ws; int ldw, ncols, ntiles, ncontrib;
  const float* part[MAX_CONTRIB];
  int splits[MAX_CONTRIB];
  int block_begin, accum;
  int bt;                 // tile width of the partials (128 or 256)
  int mirror;             // 1: also store the strict lower triangle (the grouped EMA
                          // then reads whole rows, no column walks)
};
constexpr int MAX_RED_JOBS = 24;
struct RedBatch {
  int count, pad[3];
  RedJob job[MAX_RED_JOBS];
};
static_assert(sizeof(RedBatch) <= 4096, "kernel arguments are limited to 4 KB");

// Each workgroup takes a 32 x 32 block (a float4 of one row per thread) of
// one tile pair: RED_WG = 16 workgroups per 128-wide tile pair (64 per
// 256-wide one).  The split loop loads 8 partials at a time (independent, in
// flight together) and adds them in order: the summation order
// (contribution, split) is fixed, so the result is deterministic.
constexpr int RED_WG = (BT * BT) / 1024;

__global__ __launch_bounds__(256) void tile_reduce_kernel(const RedBatch* __restrict__ batch) {
  const RedJob* t = batch->job;
  int lo = 0, hi = batch->count - 1;
  const int b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].block_begin <= b) lo = mid; else hi = mid - 1;
  }
  const RedJob& J = t[lo];
  const int bt = J.bt, bt2 = bt * bt, rwg = bt2 / 1024, nbc = bt / 32;
  const int loc = b - J.block_begin;
  const int tile = loc / rwg, part = loc - tile * rwg;
  int tt = tile, ti = 0, rem = J.ntiles;
  while (tt >= rem) { tt -= rem; ++ti; --rem; }
  const int tj = ti + tt;
  const int tp = J.ntiles * (J.ntiles + 1) / 2;
  const int br = part / nbc, bc = part - br * nbc;        // 32 x 32 block of the tile
  const int lr = threadIdx.x >> 3, c4 = (threadIdx.x & 7) * 4;
  const int e = (br * 32 + lr) * bt + bc * 32 + c4;       // 4 consecutive elements of a row
  const long long sstride = (long long)tp * bt2 / 4;    // float4 stride between splits
  fx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < J.ncontrib; ++c) {
    const AS1 fx4* pc = (const AS1 fx4*)(gptr(J.part[c]) + (long long)tile * bt2 + e);
    const int ns = J.splits[c];
    int sp = 0;
    for (; sp + 8 <= ns; sp += 8) {
      fx4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pc[(long long)(sp + u) * sstride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; sp < ns; ++sp) acc += pc[(long long)sp * sstride];
  }
  const int row = ti * bt + br * 32 + lr, col0 = tj * bt + bc * 32 + c4;
  AS1 float* w = gptr(J.ws) + (long long)row * J.ldw + col0;
  const bool add = J.accum != 0;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (row <= col0 + u && col0 + u < J.ncols) w[u] = add ? w[u] + acc[u] : acc[u];
  if (!J.mirror) return;
  // mirror: ws[col][row] = ws[row][col] for row < col (the same values as
  // the upper store: the lower triangle is bitwise its mirror), through an
  // LDS transpose of the block; consecutive lanes store consecutive
  // elements of a mirrored row (128-byte runs)
  __shared__ float tr[32][33];
#pragma unroll
  for (int u = 0; u < 4; ++u) tr[lr][c4 + u] = acc[u];
  __syncthreads();
  const int r0 = ti * bt + br * 32, q0 = tj * bt + bc * 32;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = k * 256 + threadIdx.x;
    const int mr = idx >> 5, mc = idx & 31;               // mirrored row / column in the block
    const int grow = q0 + mr, gcol = r0 + mc;
    if (gcol < grow && grow < J.ncols) {
      AS1 float* m = gptr(J.ws) + (long long)grow * J.ldw + gcol;
      const float v = tr[mc][mr];
      *m = add ? *m + v : v;
    }
  }
}

// LANE_COLS = true when channels are the unit-stride dim (NHWC / Linear):
// consecutive lanes then gather consecutive columns (coalesced); otherwise
// (NCHW) consecutive lanes gather consecutive rows (= consecutive ow).
template <int DT, bool LANE_COLS>
__global__ __launch_bounds__(256) void syrk_patch_kernel(PatchArgs p) {
  typedef typename DTypeTraits<DT>::raw_t raw_t;
  constexpr int LDK = SyrkCfg<DT>::LDK;
  __shared__ __attribute__((aligned(16))) raw_t smem[2 * BT * LDK];
  raw_t* sA = smem;
  raw_t* sB = smem + BT * LDK;

  // upper-triangular tile decode: blockIdx.x -> (ti <= tj)
  int t = blockIdx.x, ti = 0, rem = p.ntiles;
  while (t >= rem) { t -= rem; ++ti; --rem; }
  const int tj = ti + t;
  const bool diag = (ti == tj);

  const long long r_begin = (long long)blockIdx.y * p.rows_per_split;
  long long r_end = r_begin + p.rows_per_split;
  if (r_end > p.M) r_end = p.M;
  if (r_begin >= r_end) return;
  const int nk = (int)((r_end - r_begin + BK - 1) / BK);

  const raw_t* x = (const raw_t*)p.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;

  // ---- loader geometry ----
  // LANE_COLS : col = tid & 127, rows rg*16 .. rg*16+15, rg = tid >> 7
  // !LANE_COLS: row = tid & 31,  cols cg*16 .. cg*16+15, cg = tid >> 5
  constexpr int NPER = 16;
  ColInfo ca[LANE_COLS ? 1 : NPER], cb[LANE_COLS ? 1 : NPER];
  if (LANE_COLS) {
    int col = tid & 127;
    ca[0] = make_col(p, ti * BT + col);
    cb[0] = make_col(p, tj * BT + col);
  } else {
    int cg = tid >> 5;
#pragma unroll
    for (int q = 0; q < NPER; ++q) {
      ca[q] = make_col(p, ti * BT + cg * 16 + q);
      cb[q] = make_col(p, tj * BT + cg * 16 + q);
    }
  }
  raw_t va[NPER], vb[NPER];

  auto load_step = [&](int k) {
    long long r0 = r_begin + (long long)k * BK;
    if (LANE_COLS) {
      int rg = tid >> 7;
      long long row = r0 + rg * 16;
      // decompose the first row once, then walk the next 15 incrementally
      long long rs = row < r_end ? row : r_begin;
      long long ohw = (long long)p.OH * p.OW;
      long long b = rs / ohw;
      int rr = (int)(rs - b * ohw);
      int oh = rr / p.OW, ow = rr - oh * p.OW;
#pragma unroll
      for (int q = 0; q < NPER; ++q) {
        bool ok = (row + q) < r_end;
        int hb = oh * p.sth - p.ph;
        int wb = ow * p.stw - p.pw;
        long long base = b * p.sb + (long long)hb * p.sh + (long long)wb * p.sw;
        va[q] = gather<DT>(p, x, base, hb, wb, ok, ca[0]);
        if (!diag) vb[q] = gather<DT>(p, x, base, hb, wb, ok, cb[0]);
        if (++ow == p.OW) { ow = 0; if (++oh == p.OH) { oh = 0; ++b; } }
      }
    } else {
      long long row = r0 + (tid & 31);
      bool ok = row < r_end;
      long long base = 0; int hb = 0, wb = 0;
      if (ok) decompose_row(p, row, base, hb, wb);
#pragma unroll
      for (int q = 0; q < NPER; ++q) {
        va[q] = gather<DT>(p, x, base, hb, wb, ok, ca[q]);
        if (!diag) vb[q] = gather<DT>(p, x, base, hb, wb, ok, cb[q]);
      }
    }
  };

  auto store_step = [&]() {
    if (LANE_COLS) {
      int col = tid & 127, rg = tid >> 7;
      raw_t* da = sA + col * LDK + rg * 16;
      raw_t* db = sB + col * LDK + rg * 16;
#pragma unroll
      for (int q = 0; q < NPER; ++q) { da[q] = va[q]; if (!diag) db[q] = vb[q]; }
    } else {
      int r = tid & 31, cg = tid >> 5;
#pragma unroll
      for (int q = 0; q < NPER; ++q) {
        sA[(cg * 16 + q) * LDK + r] = va[q];
        if (!diag) sB[(cg * 16 + q) * LDK + r] = vb[q];
      }
    }
  };

  // ---- MFMA geometry: 4 waves as 2x2, each a 64x64 sub-tile = 2x2 MFMA 32x32 tiles
  const int wr = wave >> 1, wc = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;
  f32x16_t acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  const raw_t* sBr = diag ? sA : sB;

  load_step(0);
  for (int k = 0; k < nk; ++k) {
    store_step();
    __syncthreads();
    if (k + 1 < nk) load_step(k + 1);   // global gathers in flight under the MFMAs
    if constexpr (DT == KDT_F32) {
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
        float a[2], b[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) a[m] = sA[(wr * 64 + m * 32 + lr) * LDK + ks * 2 + lh];
#pragma unroll
        for (int n = 0; n < 2; ++n) b[n] = sBr[(wc * 64 + n * 32 + lr) * LDK + ks * 2 + lh];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m], b[n], acc[m][n], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        typedef typename std::conditional<DT == KDT_BF16, bf16x8_t, f16x8_t>::type frag_t;
        frag_t a[2], b[2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
          a[m] = *(const frag_t*)(sA + (wr * 64 + m * 32 + lr) * LDK + ks * 16 + lh * 8);
#pragma unroll
        for (int n = 0; n < 2; ++n)
          b[n] = *(const frag_t*)(sBr + (wc * 64 + n * 32 + lr) * LDK + ks * 16 + lh * 8);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            if constexpr (DT == KDT_BF16)
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
            else
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m], b[n], acc[m][n], 0, 0, 0);
          }
      }
    }
    __syncthreads();
  }

  store_tile(p, acc, blockIdx.x, blockIdx.y, ti, tj, diag, wr, wc, lr, lh);
}

// ---------------------------------------------------------------------------
// syrk_vec: the channels-contiguous (NHWC / Linear) fast path of syrk_patch.
// Columns are processed in the *internal* order (i, j, c) -- channel fastest,
// which is the memory order of a channels_last activation -- so 8 consecutive
// columns of one patch row are ONE 16-byte load.  Each thread gathers an 8x8
// (rows x columns) block with 8 such loads, transposes it in registers and
// stores 8 k-contiguous 16-byte rows into the [column][k] LDS image that the
// MFMA fragments read with ds_read_b128.  The factor EMA kernel maps the
// internal order back to the reference order (c, i, j) (factor_ema perm).
// Requirements (checked on the host): 16-bit dtype, channel stride 1,
// C % 8 == 0, every other stride % 8 == 0, 16-byte aligned base.
constexpr int VBK = 64;                 // patch rows per k-step (default configuration)
// LDS of one syrk_vec workgroup: two [BT][VB + 8] operand images and the
// double-buffered row table (VB 16-byte entries per slot)
template <int VB, int TW = BT> struct SyrkVecLds {
  static_assert(VB == 64, "the row decode is one wave: VB rows per k-step");
  static constexpr int ELEMS = 2 * TW * (VB + 8) + 2 * VB * 8;
};
// 16-byte gather constants: zeros, and the ones column's first chunk [1, 0 x 7]
// as bf16 and as f16
__device__ __attribute__((aligned(16))) const uint16_t g_syrk_const[3][8] = {
    {0, 0, 0, 0, 0, 0, 0, 0}, {0x3f80, 0, 0, 0, 0, 0, 0, 0}, {0x3c00, 0, 0, 0, 0, 0, 0, 0}};

__device__ __forceinline__ uint32_t pack_lo(uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); }
__device__ __forceinline__ uint32_t pack_hi(uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); }
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));   // native vector: selects stay in VGPRs
__device__ __forceinline__ uint32_t u4get(const u32x4_t& v, int i) { return v[i]; }

// One (upper-triangular tile pair, row split) work item of syrk_vec.
// VB: patch rows per k-step (LDS rows of VB + 8 elements keep the b128
// fragment reads conflict-free); the next k-step's loads are in flight under
// this one's MFMAs.  Measured on ResNet-50's factor step (SPLIT_ROWS 2048,
// profiles/r3_factors_cfg*.log): 64 rows 4.11 ms; 128 rows 4.95 ms (two
// workgroups per CU instead of three); two k-steps of loads in flight 7.9-8.0
// ms (a second register set halves occupancy) -- 64 rows, one ahead, stays.
// The gather goes through global-address-space loads: with flat loads the
// MFMA step's LDS waits (lgkmcnt) also waited for the next k-step's gather,
// so nothing overlapped; 4.11 -> 3.66 ms (profiles/r3_factors_global_loads.log).
// The per-row decode moved into an LDS row table (below): 3.66 -> 3.34 ms
// (profiles/r3_factors_rowtable.log); what remains is mostly waiting on the
// one-k-step-ahead gather (SQ_WAIT_ANY 53 % of wave cycles, no LDS conflicts).
// An LDS-DMA version (global_load_lds into a ring of [64][128] images read
// with ds_read_b64_tr_b16, no staging registers) measured 3.46 ms with two
// stages (2 workgroups / CU) and 4.70 ms with three (1 / CU; hipcc still waits
// vmcnt(0) before some ring reads): not kept (profiles/r3_factors_dma*.log).
// TW: output tile width.  128 (4 waves, 2 x 2 of 64 x 64) or 256 (8 waves,
// 2 x 4 of 128 x 64): a 256-wide tile streams its two column panels for four
// times the products of a 128-wide one -- half the operand bytes per product
// for the wide factors, whose panel gather is what the kernel waits on.
template <int DT, int VB = VBK, int TW = BT>
__device__ __forceinline__ void syrk_vec_tile(const PatchArgs& p, int tile, int split,
                                              uint16_t* smem) {
  constexpr int VLD = VB + 8;
  constexpr int RG = VB / 64;           // 64-row groups per k-step and loader thread
  constexpr int WN = TW / 64;           // wave columns: 2 (TW 128) or 4 (TW 256)
  constexpr int MI = TW / 64, NJ = 2;   // 32x32 blocks per wave: rows x columns
  uint16_t* sA = smem;
  uint16_t* sB = smem + TW * VLD;

  int t = tile, ti = 0, rem = p.ntiles;
  while (t >= rem) { t -= rem; ++ti; --rem; }
  const int tj = ti + t;
  const bool diag = (ti == tj);

  const long long r_begin = (long long)split * p.rows_per_split;
  long long r_end = r_begin + p.rows_per_split;
  if (r_end > p.M) r_end = p.M;
  if (r_begin >= r_end) return;
  const int nk = (int)((r_end - r_begin + VB - 1) / VB);

  // global address space: a plain pointer from the problem table compiles to
  // flat loads, which count on lgkmcnt too, so the MFMA step's LDS fragment
  // waits would also wait for the next k-step's gather (no overlap)
  const AS1 uint16_t* x = gptr((const uint16_t*)p.x);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // loader role: operand (0 = A tile ti, 1 = B tile tj), row group, column chunk.
  // Row group fastest: the 8 lanes of one ds_write_b128 lane group store the
  // same LDS rows at 8 different k offsets = 32 distinct banks.  (Column chunk
  // fastest put them 8 LDS rows apart = 288 dwords = the same 4 banks: 8-way
  // conflicts, 72 % of the kernel's LDS cycles, profiles/README.md.)  A wave's
  // global loads still read 128 contiguous bytes per patch row.
  const int op = tid / TW;
  const int rg = tid & 7;               // rows rg*8 .. rg*8+7 of each 64-row group
  const int cc = (tid % TW) >> 3;       // columns cc*8 .. cc*8+7 of the tile
  const bool loader = !(diag && op == 1);
  const int gcol = (op ? tj : ti) * TW + cc * 8;
  // chunk kind: 0 = data, 1 = bias (first column of the chunk is the ones column), 2 = zero
  int kind = 2, coff = 0, di = 0, dj = 0;
  if (gcol < p.kcols) {
    const int rij = gcol / p.C, c0 = gcol - rij * p.C;
    const int i = rij / p.kw, j = rij - i * p.kw;
    di = i * p.dh; dj = j * p.dw;
    coff = (int)(c0 + (long long)di * p.sh + (long long)dj * p.sw);
    kind = 0;
  } else if (gcol < p.ncols) {
    kind = 1;
  }

  u32x4_t blk[RG][8];
  // Row table: the (b, oh, ow) decode of a patch row is shared by the 16
  // column chunks (and both operands) of the tile, so one wave decodes the
  // next k-step's VB rows into LDS (16 B per row: the pixel's element offset
  // and its top-left (h, w)) and every loader reads it back -- the per-row
  // 64-bit divisions / multiplies made the gather VALU-bound (~45 vector
  // instructions per 16-B load; the MFMAs of a k-step hide ~24 cycles each).
  // Padding / bias / zero / past-the-split elements load from a 16-B constant
  // (zeros, or the ones column's [1, 0, ...]) instead of being masked: no
  // select on the loaded data, one pointer select per row.
  int4* rtab = (int4*)(smem + 2 * TW * VLD);            // [2][VB] entries
  constexpr int ROW_NONE = -(1 << 30);                  // hs of a row past the split
  const AS1 u32x4_t* zeros = gptr((const u32x4_t*)g_syrk_const[0]);
  const AS1 u32x4_t* alt = (kind == 1) ? gptr((const u32x4_t*)g_syrk_const[DT == KDT_BF16 ? 1 : 2])
                                      : zeros;
  // kind != 0: no (h, w) passes the bounds test
  if (kind != 0) { di = ROW_NONE; dj = 0; }
  auto decode_rows = [&](int k) {
    if (tid < VB) {                                     // wave 0 (VB = 64)
      const long long r = r_begin + (long long)k * VB + tid;
      int4 e = make_int4(0, 0, ROW_NONE, 0);
      if (r < r_end) {
        const long long ohw = (long long)p.OH * p.OW;
        long long b;
        int rr;
        if (p.M < (1ll << 31)) {      // wave-uniform: 32-bit divisions
          const unsigned bu = (unsigned)r / (unsigned)ohw;
          b = bu;
          rr = (int)((unsigned)r - bu * (unsigned)ohw);
        } else {
          b = r / ohw;
          rr = (int)(r - b * ohw);
        }
        const int oh = (int)((unsigned)rr / (unsigned)p.OW), ow = rr - oh * p.OW;
        const int hs = oh * p.sth - p.ph, ws = ow * p.stw - p.pw;
        const long long off = b * p.sb + (long long)hs * p.sh + (long long)ws * p.sw;
        e = make_int4((int)(unsigned)(off & 0xffffffffll), (int)(off >> 32), hs, ws);
      }
      // row j at slot j ^ ((j >> 3) & 7): conflict-free for this store (slots
      // mod 8 distinct in each 8-lane group) and for the loaders' reads (rows
      // rg*8 + q of the 8 loader groups land on 8 distinct slots mod 16)
      const int j = tid;
      rtab[(k & 1) * VB + (j ^ ((j >> 3) & 7))] = e;
    }
  };
  // every row-table read first (one LDS wait), then branch-free integer
  // address selects, then the loads back to back (a pointer ?: per load
  // compiled to a divergent branch with an LDS read and a full lgkmcnt wait
  // inside it: eight serial LDS round trips per k-step before the loads)
  auto load_step = [&](int k, u32x4_t (&dst)[RG][8]) {
    const int4* rt = rtab + (k & 1) * VB;
    int4 ev[RG][8];
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int q = 0; q < 8; ++q) ev[g][q] = rt[g * 64 + rg * 8 + (q ^ rg)];
    const unsigned long long xb = (unsigned long long)(size_t)(x + coff);
    const unsigned long long pz = (unsigned long long)(size_t)zeros;
    const unsigned long long pa = (unsigned long long)(size_t)alt;
#pragma unroll
    for (int g = 0; g < RG; ++g) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int4 e = ev[g][q];
        const long long off = ((long long)e.y << 32) | (unsigned)e.x;
        const bool in = ((unsigned)(e.z + di) < (unsigned)p.H) & ((unsigned)(e.w + dj) < (unsigned)p.W);
        const unsigned long long pin = xb + (unsigned long long)(off * 2);
        const unsigned long long pout = (e.z != ROW_NONE) ? pa : pz;
        dst[g][q] = *(const AS1 u32x4_t*)(size_t)(in ? pin : pout);
      }
    }
  };
  auto store_step = [&](const u32x4_t (&src)[RG][8]) {
    if (!loader) return;
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      uint16_t* dst = (op ? sB : sA) + (cc * 8) * VLD + g * 64 + rg * 8;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int d = c >> 1;
        uint4 o;
        if (c & 1) {
          o.x = pack_hi(u4get(src[g][0], d), u4get(src[g][1], d));
          o.y = pack_hi(u4get(src[g][2], d), u4get(src[g][3], d));
          o.z = pack_hi(u4get(src[g][4], d), u4get(src[g][5], d));
          o.w = pack_hi(u4get(src[g][6], d), u4get(src[g][7], d));
        } else {
          o.x = pack_lo(u4get(src[g][0], d), u4get(src[g][1], d));
          o.y = pack_lo(u4get(src[g][2], d), u4get(src[g][3], d));
          o.z = pack_lo(u4get(src[g][4], d), u4get(src[g][5], d));
          o.w = pack_lo(u4get(src[g][6], d), u4get(src[g][7], d));
        }
        *(uint4*)(dst + c * VLD) = o;
      }
    }
  };

  const int wr = wave / WN, wc = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int m = 0; m < MI; ++m)
#pragma unroll
    for (int n = 0; n < NJ; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
  const uint16_t* sBr = diag ? sA : sB;

  auto mfma_step = [&]() {
    typedef typename std::conditional<DT == KDT_BF16, bf16x8_t, f16x8_t>::type frag_t;
#pragma unroll
    for (int ks = 0; ks < VB / 16; ++ks) {
      frag_t a[MI], bb[NJ];
#pragma unroll
      for (int m = 0; m < MI; ++m)
        a[m] = *(const frag_t*)(sA + (wr * 32 * MI + m * 32 + lr) * VLD + ks * 16 + lh * 8);
#pragma unroll
      for (int n = 0; n < NJ; ++n)
        bb[n] = *(const frag_t*)(sBr + (wc * 32 * NJ + n * 32 + lr) * VLD + ks * 16 + lh * 8);
#pragma unroll
      for (int m = 0; m < MI; ++m)
#pragma unroll
        for (int n = 0; n < NJ; ++n) {
          if constexpr (DT == KDT_BF16)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m], bb[n], acc[m][n], 0, 0, 0);
          else
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m], bb[n], acc[m][n], 0, 0, 0);
        }
    }
  };

  decode_rows(0);
  __syncthreads();
  if (loader) load_step(0, blk);
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) decode_rows(k + 1);     // slot (k+1)&1: last read by load_step(k-1)
    store_step(blk);
    __syncthreads();
    if (loader && k + 1 < nk) load_step(k + 1, blk);
    mfma_step();
    __syncthreads();
  }

  store_tile<TW, MI, NJ>(p, acc, tile, split, ti, tj, diag, wr, wc, lr, lh);
}

template <int DT>
__global__ __launch_bounds__(256) void syrk_vec_kernel(PatchArgs p) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[SyrkVecLds<VBK>::ELEMS];
  syrk_vec_tile<DT>(p, blockIdx.x, blockIdx.y, smem);
}

// Grouped form: every channels-contiguous factor of a K-FAC factor step in
// ONE launch (each problem owns `blocks` = tile pairs x row splits blocks
// starting at `block_begin`), so the small factors no longer run as
// under-filled launches of their own.
struct SyrkProblem {
  PatchArgs p;
  int block_begin, blocks, dtype, tw;   // tw: tile width (128 / 256)
};

// Tables travel BY VALUE in the kernel arguments (< 4 KB), so a launch is
// capturable into a hipGraph with its problem pointers baked in (no H2D copy).
constexpr int MAX_SYRK_PROBLEMS = 22;
struct SyrkBatch {
  int count, pad[3];
  SyrkProblem prob[MAX_SYRK_PROBLEMS];
};
static_assert(sizeof(SyrkBatch) <= 4096, "kernel arguments are limited to 4 KB");

template <int DT, int TW = BT, int VB = VBK>
__global__ __launch_bounds__(2 * TW) void syrk_vec_grouped_kernel(const SyrkBatch* __restrict__ batch) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[SyrkVecLds<VB, TW>::ELEMS];
  const SyrkProblem* t = batch->prob;
  const int count = batch->count;
  int lo = 0, hi = count - 1;
  // hardware order: an XCD-contiguous remap (a split's tiles on one L2)
  // measured 3.34 -> 3.43 ms (profiles/r3_factors_xcd_remap.log)
  const int b = blockIdx.x;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].block_begin <= b) lo = mid; else hi = mid - 1;
  }
  const SyrkProblem& P = t[lo];
  const int local = b - P.block_begin;
  const int tiles = P.p.ntiles * (P.p.ntiles + 1) / 2;
  syrk_vec_tile<DT, VB, TW>(P.p, local % tiles, local / tiles, smem);
}

// ---------------------------------------------------------------------------
// fp32 inputs with few channels (ResNet's conv1: C = 3) onto the channels-
// contiguous MFMA path: x * s is split into fp16 hi / lo planes, channels
// [hi_0 .. hi_{C-1}, lo_0 .. lo_{C-1}, 0 ..] of an 8-channel NHWC tensor
// (22 significand bits; s = 2^k puts max |x| s in [2^13, 2^14)), and the
// factor is the sum of the SYRK's four plane-pair blocks scaled by 1 / s^2
// (a device factor: the SYRK store's dscale).  The generic fp32 SYRK this
// replaces ran conv1's A factor (401408 x 147) at 0.51 ms on the f32 MFMA.
constexpr int SPLIT_BLOCKS = 512;

__device__ __forceinline__ float block_max256(float m) {
  __shared__ float red[4];
  for (int d = 32; d > 0; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return m;
}

// per-block max |x| -> part[blockIdx.x] (fixed grid, no atomics)
__global__ __launch_bounds__(256) void split_absmax_kernel(const float* __restrict__ x, int C,
                                                           int H, int W, long long sb,
                                                           long long sc, long long sh,
                                                           long long sw, long long total,
                                                           float* __restrict__ part) {
  float m = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const long long b = t / H;
    m = fmaxf(m, fabsf(x[b * sb + c * sc + h * sh + w * sw]));
  }
  m = block_max256(m);
  if (threadIdx.x == 0) part[blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void split_f16_kernel(const float* __restrict__ x, int C, int H,
                                                        int W, long long sb, long long sc,
                                                        long long sh, long long sw, long long npix,
                                                        const float* __restrict__ part,
                                                        uint4* __restrict__ out,
                                                        float* __restrict__ dscale) {
  float m = 0.f;
  for (int i = threadIdx.x; i < SPLIT_BLOCKS; i += 256) m = fmaxf(m, part[i]);
  m = block_max256(m);
  int e = 0;
  (void)frexpf(m, &e);
  int k = (m > 0.f && m <= 3.0e38f) ? 14 - e : 0;
  k = k < -60 ? -60 : (k > 60 ? 60 : k);
  const float s = ldexpf(1.f, k);
  if (blockIdx.x == 0 && threadIdx.x == 0) *dscale = ldexpf(1.f, -2 * k);
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < npix; p += (long long)gridDim.x * 256) {
    const int w = (int)(p % W);
    long long t = p / W;
    const int h = (int)(t % H);
    const long long b = t / H;
    const float* px = x + b * sb + h * sh + w * sw;
    unsigned short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < C; ++c) {
      const float y = px[c * sc] * s;
      const _Float16 hi = (_Float16)y;
      const _Float16 lo = (_Float16)(y - (float)hi);
      v[c] = __builtin_bit_cast(unsigned short, hi);
      v[C + c] = __builtin_bit_cast(unsigned short, lo);
    }
    uint4 o;
    o.x = v[0] | ((unsigned)v[1] << 16);
    o.y = v[2] | ((unsigned)v[3] << 16);
    o.z = v[4] | ((unsigned)v[5] << 16);
    o.w = v[6] | ((unsigned)v[7] << 16);
    out[p] = o;
  }
}

// Grouped EMA (with the internal->reference permutation): one block row per
// (factor, row i).
struct EmaJob {
  void* state; const float* ws;
  int n, ldw, kcols, C, kk, sdtype, row_begin;
  int full;              // ws holds both triangles (tile_reduce mirror): row reads only
  float a1, a2;
  int mode;
  int cint;              // channels of the internal order (C, or 8 for split planes)
  int lo;                // 0, or the channel offset of the low plane (kfac_split_f16):
                         // the factor is the sum of the four plane-pair blocks
  int pad3;
  const float* keep;     // nullptr, or device flag: 0 leaves the factor untouched (AMP)
};

// Reference column order (c, i, j) -> internal order (i, j, c) of syrk_vec
// with `cint` channels per tap.
__device__ __forceinline__ int perm_col(int x, int kcols, int C, int kk, int cint) {
  if (x >= kcols || (kk == 1 && cint == C)) return x;
  const int c = x / kk, r = x - c * kk;
  return r * cint + c;
}
__device__ __forceinline__ int perm_col(int x, int kcols, int C, int kk) {
  return perm_col(x, kcols, C, kk, C);
}

// EMA with the internal->reference column permutation (see syrk_vec).
template <int SDT>
__global__ __launch_bounds__(256) void factor_ema_perm_kernel(
    typename DTypeTraits<SDT>::raw_t* __restrict__ state, const float* __restrict__ ws,
    int n, int ldw, float a1, float a2, int mode, int kcols, int C, int kk,
    const float* __restrict__ keep) {
  typedef DTypeTraits<SDT> Tr;
  if (keep != nullptr && *keep == 0.f) return;
  const int i = blockIdx.y;
  const int pi = perm_col(i, kcols, C, kk);
  for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    const int pj = perm_col(j, kcols, C, kk);
    const float w = (pi <= pj) ? ws[(long long)pi * ldw + pj] : ws[(long long)pj * ldw + pi];
    const long long o = (long long)i * n + j;
    const float s = (mode == 0) ? (Tr::to_f32(state[o]) * a1 + w) * a2 : w;
    state[o] = Tr::from_f32(s);
  }
}

template <int SDT>
__device__ __forceinline__ void ema_perm_row(const EmaJob& J, int i) {
  typedef DTypeTraits<SDT> Tr;
  if (J.keep != nullptr && *J.keep == 0.f) return;
  typename Tr::raw_t* state = (typename Tr::raw_t*)J.state;
  const int pi = perm_col(i, J.kcols, J.C, J.kk, J.cint);
  const float* wrow = J.ws + (long long)pi * J.ldw;
  const float* wlo = wrow + (long long)J.lo * J.ldw;
  for (int j = threadIdx.x; j < J.n; j += 256) {
    const int pj = perm_col(j, J.kcols, J.C, J.kk, J.cint);
    float w;
    if (J.lo)      // (hi + lo)^T (hi + lo): the four plane-pair blocks (full ws),
                   // added in an order the transpose reproduces bitwise
      w = (wrow[pj] + wlo[pj + J.lo]) + (wrow[pj + J.lo] + wlo[pj]);
    else
      w = (J.full || pi <= pj) ? wrow[pj] : J.ws[(long long)pj * J.ldw + pi];
    const long long o = (long long)i * J.n + j;
    const float v = (J.mode == 0) ? (Tr::to_f32(state[o]) * J.a1 + w) * J.a2 : w;
    state[o] = Tr::from_f32(v);
  }
}

constexpr int MAX_EMA_JOBS = 50;
struct EmaBatch {
  int count, pad[3];
  EmaJob job[MAX_EMA_JOBS];
};
static_assert(sizeof(EmaBatch) <= 4096, "kernel arguments are limited to 4 KB");

__global__ __launch_bounds__(256) void factor_ema_grouped_kernel(const EmaBatch* __restrict__ batch) {
  const EmaJob* t = batch->job;
  const int count = batch->count;
  int lo = 0, hi = count - 1;
  const int b = blockIdx.x;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].row_begin <= b) lo = mid; else hi = mid - 1;
  }
  const EmaJob& J = t[lo];
  const int i = b - J.row_begin;
  if (J.sdtype == KDT_F32) ema_perm_row<KDT_F32>(J, i);
  else if (J.sdtype == KDT_BF16) ema_perm_row<KDT_BF16>(J, i);
  else ema_perm_row<KDT_F16>(J, i);
}

// state = a2 * (a1 * state + ws_sym)   (mode 0: EMA, a1 = alpha/(1-alpha), a2 = 1-alpha)
// state = ws_sym                       (mode 1: assign)
// The workspace holds only the upper triangle; (i, j) with i > j reads ws[j][i].
template <int SDT>
__global__ __launch_bounds__(256) void factor_ema_kernel(
    typename DTypeTraits<SDT>::raw_t* __restrict__ state, const float* __restrict__ ws,
    int n, int ldw, float a1, float a2, int mode, const float* __restrict__ keep) {
  typedef DTypeTraits<SDT> Tr;
  if (keep != nullptr && *keep == 0.f) return;
  __shared__ float tile[32][33];
  const int bi = blockIdx.y, bj = blockIdx.x;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  if (bi > bj) {
    for (int r = ty; r < 32; r += 8) {
      int i = bj * 32 + r, j = bi * 32 + tx;
      tile[r][tx] = (i < n && j < n) ? ws[(long long)i * ldw + j] : 0.f;
    }
    __syncthreads();
  }
  for (int r = ty; r < 32; r += 8) {
    int i = bi * 32 + r, j = bj * 32 + tx;
    if (i >= n || j >= n) continue;
    float w;
    if (bi > bj) w = tile[tx][r];
    else w = (i <= j) ? ws[(long long)i * ldw + j] : ws[(long long)j * ldw + i];
    long long o = (long long)i * n + j;
    float s = (mode == 0) ? (Tr::to_f32(state[o]) * a1 + w) * a2 : w;
    state[o] = Tr::from_f32(s);
  }
}

// Pack the upper triangle (row-major, diagonal included) of a symmetric n x n
// matrix into `out` (dtype of the matrix).
template <int DT>
__global__ void triu_pack_kernel(const typename DTypeTraits<DT>::raw_t* __restrict__ a,
                                 typename DTypeTraits<DT>::raw_t* __restrict__ out, int n) {
  const int i = blockIdx.y;
  const long long row_off = (long long)i * n - (long long)i * (i - 1) / 2;  // packed start of row i
  for (int j = i + blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    out[row_off + (j - i)] = a[(long long)i * n + j];
}

// Unpack + mirror + scale (scale = 1/world folds the AVERAGE in).
template <int DT>
__global__ __launch_bounds__(256) void triu_unpack_kernel(
    const typename DTypeTraits<DT>::raw_t* __restrict__ packed,
    typename DTypeTraits<DT>::raw_t* __restrict__ a, int n, float scale) {
  typedef DTypeTraits<DT> Tr;
  __shared__ float tile[32][33];
  const int bi = blockIdx.y, bj = blockIdx.x;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  auto pidx = [n](long long i, long long j) { return i * n - i * (i - 1) / 2 + (j - i); };
  if (bi > bj) {
    for (int r = ty; r < 32; r += 8) {
      int i = bj * 32 + r, j = bi * 32 + tx;
      tile[r][tx] = (i < n && j < n) ? Tr::to_f32(packed[pidx(i, j)]) : 0.f;
    }
    __syncthreads();
  }
  for (int r = ty; r < 32; r += 8) {
    int i = bi * 32 + r, j = bj * 32 + tx;
    if (i >= n || j >= n) continue;
    float v;
    if (bi > bj) v = tile[tx][r];
    else v = Tr::to_f32(packed[(i <= j) ? pidx(i, j) : pidx(j, i)]);
    a[(long long)i * n + j] = Tr::from_f32(v * scale);
  }
}

}  // namespace

// ------------------------------------------------------------------ C ABI
KFAC_API int kfac_syrk_patch(int dtype, const void* x, long long sb, long long sc, long long sh,
                             long long sw, int B, int C, int H, int W, int kh, int kw, int sth,
                             int stw, int ph, int pw, int dh, int dw, int has_bias, float scale,
                             float* ws, int ldw, int max_blocks, float* part,
                             const float* dscale, hipStream_t stream) {
  PatchArgs p;
  p.part = part;
  p.dscale = dscale;
  p.x = x; p.sb = sb; p.sc = sc; p.sh = sh; p.sw = sw;
  p.B = B; p.C = C; p.H = H; p.W = W;
  p.kh = kh; p.kw = kw; p.sth = sth; p.stw = stw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.OH = (H + 2 * ph - dh * (kh - 1) - 1) / sth + 1;
  p.OW = (W + 2 * pw - dw * (kw - 1) - 1) / stw + 1;
  p.kcols = C * kh * kw;
  p.ncols = p.kcols + (has_bias ? 1 : 0);
  p.M = (long long)B * p.OH * p.OW;
  p.ntiles = (p.ncols + BT - 1) / BT;
  p.scale = scale; p.ws = ws; p.ldw = ldw;
  if (p.M <= 0 || p.OH <= 0 || p.OW <= 0) return 0;
  const int tiles = p.ntiles * (p.ntiles + 1) / 2;
  // split the row dimension so the grid covers the chip several times over
  if (max_blocks <= 0) max_blocks = 2048;
  long long ksteps = (p.M + BK - 1) / BK;
  long long splits = (max_blocks + tiles - 1) / tiles;
  if (splits < 1) splits = 1;
  if (splits > ksteps) splits = ksteps;
  long long steps_per = (ksteps + splits - 1) / splits;
  p.rows_per_split = steps_per * BK;
  splits = (p.M + p.rows_per_split - 1) / p.rows_per_split;
  dim3 grid(tiles, (unsigned)splits), block(256);
  const bool lane_cols = (sc == 1);
  if (dtype == KDT_BF16) {
    if (lane_cols) hipLaunchKernelGGL((syrk_patch_kernel<KDT_BF16, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((syrk_patch_kernel<KDT_BF16, false>), grid, block, 0, stream, p);
  } else if (dtype == KDT_F16) {
    if (lane_cols) hipLaunchKernelGGL((syrk_patch_kernel<KDT_F16, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((syrk_patch_kernel<KDT_F16, false>), grid, block, 0, stream, p);
  } else if (dtype == KDT_F32) {
    if (lane_cols) hipLaunchKernelGGL((syrk_patch_kernel<KDT_F32, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((syrk_patch_kernel<KDT_F32, false>), grid, block, 0, stream, p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// Fast path entry: returns 1 when syrk_vec ran (columns in internal order),
// 0 when the inputs do not qualify (caller falls back to kfac_syrk_patch).
KFAC_API int kfac_syrk_vec(int dtype, const void* x, long long sb, long long sc, long long sh,
                           long long sw, int B, int C, int H, int W, int kh, int kw, int sth,
                           int stw, int ph, int pw, int dh, int dw, int has_bias, float scale,
                           float* ws, int ldw, int max_blocks, float* part,
                           const float* dscale, hipStream_t stream) {
  if (!(dtype == KDT_BF16 || dtype == KDT_F16)) return 0;
  if (sc != 1 || (C % 8) || (sb % 8) || (H > 1 && (sh % 8)) || (W > 1 && (sw % 8)) ||
      (((uintptr_t)x) & 15))
    return 0;
  PatchArgs p;
  p.part = part;
  p.dscale = dscale;
  p.x = x; p.sb = sb; p.sc = sc; p.sh = sh; p.sw = sw;
  p.B = B; p.C = C; p.H = H; p.W = W;
  p.kh = kh; p.kw = kw; p.sth = sth; p.stw = stw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.OH = (H + 2 * ph - dh * (kh - 1) - 1) / sth + 1;
  p.OW = (W + 2 * pw - dw * (kw - 1) - 1) / stw + 1;
  p.kcols = C * kh * kw;
  p.ncols = p.kcols + (has_bias ? 1 : 0);
  p.M = (long long)B * p.OH * p.OW;
  p.ntiles = (p.ncols + BT - 1) / BT;
  p.scale = scale; p.ws = ws; p.ldw = ldw;
  if (p.M <= 0 || p.OH <= 0 || p.OW <= 0) return 1;
  const int tiles = p.ntiles * (p.ntiles + 1) / 2;
  if (max_blocks <= 0) max_blocks = 2048;
  long long ksteps = (p.M + VBK - 1) / VBK;
  long long splits = (max_blocks + tiles - 1) / tiles;
  if (splits < 1) splits = 1;
  if (splits > ksteps) splits = ksteps;
  long long steps_per = (ksteps + splits - 1) / splits;
  p.rows_per_split = steps_per * VBK;
  splits = (p.M + p.rows_per_split - 1) / p.rows_per_split;
  dim3 grid(tiles, (unsigned)splits), block(256);
  if (dtype == KDT_BF16)
    hipLaunchKernelGGL(syrk_vec_kernel<KDT_BF16>, grid, block, 0, stream, p);
  else
    hipLaunchKernelGGL(syrk_vec_kernel<KDT_F16>, grid, block, 0, stream, p);
  int err = (int)hipGetLastError();
  return err ? -err : 1;
}

KFAC_API int kfac_factor_ema_perm(int sdtype, void* state, const float* ws, int n, int ldw,
                                  float alpha, int mode, int kcols, int C, int kk,
                                  const float* keep, hipStream_t stream) {
  float a1 = 0.f, a2 = 1.f;
  if (mode == 0) { a1 = alpha / (1.f - alpha); a2 = 1.f - alpha; }
  dim3 grid((n + 255) / 256 < 8 ? (n + 255) / 256 : 8, n), block(256);
  if (sdtype == KDT_F32)
    hipLaunchKernelGGL(factor_ema_perm_kernel<KDT_F32>, grid, block, 0, stream, (float*)state, ws, n, ldw, a1, a2, mode, kcols, C, kk, keep);
  else if (sdtype == KDT_BF16)
    hipLaunchKernelGGL(factor_ema_perm_kernel<KDT_BF16>, grid, block, 0, stream, (uint16_t*)state, ws, n, ldw, a1, a2, mode, kcols, C, kk, keep);
  else if (sdtype == KDT_F16)
    hipLaunchKernelGGL(factor_ema_perm_kernel<KDT_F16>, grid, block, 0, stream, (uint16_t*)state, ws, n, ldw, a1, a2, mode, kcols, C, kk, keep);
  else
    return -1;
  return (int)hipGetLastError();
}

KFAC_API int kfac_factor_ema(int sdtype, void* state, const float* ws, int n, int ldw, float alpha,
                             int mode, const float* keep, hipStream_t stream) {
  float a1 = 0.f, a2 = 1.f;
  if (mode == 0) { a1 = alpha / (1.f - alpha); a2 = 1.f - alpha; }
  int nb = (n + 31) / 32;
  dim3 grid(nb, nb), block(256);
  if (sdtype == KDT_F32)
    hipLaunchKernelGGL(factor_ema_kernel<KDT_F32>, grid, block, 0, stream, (float*)state, ws, n, ldw, a1, a2, mode, keep);
  else if (sdtype == KDT_BF16)
    hipLaunchKernelGGL(factor_ema_kernel<KDT_BF16>, grid, block, 0, stream, (uint16_t*)state, ws, n, ldw, a1, a2, mode, keep);
  else if (sdtype == KDT_F16)
    hipLaunchKernelGGL(factor_ema_kernel<KDT_F16>, grid, block, 0, stream, (uint16_t*)state, ws, n, ldw, a1, a2, mode, keep);
  else
    return -1;
  return (int)hipGetLastError();
}

KFAC_API int kfac_triu_pack(int dtype, const void* a, void* out, int n, hipStream_t stream) {
  dim3 grid((n + 255) / 256, n), block(256);
  if (dtype == KDT_F32)
    hipLaunchKernelGGL(triu_pack_kernel<KDT_F32>, grid, block, 0, stream, (const float*)a, (float*)out, n);
  else if (dtype == KDT_BF16)
    hipLaunchKernelGGL(triu_pack_kernel<KDT_BF16>, grid, block, 0, stream, (const uint16_t*)a, (uint16_t*)out, n);
  else if (dtype == KDT_F16)
    hipLaunchKernelGGL(triu_pack_kernel<KDT_F16>, grid, block, 0, stream, (const uint16_t*)a, (uint16_t*)out, n);
  else
    return -1;
  return (int)hipGetLastError();
}

KFAC_API int kfac_triu_unpack(int dtype, const void* packed, void* a, int n, float scale,
                              hipStream_t stream) {
  int nb = (n + 31) / 32;
  dim3 grid(nb, nb), block(256);
  if (dtype == KDT_F32)
    hipLaunchKernelGGL(triu_unpack_kernel<KDT_F32>, grid, block, 0, stream, (const float*)packed, (float*)a, n, scale);
  else if (dtype == KDT_BF16)
    hipLaunchKernelGGL(triu_unpack_kernel<KDT_BF16>, grid, block, 0, stream, (const uint16_t*)packed, (uint16_t*)a, n, scale);
  else if (dtype == KDT_F16)
    hipLaunchKernelGGL(triu_unpack_kernel<KDT_F16>, grid, block, 0, stream, (const uint16_t*)packed, (uint16_t*)a, n, scale);
  else
    return -1;
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ grouped API
KFAC_API int kfac_syrk_problem_size() { return (int)sizeof(SyrkProblem); }
KFAC_API int kfac_ema_job_size() { return (int)sizeof(EmaJob); }

// Fill the derived fields of a SyrkProblem from the user fields (host side):
// returns the number of blocks, or 0 when the input does not qualify for the
// channels-contiguous path.  split_rows: target patch rows per block.
KFAC_API int kfac_syrk_problem_init(SyrkProblem* P, int block_begin, int dtype, const void* x,
                                    long long sb,
                                    long long sc, long long sh, long long sw, int B, int C, int H,
                                    int W, int kh, int kw, int sth, int stw, int ph, int pw, int dh,
                                    int dw, int has_bias, float scale, float* ws, int ldw,
                                    long long split_rows, int tile_width) {
  if (tile_width != 128 && tile_width != 256) return 0;
  if (!(dtype == KDT_BF16 || dtype == KDT_F16)) return 0;
  if (sc != 1 || (C % 8) || (sb % 8) || (H > 1 && (sh % 8)) || (W > 1 && (sw % 8)) ||
      (((uintptr_t)x) & 15))
    return 0;
  PatchArgs& p = P->p;
  p.part = nullptr;      // kfac_syrk_problem_set_part
  p.dscale = nullptr;    // kfac_syrk_problem_set_dscale
  p.x = x; p.sb = sb; p.sc = sc; p.sh = sh; p.sw = sw;
  p.B = B; p.C = C; p.H = H; p.W = W;
  p.kh = kh; p.kw = kw; p.sth = sth; p.stw = stw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.OH = (H + 2 * ph - dh * (kh - 1) - 1) / sth + 1;
  p.OW = (W + 2 * pw - dw * (kw - 1) - 1) / stw + 1;
  p.kcols = C * kh * kw;
  p.ncols = p.kcols + (has_bias ? 1 : 0);
  p.M = (long long)B * p.OH * p.OW;
  p.ntiles = (p.ncols + tile_width - 1) / tile_width;
  p.scale = scale; p.ws = ws; p.ldw = ldw;
  if (p.M <= 0) return 0;
  if (split_rows < VBK) split_rows = VBK;
  split_rows = (split_rows + VBK - 1) / VBK * VBK;
  long long splits = (p.M + split_rows - 1) / split_rows;
  p.rows_per_split = (p.M + splits - 1) / splits;
  p.rows_per_split = (p.rows_per_split + VBK - 1) / VBK * VBK;
  splits = (p.M + p.rows_per_split - 1) / p.rows_per_split;
  P->dtype = dtype;
  P->block_begin = block_begin;
  P->tw = tile_width;
  P->blocks = (int)(splits * (p.ntiles * (p.ntiles + 1) / 2));
  return P->blocks;
}

// host_table: `count` SyrkProblem records (block_begin relative to the
// first); launched in batches of MAX_SYRK_PROBLEMS.
// The 256-wide problems go first (their long k-loops start first), then the
// 128-wide ones; one launch per tile width and MAX_SYRK_PROBLEMS problems.
KFAC_API int kfac_syrk_grouped(const void* host_table, int count, int dtype, hipStream_t stream) {
  const SyrkProblem* t = (const SyrkProblem*)host_table;
  if (dtype != KDT_BF16 && dtype != KDT_F16) return -1;
  for (int tw : {256, 128}) {
    std::vector<int> sel;
    for (int k = 0; k < count; ++k)
      if (t[k].tw == tw) sel.push_back(k);
    for (size_t base = 0; base < sel.size(); base += MAX_SYRK_PROBLEMS) {
      SyrkBatch b;
      memset(&b, 0, sizeof(b));   // deterministic table bytes (devtable key)
      b.count = (int)std::min(sel.size() - base, (size_t)MAX_SYRK_PROBLEMS);
      int blocks = 0;
      for (int k = 0; k < b.count; ++k) {
        b.prob[k] = t[sel[base + k]];
        b.prob[k].block_begin = blocks;
        blocks += b.prob[k].blocks;
      }
      if (blocks == 0) continue;
      int terr = 0;
      const SyrkBatch* d = (const SyrkBatch*)kfac_devtable::get(&b, sizeof(b), stream, &terr);
      if (!d) return terr;
      if (tw == 256) {
        if (dtype == KDT_BF16)
          hipLaunchKernelGGL((syrk_vec_grouped_kernel<KDT_BF16, 256>), dim3(blocks), dim3(512), 0,
                             stream, d);
        else
          hipLaunchKernelGGL((syrk_vec_grouped_kernel<KDT_F16, 256>), dim3(blocks), dim3(512), 0,
                             stream, d);
      } else {
        if (dtype == KDT_BF16)
          hipLaunchKernelGGL((syrk_vec_grouped_kernel<KDT_BF16, 128>), dim3(blocks), dim3(256), 0,
                             stream, d);
        else
          hipLaunchKernelGGL((syrk_vec_grouped_kernel<KDT_F16, 128>), dim3(blocks), dim3(256), 0,
                             stream, d);
      }
      int err = (int)hipGetLastError();
      if (err) return err;
    }
  }
  return 0;
}

// x: (B, C, H, W) fp32 with any strides, C <= 4; out: B*H*W x 8 fp16 (NHWC,
// 16-byte aligned); part: SPLIT_BLOCKS floats of scratch; dscale: 1 float.
KFAC_API int kfac_split_f16(const float* x, int B, int C, int H, int W, long long sb,
                            long long sc, long long sh, long long sw, void* out, float* part,
                            float* dscale, hipStream_t stream) {
  if (C < 1 || C > 4 || B < 1 || H < 1 || W < 1 || ((uintptr_t)out & 15)) return -2;
  const long long npix = (long long)B * H * W;
  hipLaunchKernelGGL(split_absmax_kernel, dim3(SPLIT_BLOCKS), dim3(256), 0, stream, x, C, H, W,
                     sb, sc, sh, sw, npix * C, part);
  long long nb = (npix + 255) / 256;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(split_f16_kernel, dim3((unsigned)nb), dim3(256), 0, stream, x, C, H, W, sb,
                     sc, sh, sw, npix, part, (uint4*)out, dscale);
  return (int)hipGetLastError();
}
KFAC_API int kfac_split_blocks() { return SPLIT_BLOCKS; }

KFAC_API int kfac_ema_grouped(const void* host_table, int count, hipStream_t stream) {
  const EmaJob* t = (const EmaJob*)host_table;
  for (int base = 0; base < count; base += MAX_EMA_JOBS) {
    EmaBatch b;
    memset(&b, 0, sizeof(b));   // deterministic table bytes (devtable key)
    b.count = count - base < MAX_EMA_JOBS ? count - base : MAX_EMA_JOBS;
    int rows = 0;
    for (int k = 0; k < b.count; ++k) {
      b.job[k] = t[base + k];
      b.job[k].row_begin = rows;
      rows += b.job[k].n;
    }
    if (rows == 0) continue;
    int terr = 0;
    const EmaBatch* d = (const EmaBatch*)kfac_devtable::get(&b, sizeof(b), stream, &terr);
    if (!d) return terr;
    hipLaunchKernelGGL(factor_ema_grouped_kernel, dim3(rows), dim3(256), 0, stream, d);
    int err = (int)hipGetLastError();
    if (err) return err;
  }
  return 0;
}

// Row splits kfac_syrk_patch (vec = 0) / kfac_syrk_vec (vec = 1) use for M
// patch rows and ncols columns: a partial buffer holds splits x tile pairs x
// 128 x 128 floats.
KFAC_API long long kfac_syrk_splits(int vec, long long M, int ncols, int max_blocks) {
  const long long bk = vec ? VBK : BK;
  const int nt = (ncols + BT - 1) / BT, tiles = nt * (nt + 1) / 2;
  if (M <= 0) return 0;
  if (max_blocks <= 0) max_blocks = 2048;
  long long ksteps = (M + bk - 1) / bk;
  long long splits = (max_blocks + tiles - 1) / tiles;
  if (splits < 1) splits = 1;
  if (splits > ksteps) splits = ksteps;
  const long long rps = (ksteps + splits - 1) / splits * bk;
  return (M + rps - 1) / rps;
}

KFAC_API void kfac_syrk_problem_set_part(SyrkProblem* P, float* part) { P->p.part = part; }
KFAC_API void kfac_syrk_problem_set_dscale(SyrkProblem* P, const float* dscale) {
  P->p.dscale = dscale;
}

KFAC_API int kfac_red_job_size() { return (int)sizeof(RedJob); }
KFAC_API int kfac_red_max_contrib() { return MAX_CONTRIB; }

// host_jobs: `count` RedJob records (block_begin filled in here): one launch
// per MAX_RED_JOBS jobs.
KFAC_API int kfac_tile_reduce(const void* host_jobs, int count, hipStream_t stream) {
  const RedJob* t = (const RedJob*)host_jobs;
  for (int base = 0; base < count; base += MAX_RED_JOBS) {
    RedBatch b;
    memset(&b, 0, sizeof(b));   // deterministic table bytes (devtable key)
    b.count = count - base < MAX_RED_JOBS ? count - base : MAX_RED_JOBS;
    int blocks = 0;
    for (int k = 0; k < b.count; ++k) {
      b.job[k] = t[base + k];
      if (b.job[k].ncontrib > MAX_CONTRIB) return -2;
      if (b.job[k].bt != 128 && b.job[k].bt != 256) return -3;
      b.job[k].block_begin = blocks;
      blocks += (b.job[k].bt * b.job[k].bt / 1024) * (b.job[k].ntiles * (b.job[k].ntiles + 1) / 2);
    }
    if (blocks == 0) continue;
    int terr = 0;
    const RedBatch* d = (const RedBatch*)kfac_devtable::get(&b, sizeof(b), stream, &terr);
    if (!d) return terr;
    hipLaunchKernelGGL(tile_reduce_kernel, dim3(blocks), dim3(256), 0, stream, d);
    const int err = (int)hipGetLastError();
    if (err) return err;
  }
  return 0;
}
