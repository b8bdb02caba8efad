// Grouped eigenbasis preconditioning GEMM chain for gfx950.
//
// For every layer this rank preconditions (reference kfac/layers/base.py:321-362,459-470):
//     V = QG ((QG^T Grad QA) (.) D) QA^T,   D = dGdA  or  1 / (dG dA^T + damping)
// The chain runs as FOUR launches for ALL layers together (one grouped GEMM
// per stage, each block owns one 128x128 output tile of one layer's problem)
// instead of 4 library GEMMs + 1 Hadamard launch per layer:
//     S1  T1[g][a]  = sum_k QGt[g][k] Gct[a][k]            (= QG^T Grad)
//     S2  T2t[a][g] = sum_k QAt[a][k] T1[g][k] * Dt[a][g]  (= ((T1 QA) (.) D)^T)
//     S3  T3[g][a]  = sum_k QG[g][k]  T2t[a][k]            (= QG T2)
//     S4  V[g][a]   = sum_k T3[g][k]  QA[a][k]             (= T3 QA^T), + KL dot <V, Grad>
// Every stage is the same "NT" product C[m][n] = sum_k A[m][k] B[n][k] with
// both operands k-contiguous, so each operand is staged global -> LDS with
// 16-byte loads and read back as MFMA fragments with ds_read_b128; a
// transposed result is produced by swapping the operands (S2), never by a
// strided epilogue.  Operand buffers are zero-padded along k to a multiple
// of 64 by construction (ops/precond_fused.py), so the k-loop is unmasked.
//
// Precision modes:
//   PREC_BF16X3  operands stored as bf16 (hi, lo) planes (x ~= hi + lo), three
//                v_mfma_f32_32x32x16_bf16 per product (hi*hi + hi*lo + lo*hi),
//                f32 accumulation: ~1e-5 relative error on the preconditioned
//                gradient (fp32 GEMMs: ~1e-6, plain bf16: ~5e-3), at ~5x the
//                f32 MFMA rate.
//   PREC_F32     operands fp32, exact v_mfma_f32_32x32x2_f32 (exact f32
//                products, f32 accumulation), the reference's fp32 semantics.
//   PREC_BF16X6  operands as three bf16 planes (hi, mid, lo: 24 mantissa bits,
//                the fp32 significand), six bf16 MFMAs per product (all terms
//                above 2^-24 relative: lo.hi + hi.lo + mid.mid + mid.hi +
//                hi.mid + hi.hi), f32 accumulation: fp32-level error at the
//                bf16 MFMA rate.  The three planes of an operand are one
//                allocation (plane stride = lo - hi), so records keep two
//                pointers per operand.
// Auxiliary launches: `gather_grad` builds Gct planes from the .grad tensors
// (any memory layout, bias as the last K-FAC column), `split_copy` builds the
// QA/QG/QAt/QGt planes and Dt after each inverse update.
#include "pgemm.h"

#include <cstdlib>
#include <type_traits>
#include "devtable.h"

namespace {


// record of workgroup `blk`: lane i tests record i's tile_begin (records are
// sorted, record 0 starts at 0), one round trip instead of a dependent
// binary search
__device__ __forceinline__ int find_problem(const PGemm* __restrict__ t, int count, int blk) {
  const int lane = threadIdx.x & 63;
  const AS1 int* tb = (const AS1 int*)(gptr((const char*)t) + offsetof(PGemm, tile_begin));
  constexpr int STRIDE = sizeof(PGemm) / sizeof(int);
  int cnt = 0;
  for (int base = 0; base < count; base += 64) {
    const int i = base + lane;
    const int b = gld_if(tb, (long long)i * STRIDE, i < count, 0x7fffffff);
    cnt += __popcll(__ballot(b <= blk));
  }
  return cnt - 1;
}

typedef unsigned u32x4n __attribute__((ext_vector_type(4)));   // AS1 loads
typedef float fx2 __attribute__((ext_vector_type(2)));         // ds_read_b64 fragments

__device__ __forceinline__ void split_bf16(float x, uint16_t& h, uint16_t& l) {
  h = f32_to_bf16_bits(x);
  l = f32_to_bf16_bits(x - bf16_bits_to_f32(h));
}
// x = hi + mid + lo to the fp32 significand (each remainder is exact in f32)
__device__ __forceinline__ void split_bf16_3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f32_to_bf16_bits(x);
  const float r = x - bf16_bits_to_f32(h);
  m = f32_to_bf16_bits(r);
  l = f32_to_bf16_bits(r - bf16_bits_to_f32(m));
}
// store a value as the planes of precision PREC at element o of (hi, lo)
template <int PREC>
__device__ __forceinline__ void store_planes(void* hi, void* lo, long long o, float v) {
  if (PREC == PREC_BF16X3) {
    uint16_t h, l;
    split_bf16(v, h, l);
    ((uint16_t*)hi)[o] = h;
    ((uint16_t*)lo)[o] = l;
  } else if (PREC == PREC_BF16X6) {
    uint16_t h, m, l;
    split_bf16_3(v, h, m, l);
    uint16_t* H = (uint16_t*)hi;
    uint16_t* M = (uint16_t*)lo;
    H[o] = h;
    M[o] = m;
    (M + (M - H))[o] = l;
  } else if (PREC == STORE_F16X2) {
    const float x = v * (float)(1 << LP_QEXP);
    const _Float16 h = (_Float16)x;
    ((uint16_t*)hi)[o] = __builtin_bit_cast(uint16_t, h);
    ((uint16_t*)lo)[o] = f32_to_f16_bits(x - (float)h);
  } else if (PREC == STORE_BF16X1) {
    ((uint16_t*)hi)[o] = f32_to_bf16_bits(v);
  } else if (PREC == STORE_F16X1) {
    ((uint16_t*)hi)[o] = f32_to_f16_bits(v * (float)(1 << LP_QEXP));
  } else {
    ((float*)hi)[o] = v;
  }
}

// scale exponent of an fp32 operand whose max |x| has the bits `mx`: max |x| 2^e
// lands in [2^13, 2^14) (fp16 max 65504); 0 for an all-zero or non-finite
// operand (inf / NaN then propagate through the conversions)
__device__ __forceinline__ int lp_exp(unsigned mx) {
  const int ex = (int)((mx >> 23) & 0xff);
  return (mx == 0u || ex == 0xff) ? 0 : 14 - (ex - 127) - 1;
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((unsigned)(127 + e) << 23); }

// Tile geometry: BM x BN output tile per workgroup of WM x WN waves (each
// wave owns a (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA tiles), TK = 32 deep
// k-steps staged through one LDS image with the next k-step's global loads in
// flight under the MFMAs.  Two instantiations are launched per stage:
//   big   256 x 256, 8 waves (2 x 4), 128 x 64 per wave: half the operand
//         traffic per FLOP of the small tile -- the stage is bound by operand
//         bandwidth (measured 5 TB/s at 128 x 128, profiles/r1_pgemm_variants.log)
//   small 128 x 128, 4 waves (2 x 2), 64 x 64 per wave, for problems with a
//         dimension below 256 (layers with 64..192 channels)
constexpr int TK = 32;

// WPE: minimum waves per SIMD the register allocator must allow (1 = no
// constraint).  WPE 2 caps VGPR + AGPR at 256: two 4-wave workgroups per CU,
// one computing while the other waits at its k-step barrier.
// DBUF: two LDS images -- the next k-step is stored into the idle image
// right after the MFMAs, one barrier per k-step instead of two.
// XCD: tiles that share the larger operand's panel are given block indices
// equal mod 8 -- the same XCD, so the panel is fetched into one L2 instead of
// several (blocks are dealt round-robin over the 8 XCDs)
template <int PREC, int BM, int BN, int WM, int WN, int WPE = 1, bool DBUF = false,
          bool XCD = false>
__global__ __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(WPE)))
void pgemm_kernel(const PGemm* __restrict__ table, int count, double* __restrict__ kl) {
  constexpr bool X3 = (PREC == PREC_BF16X3), X6 = (PREC == PREC_BF16X6);
  constexpr bool X6F = (PREC == PREC_BF16X6F);     // fp32 in memory, planes in LDS
  constexpr bool X6A = (PREC == PREC_BF16X6A), X6B = (PREC == PREC_BF16X6B);
  // low-plane mixed modes (pgemm.h): LPA / LPB = which operand is the planes one
  constexpr bool LPA = PREC == PREC_F16X3A || PREC == PREC_H1A || PREC == PREC_F1A;
  constexpr bool LPB = PREC == PREC_F16X3B || PREC == PREC_H1B || PREC == PREC_F1B;
  constexpr bool F3F = PREC == PREC_F16X3F;      // both operands fp32, fixed scales
  constexpr bool LP = LPA || LPB || F3F;
  constexpr bool LPH = PREC == PREC_F16X3A || PREC == PREC_F16X3B || PREC == PREC_F1A ||
                       PREC == PREC_F1B || F3F;    // fp16 (scaled) vs bf16
  constexpr int LPN = (PREC == PREC_F16X3A || PREC == PREC_F16X3B || F3F) ? 2 : 1;   // planes
  constexpr bool PA = X6A || LPA, PB = X6B || LPB;  // plane operand in memory
  constexpr bool X6M = X6A || X6B || LP;          // one operand planes, one fp32
  constexpr bool SPL = X3 || X6;                  // split-bf16 planes in memory
  constexpr bool SWZ = X6F || X6M;                // 64-byte swizzled LDS rows
  constexpr bool IMG16 = SPL || SWZ;              // bf16 plane image in LDS
  constexpr int NT = 64 * WM * WN;                // threads
  constexpr int MI = BM / WM / 32, NJ = BN / WN / 32;
  // 80-byte rows: conflict-free ds_read_b128 (guide: LDS banking).  X6F
  // writes 8-byte plane quads, and 80-byte rows put the two rows of a
  // ds_write_b64 lane group on overlapping banks (bank-conflict cycles ~ LDS-
  // active cycles, profiles/r3_pmc_x6f_a.csv): X6F keeps 64-byte rows with the
  // 16-byte pieces XOR-swizzled by (row >> 2) & 3 -- writes (two rows = 32
  // banks) and the b128 fragment reads (16 rows = 16 disjoint 4-bank spans)
  // both conflict-free
  constexpr int LDB16 = SWZ ? TK : TK + 8;
  constexpr int LDF32 = TK + 4;   // 16-byte aligned chunk writes
  // one LDS array (guide: a second __shared__ object can de-pipeline loads)
  constexpr int PL = LP ? LPN : ((X6 || SWZ) ? 3 : (X3 ? 2 : 1));   // planes
  constexpr int LDS_BYTES = IMG16 ? (PL * (BM + BN) * LDB16 * 2) : ((BM + BN) * LDF32 * 4);
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES * (DBUF ? 2 : 1)];

  // Workgroups keep the hardware dispatch order (round-robin over the 8
  // XCDs).  An XCD-contiguous remap (guide T1) measured 2.11 -> 4.62 ms on the
  // ResNet-50 chain (profiles/r3_pgemm_xcd_remap.log): over a ragged grouped
  // grid it hands one XCD all the tiles of the big-K problems.  XCD (below)
  // only permutes tiles WITHIN a problem, in groups of 8 panels, so every XCD
  // still gets an equal share of every problem at the same time.
  const int pi = find_problem(table, count, blockIdx.x);
  const PGemm P = table[pi];                      // uniform: scalar registers
  const AS1 unsigned char* const Ah = (const AS1 unsigned char*)P.a_hi;
  const AS1 unsigned char* const Al = (const AS1 unsigned char*)P.a_lo;
  const AS1 unsigned char* const Bh = (const AS1 unsigned char*)P.b_hi;
  const AS1 unsigned char* const Bl = (const AS1 unsigned char*)P.b_lo;
  const long long lda = P.lda, ldb = P.ldb;
  const int local = blockIdx.x - P.tile_begin;
  int tm = local / P.tiles_n, tn = local - tm * P.tiles_n;
  if constexpr (XCD) {
    const int nt = (pi + 1 < count ? table[pi + 1].tile_begin : (int)gridDim.x) - P.tile_begin;
    const int tiles_m = nt / P.tiles_n, tiles_n = P.tiles_n;
    // group along the dimension with more panels; the remainder (fewer than
    // 8 panels) keeps the row-major order
    const bool by_a = tiles_m >= tiles_n;
    const int np = by_a ? tiles_m : tiles_n, other = by_a ? tiles_n : tiles_m;
    const int full = (np / 8) * 8 * other;
    int pa, ob;
    if (local < full) {
      const int i = local >> 3;
      pa = 8 * (i / other) + (local & 7);
      ob = i % other;
    } else {
      const int r = local - full;
      pa = (np / 8) * 8 + r / other;
      ob = r % other;
    }
    tm = by_a ? pa : ob;
    tn = by_a ? ob : pa;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int M = P.M, N = P.N;
  // device-sized problems (csrc/eig_dc.hip patches M / K at run time and
  // launches the worst-case tile grid): tiles past the problem exit at once
  if (m0 >= M || n0 >= N) {
    if (kl != nullptr && threadIdx.x == 0) kl[blockIdx.x] = 0.0;   // its partial slot
    return;
  }
  const int ksteps = (P.K + TK - 1) / TK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- loader: 16-byte chunks.  bf16 planes: per operand 2 planes x rows x 4
  // chunks (8 elements); f32: rows x 8 chunks (4 elements)
  // per operand: planes in memory (bf16, 8 elements per 16-byte chunk) or fp32
  constexpr bool APL = SPL || PA, BPL = SPL || PB;
  constexpr int CPRA = APL ? TK / 8 : TK / 4, CPRB = BPL ? TK / 8 : TK / 4;   // chunks per row and plane
  constexpr int MPLA = APL ? PL : 1, MPLB = BPL ? PL : 1;                     // planes in memory
  constexpr int ESZA = APL ? 2 : 4, ESZB = BPL ? 2 : 4;
  constexpr int CA = MPLA * BM * CPRA, CB = MPLB * BN * CPRB;
  constexpr int QA = CA / NT, QB = CB / NT;
  static_assert(CA % NT == 0 && CB % NT == 0, "loader split");
  // a chunk round stays in one plane: the plane index is a compile-time
  // constant (a run-time one turns the 3-way pointer select into a scratch
  // lookup table)
  constexpr bool PLANE_CT = (BM * CPRA) % NT == 0 && (BN * CPRB) % NT == 0;
  static_assert(!(X6 || X6M) || PLANE_CT, "3-plane loader needs whole chunk rounds per plane");
  // chunk c -> (row, k offset): chunks fastest, a wave's global loads read
  // whole 128-byte row segments
  auto chunk_rc = [&](int c, int rows, int cpr, int esz, int& row, int& kof) {
    const int cc = c % (rows * cpr);
    row = cc / cpr;
    kof = (cc % cpr) * (16 / esz);
  };
  // third plane (X6): one plane stride past the second
  const AS1 unsigned char* const A2 = Al + (Al - Ah);
  const AS1 unsigned char* const B2 = Bl + (Bl - Bh);
  // branch-free: rows past the problem read row m0 / n0 (in range) and are
  // zeroed by a select, so every load of a k-step issues back to back
  // per-thread 32-bit byte offsets of its chunks (operands < 4 GiB, checked
  // on the host); the k-step advances the uniform base pointer
  u32x4n ra[2][QA], rb[2][QB];   // two k-steps of loads in flight (set = k-step parity)
  unsigned offa[QA], offb[QB];
  bool oka[QA], okb[QB];
  // X6A / X6B: byte stride between the planes of the plane operand
  const unsigned pstride_a = PA ? (unsigned)(Al - Ah) : 0u;
  const unsigned pstride_b = PB ? (unsigned)(Bl - Bh) : 0u;
#pragma unroll
  for (int q = 0; q < QA; ++q) {
    const int c = tid + NT * q;
    int row, kof;
    chunk_rc(c, BM, CPRA, ESZA, row, kof);
    oka[q] = m0 + row < M;
    offa[q] = ((unsigned)(oka[q] ? m0 + row : m0) * (unsigned)lda + kof) * ESZA;
    if (PA) offa[q] += (unsigned)(c / (BM * CPRA)) * pstride_a;
  }
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const int c = tid + NT * q;
    int row, kof;
    chunk_rc(c, BN, CPRB, ESZB, row, kof);
    okb[q] = n0 + row < N;
    offb[q] = ((unsigned)(okb[q] ? n0 + row : n0) * (unsigned)ldb + kof) * ESZB;
    if (PB) offb[q] += (unsigned)(c / (BN * CPRB)) * pstride_b;
  }
  const u32x4n z4 = {0u, 0u, 0u, 0u};
  // low-plane fp16 modes: scale of the fp32 operand (its producer's max slot)
  const int lp_e = (LP && LPH && !F3F) ? lp_exp(*(const AS1 unsigned*)P.sc_in) : 0;
  // scale of the fp32 operand(s) as they are converted: A / B
  const float lp_sa = F3F ? pow2f(P.ea) : pow2f(lp_e);
  const float lp_sb = F3F ? pow2f(P.eb) : pow2f(lp_e);
  // X6F: buffer loads -- the per-thread byte offset stays in one VGPR and the
  // k-step advances the scalar soffset: no 64-bit address rebuilt per load
  // (operands < 4 GiB, checked on the host)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>((const unsigned char*)P.a_hi), 0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>((const unsigned char*)P.b_hi), 0, -1, 0x00020000);
  auto load = [&](int k0, auto setc) {
    constexpr int SET = decltype(setc)::value;
    if constexpr (SWZ) {
      // the k-step in the scalar offset (bytes per element per operand)
#pragma unroll
      for (int q = 0; q < QA; ++q)
        ra[SET][q] = __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)offa[q], k0 * ESZA, 0);
#pragma unroll
      for (int q = 0; q < QB; ++q)
        rb[SET][q] = __builtin_amdgcn_raw_buffer_load_b128(rsB, (int)offb[q], k0 * ESZB, 0);
      return;
    }
    constexpr int ESZ = ESZA;   // X3 / X6 (both planes) or F32 (both fp32)
    const long long kb = (long long)k0 * ESZ;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int plane = PLANE_CT ? NT * q / (BM * CPRA) : (tid + NT * q) / (BM * CPRA);
      const AS1 unsigned char* base = (X6 ? (plane == 0 ? Ah : (plane == 1 ? Al : A2))
                                          : (plane ? Al : Ah)) + kb;
      ra[SET][q] = *(const AS1 u32x4n*)(base + offa[q]);   // rows past M: zeroed at the store
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int plane = PLANE_CT ? NT * q / (BN * CPRB) : (tid + NT * q) / (BN * CPRB);
      const AS1 unsigned char* base = (X6 ? (plane == 0 ? Bh : (plane == 1 ? Bl : B2))
                                          : (plane ? Bl : Bh)) + kb;
      rb[SET][q] = *(const AS1 u32x4n*)(base + offb[q]);
    }
  };
  // LDS image: [A planes | B planes] rows of LDB16 bf16 (X3 / X6) or [A | B] rows of LDF32 f32
  // X6F: element offset of k offset `k` (a multiple of 4) in LDS row `row`
  auto x6f_off = [&](int row, int k) -> int {
    return ((((k >> 3) ^ (row >> 2)) & 3) << 3) | (k & 7);
  };
  // X6F: four fp32 values -> hi / mid / lo bf16 quads, one 8-byte LDS write
  // per plane (the split of split_bf16_3, so results equal PREC_BF16X6's)
  auto store_split = [&](uint16_t* dst, long long plane_stride, const u32x4n& v) {
    uint16_t h[4], m[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split_bf16_3(__uint_as_float(v[e]), h[e], m[e], l[e]);
    typedef unsigned u32x2n __attribute__((ext_vector_type(2)));
    const u32x2n ph = {h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16)};
    const u32x2n pm = {m[0] | ((unsigned)m[1] << 16), m[2] | ((unsigned)m[3] << 16)};
    const u32x2n pl = {l[0] | ((unsigned)l[1] << 16), l[2] | ((unsigned)l[3] << 16)};
    *(u32x2n*)dst = ph;
    *(u32x2n*)(dst + plane_stride) = pm;
    *(u32x2n*)(dst + 2 * plane_stride) = pl;
  };
  // LP: four fp32 values -> LPN fp16 (scaled by lp_s) or one bf16 quad
  auto store_lp = [&](uint16_t* dst, long long plane_stride, const u32x4n& v, float lp_s) {
    typedef unsigned u32x2n __attribute__((ext_vector_type(2)));
    uint16_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = __uint_as_float(v[e]);
      if (LPH) {
        const float xs = x * lp_s;
        const _Float16 hh = (_Float16)xs;
        h[e] = __builtin_bit_cast(uint16_t, hh);
        l[e] = f32_to_f16_bits(xs - (float)hh);
      } else {
        h[e] = f32_to_bf16_bits(x);
        l[e] = 0;
      }
    }
    const u32x2n ph = {h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16)};
    *(u32x2n*)dst = ph;
    if (LPN == 2) {
      const u32x2n pl = {l[0] | ((unsigned)l[1] << 16), l[2] | ((unsigned)l[3] << 16)};
      *(u32x2n*)(dst + plane_stride) = pl;
    }
  };
  // rows past the problem are zeroed HERE, not at the load: a select on a
  // loaded value consumes it, so the compiler waited for the next k-step's
  // loads right after issuing them -- before this k-step's MFMAs (the global
  // latency of every k-step exposed)
  auto store = [&](unsigned char* img, auto setc) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int c = tid + NT * q;
      const int plane = c / (BM * CPRA);
      int row, kof;
      chunk_rc(c, BM, CPRA, ESZA, row, kof);
      const u32x4n v = oka[q] ? ra[SET][q] : z4;
      if (PA) *(u32x4n*)((uint16_t*)img + (plane * BM + row) * LDB16 + x6f_off(row, kof)) = v;
      else if (LP) store_lp((uint16_t*)img + row * LDB16 + x6f_off(row, kof), (long long)BM * LDB16, v, lp_sa);
      else if (SWZ) store_split((uint16_t*)img + row * LDB16 + x6f_off(row, kof), (long long)BM * LDB16, v);
      else if (SPL) *(u32x4n*)((uint16_t*)img + (plane * BM + row) * LDB16 + kof) = v;
      else *(u32x4n*)((float*)img + row * LDF32 + kof) = (row & 16) ? v.zwxy : v;
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int c = tid + NT * q;
      const int plane = c / (BN * CPRB);
      int row, kof;
      chunk_rc(c, BN, CPRB, ESZB, row, kof);
      const u32x4n v = okb[q] ? rb[SET][q] : z4;
      if (PB) *(u32x4n*)((uint16_t*)img + (PL * BM + plane * BN + row) * LDB16 + x6f_off(row, kof)) = v;
      else if (LP) store_lp((uint16_t*)img + (PL * BM + row) * LDB16 + x6f_off(row, kof),
                            (long long)BN * LDB16, v, lp_sb);
      else if (SWZ) store_split((uint16_t*)img + (PL * BM + row) * LDB16 + x6f_off(row, kof),
                                (long long)BN * LDB16, v);
      else if (SPL) *(u32x4n*)((uint16_t*)img + (PL * BM + plane * BN + row) * LDB16 + kof) = v;
      else *(u32x4n*)((float*)img + (BM + row) * LDF32 + kof) = (row & 16) ? v.zwxy : v;
    }
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int arow0 = wr * (BM / WM), brow0 = wc * (BN / WN);
  using S0_ = std::integral_constant<int, 0>;
  using S1_ = std::integral_constant<int, 1>;
  auto mma = [&](const unsigned char* cur, unsigned char* nxt) {
    if constexpr (X3) {
      const uint16_t* sAh = (const uint16_t*)cur;
      const uint16_t* sAl = sAh + BM * LDB16;
      const uint16_t* sBh = sAh + 2 * BM * LDB16;
      const uint16_t* sBl = sBh + BN * LDB16;
#pragma unroll
      for (int kk = 0; kk < TK / 16; ++kk) {
        bf16x8_t bh[NJ], bl[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int off = (brow0 + j * 32 + lr) * LDB16 + kk * 16 + lh * 8;
          bh[j] = *(const bf16x8_t*)(sBh + off);
          bl[j] = *(const bf16x8_t*)(sBl + off);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int off = (arow0 + i * 32 + lr) * LDB16 + kk * 16 + lh * 8;
          const bf16x8_t ah = *(const bf16x8_t*)(sAh + off);
          const bf16x8_t al = *(const bf16x8_t*)(sAl + off);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
          }
        }
      }
    } else if constexpr (LP) {
      typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
      const uint16_t* sA0 = (const uint16_t*)cur;
      const uint16_t* sB0 = sA0 + PL * BM * LDB16;
#pragma unroll
      for (int kk = 0; kk < TK / 16; ++kk) {
        u16x8 bp[LPN][NJ], ap[LPN][MI];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = brow0 + j * 32 + lr;
          const int off = row * LDB16 + x6f_off(row, kk * 16 + lh * 8);
#pragma unroll
          for (int p = 0; p < LPN; ++p) bp[p][j] = *(const u16x8*)(sB0 + p * BN * LDB16 + off);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int row = arow0 + i * 32 + lr;
          const int off = row * LDB16 + x6f_off(row, kk * 16 + lh * 8);
#pragma unroll
          for (int p = 0; p < LPN; ++p) ap[p][i] = *(const u16x8*)(sA0 + p * BM * LDB16 + off);
        }
        // smallest terms first: lo.hi, hi.lo, hi.hi (LPN = 2), term-major
        constexpr int NTERM = LPN == 2 ? 3 : 1;
        constexpr int TA[3] = {1, 0, 0}, TBp[3] = {0, 1, 0};
#pragma unroll
        for (int t = 0; t < NTERM; ++t)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const int ta = NTERM == 1 ? 0 : TA[t], tb = NTERM == 1 ? 0 : TBp[t];
              if constexpr (LPH)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                    __builtin_bit_cast(f16x8_t, ap[ta][i]), __builtin_bit_cast(f16x8_t, bp[tb][j]),
                    acc[i][j], 0, 0, 0);
              else
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    __builtin_bit_cast(bf16x8_t, ap[ta][i]), __builtin_bit_cast(bf16x8_t, bp[tb][j]),
                    acc[i][j], 0, 0, 0);
            }
      }
    } else if constexpr (X6 || SWZ) {
      const uint16_t* sA0 = (const uint16_t*)cur;
      const uint16_t* sB0 = sA0 + 3 * BM * LDB16;
#pragma unroll
      for (int kk = 0; kk < TK / 16; ++kk) {
        bf16x8_t bp[3][NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = brow0 + j * 32 + lr;
          const int off = row * LDB16 + (SWZ ? x6f_off(row, kk * 16 + lh * 8) : kk * 16 + lh * 8);
#pragma unroll
          for (int p = 0; p < 3; ++p) bp[p][j] = *(const bf16x8_t*)(sB0 + p * BN * LDB16 + off);
        }
        bf16x8_t ap[3][MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int row = arow0 + i * 32 + lr;
          const int off = row * LDB16 + (SWZ ? x6f_off(row, kk * 16 + lh * 8) : kk * 16 + lh * 8);
#pragma unroll
          for (int p = 0; p < 3; ++p) ap[p][i] = *(const bf16x8_t*)(sA0 + p * BM * LDB16 + off);
        }
        // smallest terms first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi;
        // term-major over the MI x NJ accumulators: consecutive MFMAs are
        // independent (a dependent chain waits out each MFMA's latency).  Per
        // accumulator the order is unchanged.
        constexpr int TA[6] = {2, 0, 1, 1, 0, 0}, TB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[TA[t]][i], bp[TB[t]][j],
                                                                  acc[i][j], 0, 0, 0);
      }
    } else {
      // Fragments are read 8 bytes at a time: lane half lh covers k in
      // [16 lh, 16 lh + 16), pair m feeds two MFMAs (k = 16 lh + 2m and +1).
      // Rows with bit 4 set hold each 16-byte chunk with its halves swapped
      // (store above), so lanes lr and lr + 16 -- same bank with the 36-float
      // row stride -- read disjoint banks: conflict-free ds_read_b64 (the
      // one-float-per-lane reads of the plain k mapping were 4-way conflicted,
      // SQ_LDS_BANK_CONFLICT = 66 % of LDS cycles, profiles/README.md)
      const float* sA = (const float*)cur;
      const float* sB = sA + BM * LDF32;
      const int swz = (lr & 16) >> 3;
#pragma unroll
      for (int m = 0; m < TK / 4; ++m) {
        const int kof = (16 * lh + 2 * m) ^ swz;
        fx2 b[NJ], a[MI];
#pragma unroll
        for (int j = 0; j < NJ; ++j) b[j] = *(const fx2*)(sB + (brow0 + j * 32 + lr) * LDF32 + kof);
#pragma unroll
        for (int i = 0; i < MI; ++i) a[i] = *(const fx2*)(sA + (arow0 + i * 32 + lr) * LDF32 + kof);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
      }
    }
  };
  load(0, S0_());
  if constexpr (DBUF) {
    store(smem, S0_());
    __syncthreads();
    for (int ks = 0; ks < ksteps; ++ks) {
      const unsigned char* cur = smem + (ks & 1) * LDS_BYTES;
      // the idle image was last read in iteration ks-1, before its barrier
      unsigned char* nxt = (ks + 1 < ksteps) ? smem + ((ks + 1) & 1) * LDS_BYTES : nullptr;
      if (ks + 1 < ksteps) load((ks + 1) * TK, S0_());   // global loads in flight under the MFMAs
      mma(cur, nullptr);
      if (nxt != nullptr) store(nxt, S0_());
      __syncthreads();
    }
  } else {
    // two k-steps of global loads in flight: set (ks & 1) is stored while
    // the other set's loads are still arriving, so a k-step's loads have two
    // k-steps of MFMAs to land (one k-step, ~1.3 us, did not cover an L2
    // miss: SQ_WAIT_INST_ANY 47 % of wave cycles, profiles/r4_pmc_pgemm_*)
    // The loads are issued unconditionally (past the last k-step they
    // re-read k-step 0): the same number of loads on every path lets the
    // compiler wait vmcnt(8) for one set instead of vmcnt(0) for both.
    auto kclamp = [&](int k) { return k < ksteps ? k * TK : 0; };
    load(kclamp(1), S1_());
    for (int ks = 0; ks < ksteps; ks += 2) {
      store(smem, S0_());
      __syncthreads();
      load(kclamp(ks + 2), S0_());
      mma(smem, nullptr);
      __syncthreads();
      if (ks + 1 >= ksteps) break;
      store(smem, S1_());
      __syncthreads();
      load(kclamp(ks + 3), S1_());
      mma(smem, nullptr);
      __syncthreads();
    }
  }

  // ---- epilogue (C/D map of 32x32 MFMA: row = (r&3) + 8*(r>>2) + 4*lh, col = lr).
  // Per 32x32 block: the 16 auxiliary operands (D, damping vectors, Grad for
  // the KL dot, old C) are loaded branch-free first, then stored predicated.
  const int epi = P.epi;
  AS1 float* const Cf = (AS1 float*)P.c_hi;
  AS1 uint16_t* const Ch = (AS1 uint16_t*)P.c_hi;
  AS1 uint16_t* const Cl = (AS1 uint16_t*)P.c_lo;
  AS1 uint16_t* const C2 = Cl + (Cl - Ch);        // X6 third plane
  const AS1 float* const Dm = gptr(P.dmat);
  const AS1 float* const Vm = gptr(P.vm);
  const AS1 float* const Vn = gptr(P.vn);
  const AS1 float* const Gf = (const AS1 float*)P.g_hi;
  const AS1 uint16_t* const Gh = (const AS1 uint16_t*)P.g_hi;
  const AS1 uint16_t* const Gl = (const AS1 uint16_t*)P.g_lo;
  const AS1 uint16_t* const G2 = Gl + (Gl - Gh);
  // 32-bit element offsets (every operand < 2^32 elements, checked on the
  // host): one offset VGPR per access instead of a 64-bit address pair keeps
  // the epilogue from setting the kernel's register budget
  const unsigned ldc = (unsigned)P.ldc, ldd = (unsigned)P.ldd, ldg = (unsigned)P.ldg;
  const float damping = P.damping;
  float kl_part = 0.f;
  // LP fp16: C = acc 2^-(LP_QEXP + lp_e) (exact: a power of two)
  const float lp_unscale = (LP && LPH) ? (F3F ? pow2f(-(P.ea + P.eb)) : pow2f(-(LP_QEXP + lp_e)))
                                       : 1.f;
  float lp_max = 0.f;                             // max |stored C| (next stage's scale)
  // one straight-line loop nest per epilogue kind (a run-time kind test per
  // element would split the loads into basic blocks with a wait each)
  auto run = [&](auto kind) {
    constexpr int E = decltype(kind)::value;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + brow0 + j * 32 + lr;
        float aux[16], aux2[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + arow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const bool ok = m < M && n < N;
          aux[r] = 0.f;
          aux2[r] = 0.f;
          if constexpr (E == EPI_HADAMARD) {
            aux[r] = gld_if32(Dm, (unsigned)m * ldd + n, ok, 0.f);
          } else if constexpr (E == EPI_HADAMARD_VEC) {
            aux[r] = gld_if32(Vm, (unsigned)m, ok, 0.f);
            aux2[r] = gld_if32(Vn, (unsigned)n, ok, 0.f);
          } else if constexpr (E == EPI_FINAL) {
            const unsigned go = (unsigned)n * ldg + m;
            if constexpr (X3) {
              aux[r] = bf16_bits_to_f32(gld_if32(Gh, go, ok, (uint16_t)0));
              aux2[r] = bf16_bits_to_f32(gld_if32(Gl, go, ok, (uint16_t)0));
            } else if constexpr (X6) {
              aux[r] = bf16_bits_to_f32(gld_if32(Gh, go, ok, (uint16_t)0));
              aux2[r] = bf16_bits_to_f32(gld_if32(Gl, go, ok, (uint16_t)0)) +
                        bf16_bits_to_f32(gld_if32(G2, go, ok, (uint16_t)0));
            } else {
              aux[r] = gld_if32(Gf, go, ok, 0.f);
            }
          } else if constexpr (E == EPI_SUB) {
            aux[r] = gld_if32((const AS1 float*)Cf, (unsigned)m * ldc + n, ok, 0.f);
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + arow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m >= M || n >= N) continue;
          float v = acc[i][j][r];
          if constexpr (LP && LPH) v *= lp_unscale;
          const unsigned o = (unsigned)m * ldc + n;
          if constexpr (E == EPI_HADAMARD) v *= aux[r];
          if constexpr (E == EPI_HADAMARD_VEC) v /= (aux2[r] * aux[r] + damping);
          if constexpr (LP) lp_max = fmaxf(lp_max, fabsf(v));
          if constexpr (E == EPI_FINAL) {
            Cf[o] = v;
            kl_part += v * (aux[r] + aux2[r]);
          } else if constexpr (E == EPI_SUB) {
            Cf[o] = aux[r] - v;
          } else if constexpr (E == EPI_ATOMIC) {
            atomicAdd((float*)P.c_hi + o, v);
          } else if constexpr (X3) {
            uint16_t h, l;
            split_bf16(v, h, l);
            Ch[o] = h;
            Cl[o] = l;
          } else if constexpr (X6) {
            uint16_t h, m1, l;
            split_bf16_3(v, h, m1, l);
            Ch[o] = h;
            Cl[o] = m1;
            C2[o] = l;
          } else {
            Cf[o] = v;
          }
        }
      }
  };
  switch (epi) {
    case EPI_HADAMARD: run(std::integral_constant<int, EPI_HADAMARD>()); break;
    case EPI_HADAMARD_VEC: run(std::integral_constant<int, EPI_HADAMARD_VEC>()); break;
    case EPI_FINAL: run(std::integral_constant<int, EPI_FINAL>()); break;
    case EPI_SUB: run(std::integral_constant<int, EPI_SUB>()); break;
    case EPI_ATOMIC: run(std::integral_constant<int, EPI_ATOMIC>()); break;
    default: run(std::integral_constant<int, EPI_STORE>()); break;
  }
  if constexpr (LP) {
    // the next stage's scale: max |C| of this problem (one atomic per wave;
    // max is order-independent: deterministic); and the slot this stage frees
    if (P.sc_out != nullptr) {           // uniform: one atomic per workgroup
      float m = lp_max;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      float* lpm = (float*)(smem + 64);    // past the KL partials' slots
      if (lane == 0) lpm[wave] = m;
      __syncthreads();
      if (threadIdx.x == 0) {
        float mm = 0.f;
        for (int w = 0; w < WM * WN; ++w) mm = fmaxf(mm, lpm[w]);
        if (mm > 0.f) atomicMax(P.sc_out, __float_as_uint(mm));
      }
    }
    if (P.sc_zero != nullptr && local == 0 && threadIdx.x == 0) *P.sc_zero = 0u;
  }
  if (kl != nullptr) {
    // one f64 partial per workgroup (waves summed in order, LDS is free after
    // the k-loop's last barrier); kfac_kl_finalize adds the slots in a fixed
    // order: deterministic, no atomics
    double* red = (double*)smem;
    const double d = wave_reduce_sum_d(P.epi == EPI_FINAL ? (double)kl_part : 0.0);
    if (lane == 0) red[wave] = d;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int w = 0; w < WM * WN; ++w) s += red[w];
      kl[blockIdx.x] = s;
    }
  }
}

// ---------------------------------------------------------------- gather
// Gct[a][g] (planes or fp32, leading dim ldo) <- K-FAC gradient matrix of a
// layer: column a = (c, i, j) of the weight grad in ANY memory layout
// (element g*s0 + c*s1 + i*s2 + j*s3), the bias (if any) as column nA-1.
struct GatherJob {
  const void* w; const void* bias;
  long long s0, s1, s2, s3;
  void* o_hi; void* o_lo; long long ldo;
  int nG, nA, kk, kw, wdtype, bdtype;
  int tile_begin, tiles_g;
  // low-plane modes: max |Gct| bits (atomicMax) and the 3 slots of the
  // chain's intermediates, zeroed for this step (either may be null)
  unsigned* amax; unsigned* zero3;
};

__device__ __forceinline__ float load_any(const void* p, long long i, int dt) {
  if (dt == KDT_F32) return ((const float*)p)[i];
  if (dt == KDT_BF16) return bf16_bits_to_f32(((const uint16_t*)p)[i]);
  return f16_bits_to_f32(((const uint16_t*)p)[i]);
}

// The job table lives in an immutable, content-addressed device copy
// (csrc/devtable.h): a graph-captured launch and an eager one never share a
// mutable table (with zero_grad(set_to_none=True) every eager step allocates
// new gradients while the captured graph keeps its own), and no ~4 KB table
// travels as a by-value kernel argument (corrupted in hipGraph replays).
constexpr int MAX_GATHER = 32;   // 32 x 120 B: the batch stays under the 4 KB kernel-argument limit
struct GatherBatch {
  int count, pad[3];
  GatherJob job[MAX_GATHER];
};
static_assert(sizeof(GatherBatch) <= 4096, "kernel arguments are limited to 4 KB");

template <int PREC>
__global__ __launch_bounds__(256) void gather_grad_kernel(const GatherBatch* __restrict__ batch) {
  const GatherJob* jobs = batch->job;
  const int count = batch->count;
  __shared__ float tile[64][65];
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile_begin <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const GatherJob& J = jobs[lo];
  const int local = blockIdx.x - J.tile_begin;
  const int ta = local / J.tiles_g, tg = local - ta * J.tiles_g;
  const int a0 = ta * 64, g0 = tg * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  const int wcols = J.nA - (J.bias ? 1 : 0);
  if (J.zero3 != nullptr && local == 0 && threadIdx.x < 3) J.zero3[threadIdx.x] = 0u;
  float vmax = 0.f;
  // read: lanes walk a (column), rows g
  for (int r = ty; r < 64; r += 4) {
    const int g = g0 + r, a = a0 + tx;
    float v = 0.f;
    if (g < J.nG && a < J.nA) {
      if (a < wcols) {
        const int c = a / J.kk, rem = a - c * J.kk, i = rem / J.kw, j = rem - i * J.kw;
        v = load_any(J.w, (long long)g * J.s0 + (long long)c * J.s1 + (long long)i * J.s2 +
                              (long long)j * J.s3, J.wdtype);
      } else {
        v = load_any(J.bias, g, J.bdtype);
      }
    }
    tile[r][tx] = v;
    vmax = fmaxf(vmax, fabsf(v));
  }
  __shared__ float wmax[4];
  if (J.amax != nullptr) {     // one atomic per workgroup (all of a layer's hit one word)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = vmax;
  }
  __syncthreads();
  if (J.amax != nullptr && threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    if (m > 0.f) atomicMax(J.amax, __float_as_uint(m));
  }
  // write Gct[a][g]: lanes walk g
  for (int r = ty; r < 64; r += 4) {
    const int a = a0 + r, g = g0 + tx;
    if (a >= J.nA || g >= J.nG) continue;
    const float v = tile[tx][r];
    store_planes<PREC>(J.o_hi, J.o_lo, (long long)a * J.ldo + g, v);
  }
}

// ---------------------------------------------------------------- split
// dst[r][c] (planes or fp32, ld ldo) <- src[r][c] (fp32, ld lds), or the
// transpose dst[c][r] <- src[r][c] when `trans`.  rows x cols of src.
template <int PREC>
__global__ __launch_bounds__(256) void split_copy_kernel(const SplitJob* __restrict__ jobs,
                                                         int count) {
  __shared__ float tile[64][65];
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile_begin <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const SplitJob& J = jobs[lo];
  const int local = blockIdx.x - J.tile_begin;
  const int tr = local / J.tiles_c, tc = local - tr * J.tiles_c;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int gr = r0 + r, gc = c0 + tx;
    tile[r][tx] = (gr < J.rows && gc < J.cols) ? J.src[(long long)gr * J.lds + gc] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    int orow, ocol;
    float v;
    if (J.trans) { orow = c0 + r; ocol = r0 + tx; v = tile[tx][r]; if (orow >= J.cols || ocol >= J.rows) continue; }
    else { orow = r0 + r; ocol = c0 + tx; v = tile[r][tx]; if (orow >= J.rows || ocol >= J.cols) continue; }
    store_planes<PREC>(J.o_hi, J.o_lo, (long long)orow * J.ldo + ocol, v);
  }
}

}  // namespace

// ------------------------------------------------------------------ C ABI
// Host record layouts mirror the device structs (ops/_lib.py).
KFAC_API int kfac_pgemm_record_size() { return (int)sizeof(PGemm); }
KFAC_API int kfac_gather_record_size() { return (int)sizeof(GatherJob); }
KFAC_API int kfac_split_record_size() { return (int)sizeof(SplitJob); }

// tile: 0 = 128 x 128 (4 waves, registers capped for 2 waves per SIMD: 2.83 vs
// 3.03 ms fp32 chain, 1.49 vs 1.56 ms bf16x3 against the uncapped 272-register
// build = tile 8, profiles/r2_pgemm_occupancy.log), 1 = 256 x 256 (8 waves),
// 2 = 64 x 64 (4 waves), 3 = 128 x 128 (8 waves), 4 = 128 x 64 (4 waves);
// the table (ops/precond_fused.py) holds the problems of that tile class.
// XCD-grouped tile order for the default bf16x6 tile (ResNet-50 chain 2.023 ->
// 2.002 ms, profiles/r4_pgemm_xcd.log); KFAC_PGEMM_XCD=0 restores row-major
static const bool g_pgemm_xcd = [] {
  const char* e = getenv("KFAC_PGEMM_XCD");
  return !(e && e[0] == '0');
}();

KFAC_API int kfac_pgemm(int prec, int tile, const void* dev_table, int count, int total_tiles,
                        double* kl, hipStream_t stream) {
  if (count <= 0 || total_tiles <= 0) return 0;
  const PGemm* t = (const PGemm*)dev_table;
  dim3 g(total_tiles);
#define KFAC_PGEMM_LAUNCH(P)                                                                          \
  switch (tile) {                                                                                     \
    case 1: hipLaunchKernelGGL((pgemm_kernel<P, 256, 256, 2, 4>), g, dim3(512), 0, stream, t, count, kl); break; \
    case 2: hipLaunchKernelGGL((pgemm_kernel<P, 64, 64, 2, 2>), g, dim3(256), 0, stream, t, count, kl); break;   \
    case 3: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 4, 2>), g, dim3(512), 0, stream, t, count, kl); break; \
    case 4: hipLaunchKernelGGL((pgemm_kernel<P, 128, 64, 2, 2>), g, dim3(256), 0, stream, t, count, kl); break;  \
    case 5: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 4, 4>), g, dim3(1024), 0, stream, t, count, kl); break; \
    case 6: hipLaunchKernelGGL((pgemm_kernel<P, 256, 128, 4, 2>), g, dim3(512), 0, stream, t, count, kl); break; \
    case 7: hipLaunchKernelGGL((pgemm_kernel<P, 128, 256, 2, 4>), g, dim3(512), 0, stream, t, count, kl); break; \
    case 8: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 2, 2, 1>), g, dim3(256), 0, stream, t, count, kl); break; \
    case 9: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 2, 2, 2, true>), g, dim3(256), 0, stream, t, count, kl); break; \
    case 10: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 4, 2, 1, true>), g, dim3(512), 0, stream, t, count, kl); break; \
    case 11: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 4, 4, 1, true>), g, dim3(1024), 0, stream, t, count, kl); break; \
    default: hipLaunchKernelGGL((pgemm_kernel<P, 128, 128, 2, 2, 2>), g, dim3(256), 0, stream, t, count, kl); break; \
  }
  if (prec == PREC_BF16X3) {
    KFAC_PGEMM_LAUNCH(PREC_BF16X3)
  } else if (prec == PREC_BF16X6) {
    // default tile only (the 3-plane image is 60 KB of LDS per workgroup)
    hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6, 128, 128, 2, 2, 2>), g, dim3(256), 0, stream, t,
                       count, kl);
  } else if (prec == PREC_BF16X6F) {
    // bigger tiles for problems with M, N >= 256: less operand traffic per
    // FLOP (the chain reads its operands at ~5 TB/s from L2 / MALL)
    if (tile == 1)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 256, 256, 2, 4>), g, dim3(512), 0, stream, t,
                         count, kl);
    else if (tile == 6)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 256, 128, 4, 2>), g, dim3(512), 0, stream, t,
                         count, kl);
    else if (tile == 7)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 128, 256, 2, 4>), g, dim3(512), 0, stream, t,
                         count, kl);
    else if (tile == 9)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 128, 128, 2, 2, 2, true>), g, dim3(256), 0,
                         stream, t, count, kl);
    else if (tile == 8)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 128, 128, 2, 2, 1>), g, dim3(256), 0, stream,
                         t, count, kl);
    else if (g_pgemm_xcd)
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 128, 128, 2, 2, 2, false, true>), g, dim3(256),
                         0, stream, t, count, kl);
    else
      hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6F, 128, 128, 2, 2, 2>), g, dim3(256), 0, stream,
                         t, count, kl);
  } else if (prec == PREC_BF16X6A) {
    hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6A, 128, 128, 2, 2, 2, false, true>), g, dim3(256),
                       0, stream, t, count, kl);
  } else if (prec == PREC_BF16X6B) {
    hipLaunchKernelGGL((pgemm_kernel<PREC_BF16X6B, 128, 128, 2, 2, 2, false, true>), g, dim3(256),
                       0, stream, t, count, kl);
  } else if (prec == PREC_F16X3F) {
    if (g_pgemm_xcd)
      hipLaunchKernelGGL((pgemm_kernel<PREC_F16X3F, 128, 128, 2, 2, 2, false, true>), g, dim3(256),
                         0, stream, t, count, kl);
    else
      hipLaunchKernelGGL((pgemm_kernel<PREC_F16X3F, 128, 128, 2, 2, 2>), g, dim3(256), 0, stream,
                         t, count, kl);
  } else if (prec >= PREC_F16X3A && prec <= PREC_F1B) {
    // tile 6 / 7: 256 x 128 / 128 x 256 with 8 waves (fewer operand bytes per
    // product for problems with a dimension >= 256), else 128 x 128
#define KFAC_LP(P_)                                                                              \
  do {                                                                                           \
    if (tile == 6)                                                                               \
      hipLaunchKernelGGL((pgemm_kernel<P_, 256, 128, 4, 2, 2, false, true>), g, dim3(512), 0,     \
                         stream, t, count, kl);                                                  \
    else if (tile == 7)                                                                          \
      hipLaunchKernelGGL((pgemm_kernel<P_, 128, 256, 2, 4, 2, false, true>), g, dim3(512), 0,     \
                         stream, t, count, kl);                                                  \
    else                                                                                         \
      hipLaunchKernelGGL((pgemm_kernel<P_, 128, 128, 2, 2, 2, false, true>), g, dim3(256), 0,     \
                         stream, t, count, kl);                                                  \
  } while (0)
    switch (prec) {
      case PREC_F16X3A: KFAC_LP(PREC_F16X3A); break;
      case PREC_F16X3B: KFAC_LP(PREC_F16X3B); break;
      case PREC_H1A: KFAC_LP(PREC_H1A); break;
      case PREC_H1B: KFAC_LP(PREC_H1B); break;
      case PREC_F1A: KFAC_LP(PREC_F1A); break;
      default: KFAC_LP(PREC_F1B); break;
    }
#undef KFAC_LP
  } else if (prec == PREC_F32) {
    KFAC_PGEMM_LAUNCH(PREC_F32)
  } else {
    return -1;
  }
#undef KFAC_PGEMM_LAUNCH
  return (int)hipGetLastError();
}

// host_jobs: `count` GatherJob records (tile_begin/tiles_g filled in here).
KFAC_API int kfac_gather_grad(int prec, const void* host_jobs, int count, hipStream_t stream) {
  const GatherJob* t = (const GatherJob*)host_jobs;
  for (int base = 0; base < count; base += MAX_GATHER) {
    GatherBatch b;
    memset(&b, 0, sizeof(b));   // deterministic table bytes (devtable key)
    b.count = count - base < MAX_GATHER ? count - base : MAX_GATHER;
    int tiles = 0;
    for (int k = 0; k < b.count; ++k) {
      b.job[k] = t[base + k];
      b.job[k].tiles_g = (b.job[k].nG + 63) / 64;
      b.job[k].tile_begin = tiles;
      tiles += ((b.job[k].nA + 63) / 64) * b.job[k].tiles_g;
    }
    if (tiles == 0) continue;
    int terr = 0;
    const GatherBatch* d = (const GatherBatch*)kfac_devtable::get(&b, sizeof(b), stream, &terr);
    if (!d) return terr;
    if (prec == PREC_BF16X3)
      hipLaunchKernelGGL(gather_grad_kernel<PREC_BF16X3>, dim3(tiles), dim3(256), 0, stream, d);
    else if (prec == PREC_BF16X6)
      hipLaunchKernelGGL(gather_grad_kernel<PREC_BF16X6>, dim3(tiles), dim3(256), 0, stream, d);
    else
      hipLaunchKernelGGL(gather_grad_kernel<PREC_F32>, dim3(tiles), dim3(256), 0, stream, d);
    int err = (int)hipGetLastError();
    if (err) return err;
  }
  return 0;
}

KFAC_API int kfac_split_copy(int prec, const void* dev_jobs, int count, int total_tiles,
                             hipStream_t stream) {
  if (count <= 0 || total_tiles <= 0) return 0;
  const SplitJob* j = (const SplitJob*)dev_jobs;
  if (prec == PREC_BF16X3)
    hipLaunchKernelGGL(split_copy_kernel<PREC_BF16X3>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else if (prec == STORE_F16X2)
    hipLaunchKernelGGL(split_copy_kernel<STORE_F16X2>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else if (prec == STORE_BF16X1)
    hipLaunchKernelGGL(split_copy_kernel<STORE_BF16X1>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else if (prec == STORE_F16X1)
    hipLaunchKernelGGL(split_copy_kernel<STORE_F16X1>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else if (prec == PREC_BF16X6)
    hipLaunchKernelGGL(split_copy_kernel<PREC_BF16X6>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else
    hipLaunchKernelGGL(split_copy_kernel<PREC_F32>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  return (int)hipGetLastError();
}
