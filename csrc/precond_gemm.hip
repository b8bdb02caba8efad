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
// of 32 by construction (ops/precond_fused.py), so the k-loop is unmasked.
//
// Precision modes:
//   PREC_BF16X3  operands stored as bf16 (hi, lo) planes (x ~= hi + lo), three
//                v_mfma_f32_32x32x16_bf16 per product (hi*hi + hi*lo + lo*hi),
//                f32 accumulation: ~1e-5 relative error on the preconditioned
//                gradient (fp32 GEMMs: ~1e-6, plain bf16: ~5e-3), at ~5x the
//                f32 MFMA rate.
//   PREC_F32     operands fp32, exact v_mfma_f32_32x32x2_f32 (bitwise an fmaf
//                chain), the reference's fp32 semantics.
// Auxiliary launches: `gather_grad` builds Gct planes from the .grad tensors
// (any memory layout, bias as the last K-FAC column), `split_copy` builds the
// QA/QG/QAt/QGt planes and Dt after each inverse update.
#include "common.h"

namespace {

enum { PREC_F32 = 0, PREC_BF16X3 = 1 };
enum { EPI_STORE = 0, EPI_HADAMARD = 1, EPI_HADAMARD_VEC = 2, EPI_FINAL = 3 };

constexpr int TM = 128, TN = 128, TK = 32;
constexpr int LDB16 = TK + 8;   // 80-byte rows: conflict-free ds_read_b128 (guide: LDS banking)
constexpr int LDF32 = TK + 4;   // 144-byte rows, 16-byte aligned chunk writes

struct PGemm {
  const void* a_hi; const void* a_lo; long long lda;
  const void* b_hi; const void* b_lo; long long ldb;
  void* c_hi; void* c_lo; long long ldc;
  // EPI_HADAMARD: C *= dmat[m*ldd + n]; EPI_HADAMARD_VEC: C /= (vn[n]*vm[m] + damping)
  const float* dmat; long long ldd;
  const float* vm; const float* vn; float damping;
  // EPI_FINAL: KL dot partner Grad[m][n] = g_hi/g_lo planes of Gct at [n*ldg + m]
  const void* g_hi; const void* g_lo; long long ldg;
  int M, N, K, epi;
  int tile_begin, tiles_n;
};

__device__ __forceinline__ int find_problem(const PGemm* __restrict__ t, int count, int blk) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].tile_begin <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void split_bf16(float x, uint16_t& h, uint16_t& l) {
  h = f32_to_bf16_bits(x);
  l = f32_to_bf16_bits(x - bf16_bits_to_f32(h));
}

template <int PREC>
__global__ __launch_bounds__(256) void pgemm_kernel(const PGemm* __restrict__ table, int count,
                                                    double* __restrict__ kl) {
  constexpr bool X3 = (PREC == PREC_BF16X3);
  // one LDS array (guide: a second __shared__ object can de-pipeline loads)
  constexpr int LDS_BYTES = X3 ? (4 * TM * LDB16 * 2) : (2 * TM * LDF32 * 4);
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int pi = find_problem(table, count, blockIdx.x);
  const PGemm& P = table[pi];
  const int local = blockIdx.x - P.tile_begin;
  const int tm = local / P.tiles_n, tn = local - tm * P.tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  const int M = P.M, N = P.N;
  const int ksteps = (P.K + TK - 1) / TK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- loader: 4 x 16 B per operand per thread per k-step
  // bf16 planes: chunk c in [0,1024): plane = c>>9, row = (c & 511) >> 2, kc = c & 3 (8 elems)
  // f32:         chunk c in [0,1024): row = c >> 3, kc = c & 7 (4 elems)
  uint4 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q;
      int row, kof, plane;
      if (X3) { plane = c >> 9; row = (c & 511) >> 2; kof = (c & 3) * 8; }
      else { plane = 0; row = c >> 3; kof = (c & 7) * 4; }
      const int esz = X3 ? 2 : 4;
      {
        const int gm = m0 + row;
        const unsigned char* base = (const unsigned char*)(plane ? P.a_lo : P.a_hi);
        ra[q] = (gm < M) ? *(const uint4*)(base + ((long long)gm * P.lda + k0 + kof) * esz)
                         : make_uint4(0, 0, 0, 0);
      }
      {
        const int gn = n0 + row;
        const unsigned char* base = (const unsigned char*)(plane ? P.b_lo : P.b_hi);
        rb[q] = (gn < N) ? *(const uint4*)(base + ((long long)gn * P.ldb + k0 + kof) * esz)
                         : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q;
      if (X3) {
        const int plane = c >> 9, row = (c & 511) >> 2, kof = (c & 3) * 8;
        uint16_t* sAp = (uint16_t*)smem + (plane * TM) * LDB16;            // A hi | A lo
        uint16_t* sBp = (uint16_t*)smem + (2 * TM + plane * TM) * LDB16;   // B hi | B lo
        *(uint4*)(sAp + row * LDB16 + kof) = ra[q];
        *(uint4*)(sBp + row * LDB16 + kof) = rb[q];
      } else {
        const int row = c >> 3, kof = (c & 7) * 4;
        float* sA = (float*)smem;
        float* sB = (float*)smem + TM * LDF32;
        *(uint4*)(sA + row * LDF32 + kof) = ra[q];
        *(uint4*)(sB + row * LDF32 + kof) = rb[q];
      }
    }
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load(0);
  for (int ks = 0; ks < ksteps; ++ks) {
    store();
    __syncthreads();
    if (ks + 1 < ksteps) load((ks + 1) * TK);
    if constexpr (X3) {
      const uint16_t* sAh = (const uint16_t*)smem;
      const uint16_t* sAl = sAh + TM * LDB16;
      const uint16_t* sBh = sAh + 2 * TM * LDB16;
      const uint16_t* sBl = sAh + 3 * TM * LDB16;
#pragma unroll
      for (int kk = 0; kk < TK / 16; ++kk) {
        bf16x8_t ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int off = (wr * 64 + i * 32 + lr) * LDB16 + kk * 16 + lh * 8;
          ah[i] = *(const bf16x8_t*)(sAh + off);
          al[i] = *(const bf16x8_t*)(sAl + off);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int off = (wc * 64 + j * 32 + lr) * LDB16 + kk * 16 + lh * 8;
          bh[j] = *(const bf16x8_t*)(sBh + off);
          bl[j] = *(const bf16x8_t*)(sBl + off);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
    } else {
      const float* sA = (const float*)smem;
      const float* sB = sA + TM * LDF32;
#pragma unroll
      for (int kk = 0; kk < TK / 2; ++kk) {
        float a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = sA[(wr * 64 + i * 32 + lr) * LDF32 + kk * 2 + lh];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = sB[(wc * 64 + j * 32 + lr) * LDF32 + kk * 2 + lh];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue (C/D map of 32x32 MFMA: row = (r&3) + 8*(r>>2) + 4*lh, col = lr)
  float kl_part = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int n = n0 + wc * 64 + j * 32 + lr;
        if (m >= M || n >= N) continue;
        float v = acc[i][j][r];
        if (P.epi == EPI_HADAMARD) v *= P.dmat[(long long)m * P.ldd + n];
        else if (P.epi == EPI_HADAMARD_VEC) v /= (P.vn[n] * P.vm[m] + P.damping);
        const long long o = (long long)m * P.ldc + n;
        if (P.epi == EPI_FINAL) {
          ((float*)P.c_hi)[o] = v;
          const long long go = (long long)n * P.ldg + m;
          float g;
          if (X3) g = bf16_bits_to_f32(((const uint16_t*)P.g_hi)[go]) +
                      bf16_bits_to_f32(((const uint16_t*)P.g_lo)[go]);
          else g = ((const float*)P.g_hi)[go];
          kl_part += v * g;
        } else if (X3) {
          uint16_t h, l;
          split_bf16(v, h, l);
          ((uint16_t*)P.c_hi)[o] = h;
          ((uint16_t*)P.c_lo)[o] = l;
        } else {
          ((float*)P.c_hi)[o] = v;
        }
      }
  if (P.epi == EPI_FINAL && kl != nullptr) {
    double d = wave_reduce_sum_d((double)kl_part);
    if (lane == 0) atomicAdd(kl, d);
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
};

__device__ __forceinline__ float load_any(const void* p, long long i, int dt) {
  if (dt == KDT_F32) return ((const float*)p)[i];
  if (dt == KDT_BF16) return bf16_bits_to_f32(((const uint16_t*)p)[i]);
  return f16_bits_to_f32(((const uint16_t*)p)[i]);
}

template <int PREC>
__global__ __launch_bounds__(256) void gather_grad_kernel(const GatherJob* __restrict__ jobs,
                                                          int count) {
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
  }
  __syncthreads();
  // write Gct[a][g]: lanes walk g
  for (int r = ty; r < 64; r += 4) {
    const int a = a0 + r, g = g0 + tx;
    if (a >= J.nA || g >= J.nG) continue;
    const float v = tile[tx][r];
    const long long o = (long long)a * J.ldo + g;
    if (PREC == PREC_BF16X3) {
      uint16_t h, l;
      split_bf16(v, h, l);
      ((uint16_t*)J.o_hi)[o] = h;
      ((uint16_t*)J.o_lo)[o] = l;
    } else {
      ((float*)J.o_hi)[o] = v;
    }
  }
}

// ---------------------------------------------------------------- split
// dst[r][c] (planes or fp32, ld ldo) <- src[r][c] (fp32, ld lds), or the
// transpose dst[c][r] <- src[r][c] when `trans`.  rows x cols of src.
struct SplitJob {
  const float* src; long long lds;
  void* o_hi; void* o_lo; long long ldo;
  int rows, cols, trans, tile_begin, tiles_c;
};

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
    const long long o = (long long)orow * J.ldo + ocol;
    if (PREC == PREC_BF16X3) {
      uint16_t h, l;
      split_bf16(v, h, l);
      ((uint16_t*)J.o_hi)[o] = h;
      ((uint16_t*)J.o_lo)[o] = l;
    } else {
      ((float*)J.o_hi)[o] = v;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------ C ABI
// Host record layouts mirror the device structs (ops/_lib.py).
KFAC_API int kfac_pgemm_record_size() { return (int)sizeof(PGemm); }
KFAC_API int kfac_gather_record_size() { return (int)sizeof(GatherJob); }
KFAC_API int kfac_split_record_size() { return (int)sizeof(SplitJob); }

KFAC_API int kfac_pgemm(int prec, const void* dev_table, int count, int total_tiles, double* kl,
                        hipStream_t stream) {
  if (count <= 0 || total_tiles <= 0) return 0;
  const PGemm* t = (const PGemm*)dev_table;
  if (prec == PREC_BF16X3)
    hipLaunchKernelGGL(pgemm_kernel<PREC_BF16X3>, dim3(total_tiles), dim3(256), 0, stream, t, count, kl);
  else if (prec == PREC_F32)
    hipLaunchKernelGGL(pgemm_kernel<PREC_F32>, dim3(total_tiles), dim3(256), 0, stream, t, count, kl);
  else
    return -1;
  return (int)hipGetLastError();
}

KFAC_API int kfac_gather_grad(int prec, const void* dev_jobs, int count, int total_tiles,
                              hipStream_t stream) {
  if (count <= 0 || total_tiles <= 0) return 0;
  const GatherJob* j = (const GatherJob*)dev_jobs;
  if (prec == PREC_BF16X3)
    hipLaunchKernelGGL(gather_grad_kernel<PREC_BF16X3>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else
    hipLaunchKernelGGL(gather_grad_kernel<PREC_F32>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  return (int)hipGetLastError();
}

KFAC_API int kfac_split_copy(int prec, const void* dev_jobs, int count, int total_tiles,
                             hipStream_t stream) {
  if (count <= 0 || total_tiles <= 0) return 0;
  const SplitJob* j = (const SplitJob*)dev_jobs;
  if (prec == PREC_BF16X3)
    hipLaunchKernelGGL(split_copy_kernel<PREC_BF16X3>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  else
    hipLaunchKernelGGL(split_copy_kernel<PREC_F32>, dim3(total_tiles), dim3(256), 0, stream, j, count);
  return (int)hipGetLastError();
}
