// Grouped "NT" GEMM records shared by the preconditioning chain
// (csrc/precond_gemm.hip) and the eigensolver back-transformation
// (csrc/eig_backtransform.hip).  Host mirrors: ops/precond_fused.py (layout sizes
// are checked at load through kfac_*_record_size).
#pragma once
#include "common.h"

// PREC_BF16X6F: the bf16x6 products of PREC_BF16X6 on fp32 operands, split
// into the three planes while they are staged into LDS (4 B per element
// from memory instead of 6, no plane copies of the operands)
// (a register-split variant -- fp32 LDS image, planes split per MFMA
// fragment -- measured 2.55 vs 2.28 ms on ResNet-50: 2.3x the VALU work,
// profiles/r3_pgemm_mode_r.log; removed)
// PREC_BF16X6A / PREC_BF16X6B: the same products with ONE operand (A resp.
// B) stored as its three bf16 planes -- the eigenvector operands of the
// preconditioning chain, split once per inverse update -- and the other, the
// per-step operand, fp32 and split while it is staged: half the per-k-step
// split work of PREC_BF16X6F
// Low-plane mixed modes (one operand stored as 16-bit planes once per inverse
// update -- the eigenvector operand -- the other fp32, converted while staged):
// PREC_F16X3A / B: fp16 hi / lo planes, x' = x 2^e ~= hi + lo (22 significand
//   bits), three v_mfma_f32_32x32x16_f16 per product (lo.hi + hi.lo + hi.hi);
//   the eigenvector planes carry e = 14 (|q| <= 1), the fp32 operand e = 14 -
//   exponent(max |x|) from a per-problem max slot its producer filled
//   (atomicMax of |x| bits: deterministic), undone in the epilogue (exact).
// PREC_H1A / B, PREC_F1A / B: one bf16 / fp16 plane, one MFMA per product:
//   the reference's inv_dtype = bfloat16 / float16 preconditioning
//   (kfac/layers/base.py:435-441,463,470) on the grouped chain.
// PREC_F16X3F: both operands fp32, each split while staged into scaled fp16
//   hi / lo planes with a FIXED exponent from the record (ea, eb): for
//   products whose operands are bounded by construction -- the eigensolver's
//   orthogonal factors (|x| <= 1: e = 14).
enum { PREC_F32 = 0, PREC_BF16X3 = 1, PREC_BF16X6 = 2, PREC_BF16X6F = 3, PREC_BF16X6A = 4,
       PREC_BF16X6B = 5, PREC_F16X3A = 6, PREC_F16X3B = 7, PREC_H1A = 8, PREC_H1B = 9,
       PREC_F1A = 10, PREC_F1B = 11, PREC_F16X3F = 12 };
// split_copy / store_planes modes of the low-plane eigenvector operands
enum { STORE_F16X2 = 20, STORE_BF16X1 = 21, STORE_F16X1 = 22 };
constexpr int LP_QEXP = 14;      // scale exponent of the fp16 eigenvector planes
// EPI_SUB: C -= A B^T (f32); EPI_ATOMIC: C += A B^T with f32 atomics (split-K)
enum { EPI_STORE = 0, EPI_HADAMARD = 1, EPI_HADAMARD_VEC = 2, EPI_FINAL = 3, EPI_SUB = 4,
       EPI_ATOMIC = 5 };

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
  // low-plane modes: max |x| bits of the fp32 operand (read), of this stage's
  // output (atomicMax, when it feeds the next stage), a slot to zero (or null)
  const unsigned* sc_in; unsigned* sc_out; unsigned* sc_zero;
  int ea, eb;             // PREC_F16X3F: scale exponents of the A / B operands
};

// dst[r][c] (planes or fp32, ld ldo) <- src[r][c] (fp32, ld lds), or the
// transpose dst[c][r] <- src[r][c] when `trans`.  rows x cols of src.
struct SplitJob {
  const float* src; long long lds;
  void* o_hi; void* o_lo; long long ldo;
  int rows, cols, trans, tile_begin, tiles_c;
};

// C[m][n] = sum_k A[m][k] B[n][k] for every record of `dev_table` (device
// memory); operands k-contiguous and zero-padded along k to a multiple of 64.
KFAC_API int kfac_pgemm(int prec, int tile, const void* dev_table, int count, int total_tiles,
                        double* kl, hipStream_t stream);
// kl (pgemm): NULL, or this launch's per-workgroup f64 partial slots of the
// EPI_FINAL KL dot (total_tiles of them); kfac_kl_finalize sums slots in order.
KFAC_API int kfac_kl_finalize(const double* part, int n, double* out, hipStream_t stream);
KFAC_API int kfac_split_copy(int prec, const void* dev_jobs, int count, int total_tiles,
                             hipStream_t stream);
