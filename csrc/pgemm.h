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
enum { PREC_F32 = 0, PREC_BF16X3 = 1, PREC_BF16X6 = 2, PREC_BF16X6F = 3, PREC_BF16X6A = 4,
       PREC_BF16X6B = 5 };
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
