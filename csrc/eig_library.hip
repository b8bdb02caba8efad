// Tridiagonal-path eigensolver plumbing for large K-FAC factors.
//
// Large factors (n > the LDS Jacobi limit) are solved by size class: every
// factor of one n that the rank owns is stacked into ONE strided batch and
// handed to rocSOLVER's divide-and-conquer driver (sytrd + stedc + ormtr) in
// a single call, so the per-column panel latency of the tridiagonal reduction
// (the dominant cost at these sizes: profiles/r1_rocsolver_variants.log) is
// paid once per class instead of once per factor.  A rocblas handle is cached
// per HIP stream; callers drive several classes concurrently on different
// streams (ops/eigen.py).
//
// Reference semantics: kfac/layers/utils.py:45-74 (symeig, ascending
// eigenvalues); the row-major <-> column-major flip is harmless for the
// symmetric input and handled for the eigenvectors on the Python side.
#include "common.h"

#include <map>
#include <mutex>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

namespace {

std::mutex g_handle_mu;
std::map<hipStream_t, rocblas_handle> g_handles;

rocblas_handle handle_for(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_handle_mu);
  auto it = g_handles.find(stream);
  if (it != g_handles.end()) return it->second;
  rocblas_handle h = nullptr;
  if (rocblas_create_handle(&h) != rocblas_status_success) return nullptr;
  rocblas_set_stream(h, stream);
  g_handles[stream] = h;
  return h;
}

}  // namespace

// A: batch x n x n (symmetric, overwritten by eigenvectors: column-major
// eigenvector k = row k of the row-major view), D: batch x n eigenvalues
// (ascending), E: batch x n scratch, info: batch ints (device).
KFAC_API int kfac_syevd_batched(float* A, int n, int batch, float* D, float* E, int* info,
                                hipStream_t stream) {
  rocblas_handle h = handle_for(stream);
  if (!h) return -2;
  const rocblas_stride nn = (rocblas_stride)n * n;
  rocblas_status st;
  if (batch == 1)
    st = rocsolver_ssyevd(h, rocblas_evect_original, rocblas_fill_upper, n, A, n, D, E, info);
  else
    st = rocsolver_ssyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, n, A, n,
                                          nn, D, n, E, n, info, batch);
  return st == rocblas_status_success ? 0 : 1000 + (int)st;
}

// Tridiagonal divide and conquer only (for the hand-written reduction path):
// D (n) diagonal, E (n) off-diagonal, C (n x n, column-major) receives the
// eigenvectors of the tridiagonal matrix.
KFAC_API int kfac_stedc(float* D, float* E, float* C, int n, int* info, hipStream_t stream) {
  rocblas_handle h = handle_for(stream);
  if (!h) return -2;
  rocblas_status st = rocsolver_sstedc(h, rocblas_evect_tridiagonal, n, D, E, C, n, info);
  return st == rocblas_status_success ? 0 : 1000 + (int)st;
}

// Householder tridiagonalisation only (strided batch, lower/upper per `lower`):
// d, e (batch x n), tau (batch x n).  Pure kernel launches: capturable.
KFAC_API int kfac_sytrd_batched(float* A, int n, int batch, float* D, float* E, float* tau,
                                int lower, hipStream_t stream) {
  rocblas_handle h = handle_for(stream);
  if (!h) return -2;
  const rocblas_stride nn = (rocblas_stride)n * n;
  rocblas_status st = rocsolver_ssytrd_strided_batched(
      h, lower ? rocblas_fill_lower : rocblas_fill_upper, n, A, n, nn, D, n, E, n, tau, n, batch);
  return st == rocblas_status_success ? 0 : 1000 + (int)st;
}

// C <- Q C with Q from kfac_sytrd_batched (single matrix).
KFAC_API int kfac_ormtr(float* A, float* tau, float* C, int n, int lower, hipStream_t stream) {
  rocblas_handle h = handle_for(stream);
  if (!h) return -2;
  rocblas_status st = rocsolver_sormtr(h, rocblas_side_left,
                                       lower ? rocblas_fill_lower : rocblas_fill_upper,
                                       rocblas_operation_none, n, n, A, n, tau, C, n);
  return st == rocblas_status_success ? 0 : 1000 + (int)st;
}
