// Batched symmetric eigensolver for small factors (n <= 192) on gfx950.
//
// One 256-thread workgroup per matrix runs cyclic parallel Jacobi with the
// round-robin (circle) ordering: each round rotates n/2 disjoint (p, q)
// pairs at once; a sweep is n-1 rounds; sweeps repeat until a whole sweep
// applies no rotation (|a_pq| <= tol * sqrt(|a_pp a_qq|)) or max_sweeps.
// The working matrix lives in LDS with an odd leading dimension (column
// phase: consecutive lanes walk rows -> distinct banks; row phase: lanes
// walk columns -> contiguous); the eigenvector accumulator V^T lives in a
// global scratch (rows p, q of V^T are contiguous, so the update coalesces).
//
// Output matches the reference's get_eigendecomp (kfac/layers/utils.py:45-74):
// ascending eigenvalues, eigenvalues clipped at `clip` when requested, Q
// row-major with eigenvector k in column k.  Dozens of small factors of a
// ResNet are solved by one launch instead of one library call each (the
// rocSOLVER call costs ~1.6 ms even at n = 64 on MI355X: profiles/r1_probe_baseline.json).
#include "common.h"

namespace {

constexpr int MAXJ = 64;
constexpr int NMAX = 192;

struct EigJob {
  const float* A;   // input n x n (row-major, symmetric)
  float* Q;         // output eigenvectors, n x n row-major, column k = eigenvector k
  float* d;         // output eigenvalues (n), ascending
  float* Vt;        // scratch n x n
  int n;
  int pad;
};

struct EigBatch {
  int count;
  int max_sweeps;
  float tol;
  int do_clip;
  float clip;
  EigJob job[MAXJ];
};

__global__ __launch_bounds__(256) void jacobi_small_kernel(EigBatch batch) {
  extern __shared__ float S[];
  __shared__ float rc[NMAX / 2], rs[NMAX / 2], rt[NMAX / 2], rpp[NMAX / 2], rqq[NMAX / 2],
      rpq[NMAX / 2];
  __shared__ int rp[NMAX / 2], rq[NMAX / 2];
  __shared__ int nrot;
  __shared__ float dsh[NMAX];

  const EigJob J = batch.job[blockIdx.x];
  const int n = J.n;
  const int ne = n + (n & 1);     // even size; a padded index is a decoupled zero row/col
  const int ld = ne + 1;
  const int npairs = ne / 2;
  const int tid = threadIdx.x;

  for (int e = tid; e < ne * ne; e += 256) {
    int i = e / ne, j = e - i * ne;
    S[i * ld + j] = (i < n && j < n) ? J.A[(long long)i * n + j] : 0.f;
  }
  for (int e = tid; e < n * n; e += 256) {
    int i = e / n, j = e - i * n;
    J.Vt[e] = (i == j) ? 1.f : 0.f;
  }
  __syncthreads();

  const int m = ne - 1;
  for (int sweep = 0; sweep < batch.max_sweeps; ++sweep) {
    if (tid == 0) nrot = 0;
    __syncthreads();
    for (int r = 0; r < m; ++r) {
      // --- rotation parameters for the npairs disjoint pairs of round r
      for (int k = tid; k < npairs; k += 256) {
        int a, b;
        if (k == 0) { a = m; b = r; }
        else { a = (r + k) % m; b = (r - k + m) % m; }
        int p = a < b ? a : b, q = a < b ? b : a;
        float app = S[p * ld + p], aqq = S[q * ld + q], apq = S[p * ld + q];
        float c = 1.f, s = 0.f, t = 0.f;
        if (apq != 0.f && fabsf(apq) > batch.tol * sqrtf(fabsf(app) * fabsf(aqq))) {
          float theta = (aqq - app) / (2.f * apq);
          t = (theta >= 0.f ? 1.f : -1.f) / (fabsf(theta) + sqrtf(1.f + theta * theta));
          c = 1.f / sqrtf(1.f + t * t);
          s = t * c;
          atomicAdd(&nrot, 1);
        }
        rp[k] = p; rq[k] = q; rc[k] = c; rs[k] = s;
        rt[k] = t; rpp[k] = app; rqq[k] = aqq; rpq[k] = apq;
      }
      __syncthreads();
      // --- column phase: S <- S J, and V <- V J (rows p, q of V^T)
      for (int e = tid; e < npairs * ne; e += 256) {
        int k = e / ne, i = e - k * ne;
        float c = rc[k], s = rs[k];
        if (s == 0.f) continue;
        int p = rp[k], q = rq[k];
        const float tau = s / (1.f + c);
        float sp = S[i * ld + p], sq = S[i * ld + q];
        S[i * ld + p] = sp - s * (sq + tau * sp);
        S[i * ld + q] = sq + s * (sp - tau * sq);
        if (i < n && q < n) {
          float vp = J.Vt[(long long)p * n + i], vq = J.Vt[(long long)q * n + i];
          J.Vt[(long long)p * n + i] = vp - s * (vq + tau * vp);
          J.Vt[(long long)q * n + i] = vq + s * (vp - tau * vq);
        }
      }
      __syncthreads();
      // --- row phase: S <- J^T S
      for (int e = tid; e < npairs * ne; e += 256) {
        int k = e / ne, j = e - k * ne;
        float c = rc[k], s = rs[k];
        if (s == 0.f) continue;
        int p = rp[k], q = rq[k];
        const float tau = s / (1.f + c);
        float sp = S[p * ld + j], sq = S[q * ld + j];
        S[p * ld + j] = sp - s * (sq + tau * sp);
        S[q * ld + j] = sq + s * (sp - tau * sq);
      }
      __syncthreads();
      // annihilated entries are exactly zero; the rotated diagonal uses the
      // cancellation-free a_pp - t a_pq / a_qq + t a_pq (the generic two-sided
      // update of the diagonal loses ~20x accuracy in fp32)
      for (int k = tid; k < npairs; k += 256) {
        if (rs[k] != 0.f) {
          int p = rp[k], q = rq[k];
          S[p * ld + q] = 0.f; S[q * ld + p] = 0.f;
          S[p * ld + p] = rpp[k] - rt[k] * rpq[k];
          S[q * ld + q] = rqq[k] + rt[k] * rpq[k];
        }
      }
      __syncthreads();
    }
    if (nrot == 0) break;
    __syncthreads();
  }

  // --- ascending order + clip, Q[:, rank(i)] = V[:, i] = Vt[i, :]
  for (int i = tid; i < n; i += 256) dsh[i] = S[i * ld + i];
  __syncthreads();
  for (int i = tid; i < n; i += 256) {
    float di = dsh[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      float dj = dsh[j];
      rank += (dj < di) || (dj == di && j < i);
    }
    J.d[rank] = batch.do_clip ? fmaxf(di, batch.clip) : di;
    for (int k = 0; k < n; ++k) J.Q[(long long)k * n + rank] = J.Vt[(long long)i * n + k];
  }
}

}  // namespace

struct KfacEigRecord {
  const float* A;
  float* Q;
  float* d;
  float* Vt;
  long long n;
};

KFAC_API int kfac_max_small_eig_n() { return NMAX; }

KFAC_API int kfac_eig_jacobi_small(const KfacEigRecord* recs, int count, int max_sweeps, float tol,
                                   int do_clip, float clip, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)jacobi_small_kernel,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr_set = true;
  }
  for (int base = 0; base < count; base += MAXJ) {
    EigBatch b;
    b.count = count - base < MAXJ ? count - base : MAXJ;
    b.max_sweeps = max_sweeps; b.tol = tol; b.do_clip = do_clip; b.clip = clip;
    int maxn = 0;
    for (int k = 0; k < b.count; ++k) {
      const KfacEigRecord& r = recs[base + k];
      if (r.n > NMAX || r.n <= 0) return -2;
      b.job[k].A = r.A; b.job[k].Q = r.Q; b.job[k].d = r.d; b.job[k].Vt = r.Vt;
      b.job[k].n = (int)r.n; b.job[k].pad = 0;
      if (r.n > maxn) maxn = (int)r.n;
    }
    int ne = maxn + (maxn & 1);
    size_t lds = (size_t)ne * (ne + 1) * sizeof(float);
    hipLaunchKernelGGL(jacobi_small_kernel, dim3(b.count), dim3(256), lds, stream, b);
    int err = (int)hipGetLastError();
    if (err) return err;
  }
  return 0;
}
