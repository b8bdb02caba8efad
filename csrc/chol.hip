// Batched damped inverse (F + damping I)^-1 of symmetric positive definite
// K-FAC factors by Cholesky (reference kfac/layers/utils.py:76-96
// = torch.cholesky + torch.cholesky_inverse per factor, base.py:472-475).
//
// Every factor of the inverse update (any sizes) advances through ONE ragged
// launch sequence with 64-wide blocks (fp32 throughout, LAPACK spotrf/spotri
// arithmetic):
//   copy      W = lower(F) + damping I (padding rows: identity), XT = 0
//   diag(k)   one workgroup per matrix: L_kk = chol(W_kk) in LDS and its
//             triangular inverse Linv_k (both kept)
//   trsm(k)   L_ik = W_ik Linv_k^T for every block row i > k   (v_mfma 32x32x2 f32)
//   syrk(k)   W_ij -= L_ik L_jk^T for k < j <= i                 (v_mfma 32x32x2 f32)
//   trtri(i)  X = L^-1 by block rows: X_ic = -Linv_i sum_{c<=j<i} L_ij X_jc,
//             X_ii = Linv_i, stored TRANSPOSED (XT, row m = column m of X)
//   lauum     (F + damping I)^-1 = L^-T L^-1 = X^T X: one grouped NT pgemm
//             XT . XT^T for all matrices (csrc/precond_gemm.hip)
// The sequence is captured into a cached hipGraph per (records, damping).
#include "pgemm.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int CB = 64;          // block
constexpr int CMAXM = 255;      // matrices per batch
constexpr int CLD = CB + 1;     // LDS row stride

struct CMat {
  const AS1 float* F; long long ldf;   // factor (row-major, symmetric; lower triangle read)
  AS1 float* out; long long ldo;       // result
  AS1 float* W;                        // npad x npad: W, then L (lower blocks)
  AS1 float* Linv;                     // nb x CB x CB: inverses of the diagonal blocks
  AS1 float* XT;                       // npad x npad: (L^-1)^T
  AS1 int* info;                       // != 0: a pivot was not positive
  int n, nb, npad;
  float damping;
};

__device__ inline void map_wg(const int* __restrict__ offs, int nact, int* soff, int& mat,
                              int& local) {
  __shared__ int sm;
  const int t = threadIdx.x, b = blockIdx.x;
  if (t <= nact) soff[t] = offs[t];
  __syncthreads();
  if (t < nact && soff[t] <= b && b < soff[t + 1]) sm = t;
  __syncthreads();
  mat = sm;
  local = b - soff[mat];
}

// 64 x 64 block of a row-major matrix (ld) into LDS, branch-free
__device__ inline void load_block(float (*s)[CLD], const AS1 float* src, long long ld) {
  for (int e = threadIdx.x; e < CB * CB; e += 256) {
    const int i = e / CB, j = e - i * CB;
    s[i][j] = src[(long long)i * ld + j];
  }
}

// acc (4 waves: 32 x 32 quadrants of a 64 x 64 tile) += A . B^T over 64 k
__device__ inline void mfma_nt(const float (*sA)[CLD], const float (*sB)[CLD], f32x16_t& acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1, l31 = lane & 31, lh = lane >> 5;
#pragma unroll 8
  for (int s = 0; s < CB / 2; ++s) {
    const int k = 2 * s + lh;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[wr * 32 + l31][k], sB[wc * 32 + l31][k], acc,
                                               0, 0, 0);
  }
}

// C/D map of 32x32x2: element x of lane -> (row, col) of the wave's quadrant
__device__ inline void quad_rc(int x, int& r, int& c) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  r = (wave >> 1) * 32 + (x & 3) + 8 * (x >> 2) + 4 * (lane >> 5);
  c = (wave & 1) * 32 + (lane & 31);
}

__global__ __launch_bounds__(256) void chol_copy_kernel(const CMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact) {
  __shared__ int soff[CMAXM + 1];
  int mi, r;
  map_wg(offs, nact, soff, mi, r);
  const CMat M = mats[mi];
  const int n = M.n, npad = M.npad;
  for (int c = threadIdx.x; c < npad; c += 256) {
    float v = 0.f;
    if (r < n && c < n && c <= r) v = M.F[(long long)r * M.ldf + c];
    if (c == r) v += (r < n) ? M.damping : 1.f;
    M.W[(long long)r * npad + c] = v;
    M.XT[(long long)r * npad + c] = 0.f;
  }
  if (r == 0 && threadIdx.x == 0) *M.info = 0;
}

__global__ __launch_bounds__(256) void chol_diag_kernel(const CMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int k) {
  __shared__ float a[CB][CLD], x[CB][CLD];
  __shared__ int soff[CMAXM + 1];
  __shared__ int bad;
  int mi, local;
  map_wg(offs, nact, soff, mi, local);
  const CMat M = mats[mi];
  const int tid = threadIdx.x;
  const long long r0 = (long long)k * CB;
  AS1 float* blk = M.W + r0 * M.npad + r0;
  load_block(a, blk, M.npad);
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int j = 0; j < CB; ++j) {
    if (tid == 0) {
      float d = a[j][j];
      if (!(d > 0.f)) { bad = 1; d = 1.f; }
      a[j][j] = sqrtf(d);
    }
    __syncthreads();
    if (tid > j && tid < CB) a[tid][j] /= a[j][j];
    __syncthreads();
    for (int e = tid; e < CB * CB; e += 256) {
      const int i = e / CB, l = e - i * CB;
      if (l > j && i >= l) a[i][l] -= a[i][j] * a[l][j];
    }
    __syncthreads();
  }
  // x = a^-1 (lower): thread t forms column t by forward substitution
  if (tid < CB) {
    const int t = tid;
    for (int i = 0; i < CB; ++i) {
      float s = (i == t) ? 1.f : 0.f;
      if (i > t)
        for (int j = t; j < i; ++j) s -= a[i][j] * x[j][t];
      x[i][t] = (i >= t) ? s / a[i][i] : 0.f;
    }
  }
  __syncthreads();
  AS1 float* li = M.Linv + (long long)k * CB * CB;
  for (int e = tid; e < CB * CB; e += 256) {
    const int i = e / CB, j = e - i * CB;
    blk[(long long)i * M.npad + j] = (j <= i) ? a[i][j] : 0.f;
    li[e] = x[i][j];
  }
  if (tid == 0 && bad) atomicAdd((int*)M.info, 1);
}

// L_ik = W_ik Linv_k^T, i = k + 1 + local
__global__ __launch_bounds__(256) void chol_trsm_kernel(const CMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int k) {
  __shared__ float sA[CB][CLD], sB[CB][CLD];
  __shared__ int soff[CMAXM + 1];
  int mi, local;
  map_wg(offs, nact, soff, mi, local);
  const CMat M = mats[mi];
  const int i = k + 1 + local;
  AS1 float* blk = M.W + (long long)i * CB * M.npad + (long long)k * CB;
  load_block(sA, blk, M.npad);
  load_block(sB, M.Linv + (long long)k * CB * CB, CB);
  __syncthreads();
  f32x16_t acc;
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = 0.f;
  mfma_nt(sA, sB, acc);
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    int r, c;
    quad_rc(x, r, c);
    blk[(long long)r * M.npad + c] = acc[x];
  }
}

// W_ij -= L_ik L_jk^T, (i, j) = the local-th lower pair of blocks past k
__global__ __launch_bounds__(256) void chol_syrk_kernel(const CMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int k) {
  __shared__ float sA[CB][CLD], sB[CB][CLD];
  __shared__ int soff[CMAXM + 1];
  int mi, local;
  map_wg(offs, nact, soff, mi, local);
  const CMat M = mats[mi];
  int ii = 0;
  while ((ii + 1) * (ii + 2) / 2 <= local) ++ii;
  const int jj = local - ii * (ii + 1) / 2;
  const int i = k + 1 + ii, j = k + 1 + jj;
  const long long ld = M.npad;
  load_block(sA, M.W + (long long)i * CB * ld + (long long)k * CB, ld);
  load_block(sB, M.W + (long long)j * CB * ld + (long long)k * CB, ld);
  __syncthreads();
  f32x16_t acc;
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = 0.f;
  mfma_nt(sA, sB, acc);
  AS1 float* dst = M.W + (long long)i * CB * ld + (long long)j * CB;
  float old[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    int r, c;
    quad_rc(x, r, c);
    old[x] = dst[(long long)r * ld + c];
  }
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    int r, c;
    quad_rc(x, r, c);
    dst[(long long)r * ld + c] = old[x] - acc[x];
  }
}

// block row i of X = L^-1, column block c = local (<= i), written transposed
__global__ __launch_bounds__(256) void chol_trtri_kernel(const CMat* __restrict__ mats,
                                                         const int* __restrict__ offs, int nact,
                                                         int i) {
  __shared__ float sA[CB][CLD], sB[CB][CLD];
  __shared__ int soff[CMAXM + 1];
  int mi, c;
  map_wg(offs, nact, soff, mi, c);
  const CMat M = mats[mi];
  const long long ld = M.npad;
  const AS1 float* li = M.Linv + (long long)i * CB * CB;
  AS1 float* dst = M.XT + (long long)c * CB * ld + (long long)i * CB;   // XT block (c, i)
  if (c == i) {
    for (int e = threadIdx.x; e < CB * CB; e += 256) {
      const int r = e / CB, col = e - r * CB;
      dst[(long long)col * ld + r] = li[e];                 // X_ii = Linv_i
    }
    return;
  }
  f32x16_t acc;
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = 0.f;
  for (int j = c; j < i; ++j) {     // T = sum L_ij X_jc  (X_jc^T = XT block (c, j))
    load_block(sA, M.W + (long long)i * CB * ld + (long long)j * CB, ld);
    load_block(sB, M.XT + (long long)c * CB * ld + (long long)j * CB, ld);
    __syncthreads();
    mfma_nt(sA, sB, acc);
    __syncthreads();
  }
  // X_ic = -Linv_i T: T^T into sB (B operand rows = output columns), Linv_i into sA
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    int r, col;
    quad_rc(x, r, col);
    sB[col][r] = acc[x];
  }
  load_block(sA, li, CB);
  __syncthreads();
  f32x16_t acc2;
#pragma unroll
  for (int x = 0; x < 16; ++x) acc2[x] = 0.f;
  mfma_nt(sA, sB, acc2);
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    int r, col;
    quad_rc(x, r, col);
    dst[(long long)col * ld + r] = -acc2[x];
  }
}

// ------------------------------------------------------------------ host
struct CPlan {
  CMat* d_mats = nullptr;
  int* d_offs = nullptr;            // [5][nbmax][nm + 1]: copy, diag, trsm, syrk, trtri
  PGemm* d_gemm = nullptr;
  int gemm_tiles = 0;
  std::vector<int> grid[5], nact[5];
  int nbmax = 0, nm = 0;
  hipGraphExec_t exec = nullptr;
  unsigned long long used = 0;      // LRU clock
  bool pinned = false;              // enqueued into an outer capture: never evicted
};

int cdiv(int a, int b) { return (a + b - 1) / b; }

int enqueue(const CPlan& P, hipStream_t s) {
  const size_t stride = (size_t)P.nbmax * (P.nm + 1);
  auto of = [&](int kind, int step) { return P.d_offs + kind * stride + (size_t)step * (P.nm + 1); };
  hipLaunchKernelGGL(chol_copy_kernel, dim3(P.grid[0][0]), dim3(256), 0, s, P.d_mats, of(0, 0),
                     P.nact[0][0]);
  for (int k = 0; k < P.nbmax; ++k) {
    hipLaunchKernelGGL(chol_diag_kernel, dim3(P.grid[1][k]), dim3(256), 0, s, P.d_mats,
                       of(1, k), P.nact[1][k], k);
    if (P.grid[2][k] > 0)
      hipLaunchKernelGGL(chol_trsm_kernel, dim3(P.grid[2][k]), dim3(256), 0, s, P.d_mats,
                         of(2, k), P.nact[2][k], k);
    if (P.grid[3][k] > 0)
      hipLaunchKernelGGL(chol_syrk_kernel, dim3(P.grid[3][k]), dim3(256), 0, s, P.d_mats,
                         of(3, k), P.nact[3][k], k);
  }
  for (int i = 0; i < P.nbmax; ++i)
    hipLaunchKernelGGL(chol_trtri_kernel, dim3(P.grid[4][i]), dim3(256), 0, s, P.d_mats,
                       of(4, i), P.nact[4][i], i);
  int err = (int)hipGetLastError();
  if (err) return err;
  return kfac_pgemm(PREC_F32, 0, P.d_gemm, P.nm, P.gemm_tiles, nullptr, s);
}

std::mutex g_mu;
std::map<std::string, CPlan> g_plans;

}  // namespace

struct KfacCholRecord {
  const float* F; long long ldf; float* out; long long ldo; void* ws; long long n;
};

// workspace bytes per matrix of size n (256-byte aligned)
KFAC_API long long kfac_chol_ws_bytes(int n) {
  const long long nb = (n + CB - 1) / CB, npad = nb * CB;
  const long long b = 4 * (2 * npad * npad + nb * CB * CB) + 256;
  return (b + 255) / 256 * 256;
}

namespace {

constexpr int kMaxPlans = 16;
unsigned long long g_clock = 0;

CPlan* plan_for(const KfacCholRecord* recs, int count, float damping, bool capture,
                bool capturing, int* err) {
  std::vector<int> order(count);
  for (int i = 0; i < count; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return recs[a].n > recs[b].n; });
  std::vector<CMat> mats;
  for (int oi : order) {
    const KfacCholRecord& r = recs[oi];
    if (r.n < 1 || r.ldf < r.n || r.ldo < r.n) { *err = -2; return nullptr; }
    CMat M;
    memset(&M, 0, sizeof(M));
    M.F = (const AS1 float*)r.F; M.ldf = r.ldf;
    M.out = (AS1 float*)r.out; M.ldo = r.ldo;
    M.n = (int)r.n; M.nb = cdiv(M.n, CB); M.npad = M.nb * CB;
    M.damping = damping;
    float* p = (float*)r.ws;
    M.W = (AS1 float*)p; p += (long long)M.npad * M.npad;
    M.XT = (AS1 float*)p; p += (long long)M.npad * M.npad;
    M.Linv = (AS1 float*)p; p += (long long)M.nb * CB * CB;
    M.info = (AS1 int*)p;
    mats.push_back(M);
  }
  const std::string key((const char*)mats.data(), sizeof(CMat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    // the key holds the factor / output / workspace pointers and the damping:
    // fresh snapshot buffers or a damping schedule make new keys, so the cache
    // is bounded (LRU).  Eviction drains the device first (an evicted graph or
    // table may still be in flight), never inside a stream capture.
    if ((int)g_plans.size() >= kMaxPlans && !capturing) {
      auto victim = g_plans.end();
      for (auto v = g_plans.begin(); v != g_plans.end(); ++v)
        if (!v->second.pinned && (victim == g_plans.end() || v->second.used < victim->second.used))
          victim = v;
      if (victim != g_plans.end()) {
        (void)hipDeviceSynchronize();
        CPlan& V = victim->second;
        if (V.exec) (void)hipGraphExecDestroy(V.exec);
        (void)hipFree(V.d_mats);
        (void)hipFree(V.d_offs);
        (void)hipFree(V.d_gemm);
        g_plans.erase(victim);
      }
    }
    CPlan P;
    P.nm = (int)mats.size();
    P.nbmax = mats[0].nb;
    const int nm = P.nm;
    std::vector<int> offs((size_t)5 * P.nbmax * (nm + 1), 0);
    for (int kind = 0; kind < 5; ++kind) {
      P.grid[kind].assign(P.nbmax, 0);
      P.nact[kind].assign(P.nbmax, 0);
    }
    for (int step = 0; step < P.nbmax; ++step) {
      int acc[5] = {0, 0, 0, 0, 0};
      for (int i = 0; i < nm; ++i) {
        const int nb = mats[i].nb;
        int cnt[5];
        cnt[0] = step == 0 ? mats[i].npad : 0;               // copy: one workgroup per row
        cnt[1] = step < nb ? 1 : 0;                          // diag
        const int m = nb - step - 1;
        cnt[2] = m > 0 ? m : 0;                              // trsm
        cnt[3] = m > 0 ? m * (m + 1) / 2 : 0;                // syrk
        cnt[4] = step < nb ? step + 1 : 0;                   // trtri
        for (int kind = 0; kind < 5; ++kind) {
          offs[((size_t)kind * P.nbmax + step) * (nm + 1) + i] = acc[kind];
          if (cnt[kind] > 0) P.nact[kind][step] = i + 1;
          acc[kind] += cnt[kind];
        }
      }
      for (int kind = 0; kind < 5; ++kind) {
        offs[((size_t)kind * P.nbmax + step) * (nm + 1) + nm] = acc[kind];
        P.grid[kind][step] = acc[kind];
      }
    }
    std::vector<PGemm> recs_g(nm);
    int tiles = 0;
    for (int i = 0; i < nm; ++i) {
      PGemm& g = recs_g[i];
      memset(&g, 0, sizeof(g));
      const CMat& M = mats[i];
      g.a_hi = g.a_lo = (const void*)M.XT; g.lda = M.npad;
      g.b_hi = g.b_lo = (const void*)M.XT; g.ldb = M.npad;
      g.c_hi = g.c_lo = (void*)M.out; g.ldc = M.ldo;
      g.M = M.n; g.N = M.n; g.K = M.npad; g.epi = EPI_STORE;
      g.tiles_n = cdiv(M.n, 128);
      g.tile_begin = tiles;
      tiles += cdiv(M.n, 128) * g.tiles_n;
    }
    // pgemm finds a workgroup's record by tile_begin (ascending): keep order
    P.gemm_tiles = tiles;
    if ((*err = (int)hipMalloc(&P.d_mats, sizeof(CMat) * nm)) != 0) return nullptr;
    if ((*err = (int)hipMalloc(&P.d_offs, sizeof(int) * offs.size())) != 0) return nullptr;
    if ((*err = (int)hipMalloc(&P.d_gemm, sizeof(PGemm) * nm)) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(CMat) * nm,
                               hipMemcpyHostToDevice)) != 0 ||
        (*err = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * offs.size(),
                               hipMemcpyHostToDevice)) != 0 ||
        (*err = (int)hipMemcpy(P.d_gemm, recs_g.data(), sizeof(PGemm) * nm,
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    it = g_plans.emplace(key, P).first;
  }
  CPlan* plan = &it->second;
  plan->used = ++g_clock;
  if (capturing) plan->pinned = true;
  if (capture && !plan->exec) {
    static hipStream_t cap = nullptr;
    if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
    hipGraph_t graph = nullptr;
    if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      const int e1 = enqueue(*plan, cap);
      const hipError_t e2 = hipStreamEndCapture(cap, &graph);
      if (!e1 && e2 == hipSuccess && graph &&
          hipGraphInstantiate(&plan->exec, graph, nullptr, nullptr, 0) != hipSuccess)
        plan->exec = nullptr;
      if (graph) (void)hipGraphDestroy(graph);
    }
    (void)hipGetLastError();
  }
  return plan;
}

}  // namespace

// (F + damping I)^-1 for `count` SPD factors (any sizes): F row-major (ldf,
// lower triangle read), out (ldo), ws kfac_chol_ws_bytes(n) bytes each.  The
// per-matrix status (non-positive pivots) is the int at kfac_chol_info_offset(n)
// of its workspace.
KFAC_API int kfac_chol_inverse_batched(const KfacCholRecord* recs, int count, float damping,
                                       int use_graph, hipStream_t stream) {
  if (count <= 0) return 0;
  if (count > CMAXM) return -5;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  int err = 0;
  CPlan* plan = plan_for(recs, count, damping, graph, cst != hipStreamCaptureStatusNone, &err);
  if (!plan) return err ? err : -4;
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}

KFAC_API long long kfac_chol_info_offset(int n) {
  const long long nb = (n + CB - 1) / CB, npad = nb * CB;
  return 4 * (2 * npad * npad + nb * CB * CB);
}
