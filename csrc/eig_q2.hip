// Back-transformation through the bulge-chasing reflectors (Q2 of the
// two-stage eigensolver; csrc/eig_sb2st.hip writes them).  Z (eigenvectors
// of the tridiagonal matrix, one per row) <- Q2 Z.
//
// Groups: the 16 sweeps 16 g .. 16 g + 15 at one step j form
// G(g, j) = H(16g, j) ... H(16g+15, j) = I - V T V^T, V a 31 x 16 window of
// staggered reflectors starting at row 16 g + 1 + 16 j.  Q2 Z applies the
// blocks g descending and, inside a block, j ascending; group (g, j) at tick
// (G-1-g) + j keeps that order and the groups of one tick touch disjoint row
// windows (scripts/models/two_stage_model.py: apply_q2_ticks).
//
//   q2_t     one wave per group: Gram of the window, T (larft, forward)
//   q2_pass  one workgroup per (matrix, 64 eigenvectors), lane = eigenvector;
//            8 blocks per pass in the tick order (wave w = block gtop - w),
//            the touched rows streaming through an LDS window, so Z is read
//            and written once per pass rather than once per group (a launch
//            per tick over global memory was 30x slower on ResNet-50)
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int BW = 16;
constexpr int WR = 2 * BW - 1;     // window rows
constexpr int MAXM = 255;

struct Q2Mat {
  const float* v2; long long ldv2;
  float* Z; long long ldz;
  float* T;                        // [G][jmax][16][16]
  int n, G, jmax, pad;
};

__device__ inline void map_block(const int* __restrict__ offs, int nact, int* soff, int& mat,
                                 int& local) {
  __shared__ int sm;
  const int t = threadIdx.x, b = blockIdx.x;
  for (int i = t; i <= nact; i += blockDim.x) soff[i] = offs[i];   // any block size
  __syncthreads();
  for (int i = t; i < nact; i += blockDim.x)
    if (soff[i] <= b && b < soff[i + 1]) sm = i;
  __syncthreads();
  mat = sm;
  local = b - soff[mat];
}

// does sweep s have a step j (stage 2 task with >= 2 rows)?
__device__ __forceinline__ bool has_step(int n, int s, int j) {
  return s <= n - 3 && j * BW <= n - 3 - s;
}

// reflector i of group (g, j): v[l], l < 16 (v[0] = 1), tau
__device__ __forceinline__ float refl_v(const Q2Mat& M, int g, int j, int i, int l, float* tau) {
  const int s = BW * g + i;
  if (!has_step(M.n, s, j)) { if (tau) *tau = 0.f; return 0.f; }
  const AS1 float* row = gptr(M.v2) + (long long)s * M.ldv2 + BW * j;
  if (tau) *tau = row[0];
  return l == 0 ? 1.f : row[l];
}

__global__ __launch_bounds__(64) void q2_t_kernel(const Q2Mat* __restrict__ mats,
                                                  const int* __restrict__ offs, int nact) {
  __shared__ int soff[MAXM + 1];
  __shared__ float V[BW][BW];      // V[i][l] = v_i[l]
  __shared__ float tau[BW];
  __shared__ float G[BW][BW + 1];
  __shared__ float T[BW][BW + 1];
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const Q2Mat M = mats[mi];
  const int g = local / M.jmax, j = local % M.jmax;
  const int lane = threadIdx.x;
  if (!has_step(M.n, BW * g, j)) return;       // empty group (uniform)
  for (int e = lane; e < BW * BW; e += 64) {
    const int i = e / BW, l = e % BW;
    float t;
    V[i][l] = refl_v(M, g, j, i, l, &t);
    if (l == 0) tau[i] = t;
  }
  __syncthreads();
  // G[a][b] = sum_r V_win[r][a] V_win[r][b], V_win[r][i] = v_i[r - i]
  for (int e = lane; e < BW * BW; e += 64) {
    const int a = e / BW, b = e % BW;
    float s = 0.f;
    for (int r = max(a, b); r < min(a, b) + BW; ++r) s += V[a][r - a] * V[b][r - b];
    G[a][b] = s;
  }
  for (int e = lane; e < BW * (BW + 1); e += 64) (&T[0][0])[e] = 0.f;
  __syncthreads();
  for (int i = 0; i < BW; ++i) {
    const float ti = tau[i];
    float acc = 0.f;
    if (lane < i)
      for (int q = lane; q < i; ++q) acc += T[lane][q] * G[q][i];
    __syncthreads();
    if (lane < i) T[lane][i] = -ti * acc;
    else if (lane == i) T[lane][i] = ti;
    __syncthreads();
  }
  float* const out = M.T + ((long long)g * M.jmax + j) * BW * BW;
  for (int e = lane; e < BW * BW; e += 64) out[e] = T[e / BW][e % BW];
}

// One workgroup per (matrix, 64 eigenvectors): lane = eigenvector.  Blocks
// are processed QW at a time ("passes", g descending); inside a pass wave w
// owns block gtop - w and runs its step tau - w at tick tau, so the pass is
// the tick order of the groups it contains.  The rows the pass touches stream
// through a circular LDS window (ZR rows x 64 eigenvectors): every element of
// Z is read and written once per pass instead of once per group.
constexpr int QW = 8;
constexpr int ZR = 512;
struct Q2Strip { int mat, e0; };

__device__ __forceinline__ int q2_steps(int n, int g) {      // J_g
  return (BW * g <= n - 3) ? (n - 3 - BW * g) / BW + 1 : 0;
}

__global__ __launch_bounds__(QW * 64) void q2_pass_kernel(const Q2Mat* __restrict__ mats,
                                                          const Q2Strip* __restrict__ strips) {
  extern __shared__ float Lz[];                 // ZR x 64: row r at (r % ZR) * 64
  __shared__ float sV[QW][BW][BW];
  __shared__ float sT[QW][BW][BW];
  const Q2Strip S = strips[blockIdx.x];
  const Q2Mat M = mats[S.mat];
  const int n = M.n, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e = S.e0 + lane;
  const bool eok = e < n;
  AS1 float* const Zg = gptr(M.Z);
  auto zrow = [&](int r) -> float {   // Z element (row r, this lane's eigenvector)
    return eok ? Zg[(long long)r * M.ldz + e] : 0.f;
  };
  for (int gtop = M.G - 1; gtop >= 0; gtop -= QW) {
    const int glow = max(0, gtop - QW + 1);
    const int rlo = BW * glow + 1;
    int stored = rlo;
    int nticks = 0;
    for (int w = 0; w <= gtop - glow; ++w) nticks = max(nticks, w + q2_steps(n, gtop - w));
    // rows needed by tick tau: < need(tau) = min(n, 16 (gtop + tau) + 32); tick 0's
    // rows load synchronously, later ticks' 16 new rows (2 per wave) are loaded
    // one tick ahead into registers; so are each wave's V / T for its next group
    const int need0 = min(n, BW * gtop + 2 * BW);
    for (int r = rlo + wave; r < need0; r += QW) Lz[(r & (ZR - 1)) * 64 + lane] = zrow(r);
    int loaded = need0;
    float pz0 = 0.f, pz1 = 0.f, pv[4], pt[4];
    auto load_vt = [&](int tau) {
      const int g = gtop - wave, j = tau - wave;
      const bool ok = g >= glow && j >= 0 && j < q2_steps(n, g);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = lane + 64 * k;
        pv[k] = ok ? refl_v(M, g, j, idx / BW, idx % BW, nullptr) : 0.f;
        pt[k] = ok ? gptr(M.T)[((long long)g * M.jmax + j) * BW * BW + idx] : 0.f;
      }
    };
    load_vt(0);
    for (int tau = 0; tau < nticks; ++tau) {
      // V / T of this tick to the wave's LDS slot, next tick's issued
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = lane + 64 * k;
        sV[wave][idx / BW][idx % BW] = pv[k];
        sT[wave][idx / BW][idx % BW] = pt[k];
      }
      load_vt(tau + 1);
      const int need1 = min(n, BW * (gtop + tau + 1) + 2 * BW);   // rows of tick tau + 1
      {
        const int r0 = loaded + wave, r1 = loaded + wave + QW;
        pz0 = r0 < need1 ? zrow(r0) : 0.f;
        pz1 = r1 < need1 ? zrow(r1) : 0.f;
      }
      kfac_lds_barrier();      // previous tick's commits visible
      const int g = gtop - wave, j = tau - wave;
      if (g >= glow && j >= 0 && j < q2_steps(n, g)) {
        const int row0 = BW * (g + j) + 1;
        const int wr = min(WR, n - row0);
        float z[WR];
#pragma unroll
        for (int r = 0; r < WR; ++r) z[r] = r < wr ? Lz[((row0 + r) & (ZR - 1)) * 64 + lane] : 0.f;
        float p[BW];
#pragma unroll
        for (int i = 0; i < BW; ++i) {
          float s_ = 0.f;
#pragma unroll
          for (int l = 0; l < BW; ++l) s_ += sV[wave][i][l] * z[i + l];
          p[i] = s_;
        }
        float q[BW];
#pragma unroll
        for (int i = 0; i < BW; ++i) {
          float s_ = 0.f;
#pragma unroll
          for (int k = i; k < BW; ++k) s_ += sT[wave][i][k] * p[k];
          q[i] = s_;
        }
#pragma unroll
        for (int r = 0; r < WR; ++r) {
          float s_ = z[r];
#pragma unroll
          for (int i = 0; i < BW; ++i)
            if (r - i >= 0 && r - i < BW) s_ -= sV[wave][i][r - i] * q[i];
          if (r < wr) Lz[((row0 + r) & (ZR - 1)) * 64 + lane] = s_;
        }
      }
      // commit the rows of tick tau + 1 (not touched at tick tau: beyond need(tau))
      {
        const int r0 = loaded + wave, r1 = loaded + wave + QW;
        if (r0 < need1) Lz[(r0 & (ZR - 1)) * 64 + lane] = pz0;
        if (r1 < need1) Lz[(r1 & (ZR - 1)) * 64 + lane] = pz1;
        loaded = max(loaded, need1);
      }
      kfac_lds_barrier();
      // rows no later step of the pass touches go back to global memory
      int lo = n;
      for (int w = 0; w <= gtop - glow; ++w) {
        const int gw = gtop - w, jn = max(tau + 1 - w, 0);
        if (jn < q2_steps(n, gw)) lo = min(lo, BW * (gw + jn) + 1);
      }
      lo = min(lo, loaded);
      for (int r = stored + wave; r < lo; r += QW)
        if (eok) Zg[(long long)r * M.ldz + e] = Lz[(r & (ZR - 1)) * 64 + lane];
      stored = max(stored, lo);
    }
    for (int r = stored + wave; r < loaded; r += QW)
      if (eok) Zg[(long long)r * M.ldz + e] = Lz[(r & (ZR - 1)) * 64 + lane];
    __syncthreads();
  }
}

struct Q2Plan {
  Q2Mat* d_mats = nullptr;
  Q2Strip* d_strips = nullptr;
  int nstrip = 0;
  int* d_offs = nullptr;      // [nm + 1]: T-kernel workgroup offsets
  int count = 0;
  std::vector<int> grid, nact;
  hipGraphExec_t exec = nullptr;
};

int enqueue(const Q2Plan& P, hipStream_t stream) {
  if (P.grid[0] > 0)
    hipLaunchKernelGGL(q2_t_kernel, dim3(P.grid[0]), dim3(64), 0, stream, P.d_mats, P.d_offs,
                       P.nact[0]);
  if (P.nstrip > 0)
    hipLaunchKernelGGL(q2_pass_kernel, dim3(P.nstrip), dim3(QW * 64), ZR * 64 * sizeof(float),
                       stream, P.d_mats, P.d_strips);
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, Q2Plan> g_plans;

inline int q2_G(int n) { return (n - 1 + BW - 1) / BW; }
inline int q2_jmax(int n) { return n >= 3 ? (n - 3) / BW + 1 : 0; }

}  // namespace

struct KfacQ2Record {
  const float* v2; long long ldv2; float* Z; long long ldz; float* T; long long n;
};

// T workspace floats per matrix
KFAC_API long long kfac_q2_t_floats(int n) {
  return (long long)std::max(1, q2_G(n)) * std::max(1, q2_jmax(n)) * BW * BW;
}

// Z (component-major: row r = component r of all n eigenvectors of the
// tridiagonal matrix, ldz) <- Q2 Z for every matrix of the batch.
KFAC_API int kfac_q2_batched(const KfacQ2Record* recs, int count, int use_graph,
                             hipStream_t stream) {
  if (count <= 0) return 0;
  if (count > MAXM) return -5;
  std::vector<Q2Mat> mats(count);
  for (int i = 0; i < count; ++i) {
    const KfacQ2Record& r = recs[i];
    if (r.n < 2) return -2;
    Q2Mat& M = mats[i];
    memset(&M, 0, sizeof(M));
    M.v2 = r.v2; M.ldv2 = r.ldv2; M.Z = r.Z; M.ldz = r.ldz; M.T = r.T; M.n = (int)r.n;
    M.G = q2_G(M.n); M.jmax = q2_jmax(M.n);
  }
  const std::string key((const char*)mats.data(), sizeof(Q2Mat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    Q2Plan P;
    P.count = count;
    const int nm = count;
    // T kernel: one workgroup per (matrix, group); the pass kernel: one per
    // (matrix, 64 eigenvectors)
    std::vector<int> offs((size_t)nm + 1, 0);
    P.grid.assign(1, 0);
    P.nact.assign(1, 0);
    {
      int acc = 0;
      for (int i = 0; i < nm; ++i) {
        offs[i] = acc;
        const int c = mats[i].G * mats[i].jmax;
        if (c > 0) P.nact[0] = i + 1;
        acc += c;
      }
      offs[nm] = acc;
      P.grid[0] = acc;
    }
    int e = (int)hipMalloc(&P.d_mats, sizeof(Q2Mat) * nm);
    if (!e) e = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(Q2Mat) * nm, hipMemcpyHostToDevice);
    if (!e) e = (int)hipMalloc(&P.d_offs, sizeof(int) * offs.size());
    if (!e) e = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * offs.size(), hipMemcpyHostToDevice);
    std::vector<Q2Strip> strips;
    for (int i = 0; i < nm; ++i)
      for (int e0 = 0; e0 < mats[i].n; e0 += 64) strips.push_back(Q2Strip{i, e0});
    P.nstrip = (int)strips.size();
    if (!e) e = (int)hipMalloc(&P.d_strips, sizeof(Q2Strip) * strips.size());
    if (!e) e = (int)hipMemcpy(P.d_strips, strips.data(), sizeof(Q2Strip) * strips.size(),
                               hipMemcpyHostToDevice);
    static bool attr = false;
    if (!e && !attr) {
      e = (int)hipFuncSetAttribute((const void*)q2_pass_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   ZR * 64 * (int)sizeof(float));
      attr = (e == 0);
    }
    if (e) return e;
    it = g_plans.emplace(key, P).first;
  }
  Q2Plan& P = it->second;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  if (graph && !P.exec) {
    static hipStream_t cap = nullptr;
    if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
    hipGraph_t gr = nullptr;
    if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      const int e1 = enqueue(P, cap);
      const hipError_t e2 = hipStreamEndCapture(cap, &gr);
      if (!e1 && e2 == hipSuccess && gr && hipGraphInstantiate(&P.exec, gr, nullptr, nullptr, 0) != hipSuccess)
        P.exec = nullptr;
      if (gr) (void)hipGraphDestroy(gr);
    }
    (void)hipGetLastError();
  }
  if (graph && P.exec) return (int)hipGraphLaunch(P.exec, stream);
  return enqueue(P, stream);
}
