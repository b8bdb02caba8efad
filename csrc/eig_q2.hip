// Back-transformation of stage 2 of the two-stage eigensolver: Z <- Q2 Z,
// Q2 = product of the bulge-chasing reflectors (csrc/eig_sb2st.hip) in the
// order they were generated (reference semantics
// kfac/layers/utils.py:45-74 -- the eigenvectors of the factor).
//
// Z is the row view of the tridiagonal eigenvectors (row k = eigenvector k,
// components along the row, ld ldz).  Sweep s's reflectors act on disjoint
// 16-component segments [s+1+16j, s+16+16j], so Q2 Z = for s descending:
// every segment of sweep s at once.  v2[s][16 j .. 16 j + 15] = (tau, v[1..15])
// of segment j (v[0] = 1 implicit).
//
// MI355X mapping: a workgroup owns QR = 6 eigenvectors; thread t owns
// SEGMENT t of the current sweep, i.e. components s+1+16t .. s+16+16t of all
// 6 rows in registers, so every dot product and update is local (16 + 16
// FMAs per row and sweep, no lane exchange, no masking).  Component x lives
// in register slot x mod 16: from sweep s to s - 1 every thread's window
// slides down by one component, which exchanges exactly ONE slot (s mod 16)
// per row: the thread's top component goes to thread t + 1, it receives
// thread t - 1's (a DPP wave_shr:1 inside the wave, an LDS word across
// waves, the untouched Z[k][s] for thread 0).  The sweep loop is unrolled 16
// times so every slot index is static.  Model:
// scripts/models/two_stage_model.py (apply_q2).
#include "common.h"

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int QT = 384;        // threads: ceil(n / 16) + 1 <= 321 segments (n <= 5120)
constexpr int QR = 6;          // eigenvectors per workgroup (8: 256 VGPRs + spills)
constexpr int QW = QT / 64;

struct Q2Mat { float* Z; const float* v2; long long ldz, ldv2; int n, pad; };

__device__ __forceinline__ int find_mat(const int* __restrict__ offs, int count, int wg,
                                        int* local) {
  int lo = 0;
  for (int i = 1; i < count; ++i)
    if (offs[i] <= wg) lo = i;
  *local = wg - offs[lo];
  return lo;
}

__device__ __forceinline__ float wave_shr1(float v) {
  // lane l <- lane l - 1 (lane 0 keeps its own value; replaced by the caller)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x138,
                                                    0xF, 0xF, false));
}

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int QP = QR / 2;     // row pairs: one packed (v_pk_fma_f32) lane-pair per component

struct Q2State {
  f2 z[QP][16];         // z[p][k] = (row 2p, row 2p + 1) at slot k
  fx4 vn[4];            // reflectors of the next sweep (prefetched)
  float zc[QR];         // wave 0, lane l < 16: Z[k][base + l] of the current block of 16 sweeps
};

// one sweep s with PH = s mod 16 known at compile time
template <int PH>
__device__ __forceinline__ void q2_sweep(Q2State& S, int s, int t, __amdgpu_buffer_rsrc_t rsv,
                                         int vof, int ldv4, float (*sx)[QW][QR]) {
  const int lane = t & 63, w = t >> 6;
  float V[16];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    V[4 * c + 0] = S.vn[c].x; V[4 * c + 1] = S.vn[c].y;
    V[4 * c + 2] = S.vn[c].z; V[4 * c + 3] = S.vn[c].w;
  }
  // prefetch sweep s - 1 (segment t; threads past the last segment read
  // nothing: their window holds only zero padding) and, for thread 0, Z[k][s]
  {
    // buffer loads: the per-thread offset is fixed, the sweep's row offset
    // uniform (threads past the last segment get an out-of-range offset:
    // zeros, and their window holds only zero padding)
    const int sp = s > 0 ? s - 1 : 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      S.vn[c] = __builtin_amdgcn_raw_buffer_load_b128(rsv, vof + 16 * c, sp * ldv4, 0);
  }
  const float tau = V[0];
  // slot k holds component with v index i = (k - PH - 1) mod 16
  float vk[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = (k - PH - 1) & 15;
    vk[k] = (i == 0) ? 1.f : V[i];
  }
#pragma unroll
  for (int p = 0; p < QP; ++p) {
    f2 d0 = {0.f, 0.f}, d1 = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
      d0 = __builtin_elementwise_fma(S.z[p][k], (f2){vk[k], vk[k]}, d0);
      d1 = __builtin_elementwise_fma(S.z[p][k + 1], (f2){vk[k + 1], vk[k + 1]}, d1);
    }
    const f2 f = -tau * (d0 + d1);
#pragma unroll
    for (int k = 0; k < 16; ++k) S.z[p][k] = __builtin_elementwise_fma(f, (f2){vk[k], vk[k]}, S.z[p][k]);
  }
  // slide the window down one component: slot PH leaves to thread t + 1,
  // arrives from thread t - 1
  float (*buf)[QR] = sx[s & 1];
#pragma unroll
  for (int p = 0; p < QP; ++p) {
    const f2 out = S.z[p][PH];
    if (lane == 63) { buf[w][2 * p] = out.x; buf[w][2 * p + 1] = out.y; }
    S.z[p][PH] = (f2){wave_shr1(out.x), wave_shr1(out.y)};
  }
  // LDS-only barrier: __syncthreads() would also drain vmcnt, i.e. wait for
  // the next sweep's reflector prefetch issued above
  kfac_lds_barrier();
  // thread 0 takes the untouched Z[k][s] (lane PH of wave 0's block copy)
#pragma unroll
  for (int p = 0; p < QP; ++p) {
    const float z0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(S.zc[2 * p]), PH));
    const float z1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(S.zc[2 * p + 1]), PH));
    if (lane == 0)
      S.z[p][PH] = (w == 0) ? (f2){z0, z1} : (f2){buf[w - 1][2 * p], buf[w - 1][2 * p + 1]};
  }
}

__global__ __launch_bounds__(QT) void q2_kernel(const Q2Mat* __restrict__ mats,
                                                const int* __restrict__ offs, int count) {
  int blk;
  const Q2Mat M = mats[find_mat(offs, count, blockIdx.x, &blk)];
  const int n = M.n;
  const int t = threadIdx.x;
  const int k0 = blk * QR;
  __shared__ float sx[2][QW][QR];
  AS1 float* Z = gptr(M.Z);
  Q2State S;
  const int s0 = n - 3;
  // window of sweep s0: components s0+1+16t .. s0+16+16t, component x in slot x & 15
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int x = s0 + 1 + 16 * t + ((k - (s0 + 1)) & 15);
#pragma unroll
    for (int p = 0; p < QP; ++p) {
      const int r = 2 * p;
      const bool ok = x < n && s0 >= 0;
      S.z[p][k] = (f2){gld_if(Z, (long long)(k0 + r) * M.ldz + x, ok && k0 + r < n, 0.f),
                       gld_if(Z, (long long)(k0 + r + 1) * M.ldz + x, ok && k0 + r + 1 < n, 0.f)};
    }
  }
  if (s0 >= 0) {
    const __amdgpu_buffer_rsrc_t rsv = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(M.v2), 0, (int)((long long)(n - 1) * M.ldv2 * 4), 0x00020000);
    const int vof = (16 * t < n) ? 64 * t : 0x7ffffff0;
    const int ldv4 = (int)M.ldv2 * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      S.vn[c] = __builtin_amdgcn_raw_buffer_load_b128(rsv, vof + 16 * c, s0 * ldv4, 0);
    // blocks of 16 sweeps (phase PH = s mod 16 static in each unrolled body),
    // sweeps outside [0, s0] skipped (uniform)
    // wave 0, lane l < 16 keeps Z[k][base + l] of the current block (the
    // components thread 0 takes in over the block's 16 sweeps), the next
    // block's copy loaded one block ahead
    const int lane = t & 63;
    auto zblock = [&](int bs, float (&dst)[QR]) {
#pragma unroll
      for (int r = 0; r < QR; ++r) {
        const bool ok = t < 16 && bs >= 0 && k0 + r < n;
        dst[r] = gld_if(Z, (long long)(k0 + r) * M.ldz + bs + lane, ok, 0.f);
      }
    };
    zblock(s0 & ~15, S.zc);
#pragma unroll 1
    for (int base = s0 & ~15; base >= 0; base -= 16) {
      float zn[QR];
      zblock(base - 16, zn);
#define Q2_STEP(PH)                                                   \
      if (base + PH <= s0) q2_sweep<PH>(S, base + PH, t, rsv, vof, ldv4, sx);
      Q2_STEP(15) Q2_STEP(14) Q2_STEP(13) Q2_STEP(12) Q2_STEP(11) Q2_STEP(10) Q2_STEP(9)
      Q2_STEP(8) Q2_STEP(7) Q2_STEP(6) Q2_STEP(5) Q2_STEP(4) Q2_STEP(3) Q2_STEP(2)
      Q2_STEP(1) Q2_STEP(0)
#undef Q2_STEP
#pragma unroll
      for (int r = 0; r < QR; ++r) S.zc[r] = zn[r];
    }
  }
  // after sweep 0 the window is components 16t .. 16t + 15 (slot k = component 16t + k);
  // for n <= 2 nothing moved and the same holds (s0 < 0: loaded as zero, skip)
  if (s0 < 0) return;
  if (16 * t >= n) return;
#pragma unroll
  for (int r = 0; r < QR; ++r) {
    if (k0 + r >= n) continue;
    AS1 float* o = Z + (long long)(k0 + r) * M.ldz + 16 * t;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      fx4 a;
      const int p = r >> 1;
      a.x = (r & 1) ? S.z[p][4 * c + 0].y : S.z[p][4 * c + 0].x;
      a.y = (r & 1) ? S.z[p][4 * c + 1].y : S.z[p][4 * c + 1].x;
      a.z = (r & 1) ? S.z[p][4 * c + 2].y : S.z[p][4 * c + 2].x;
      a.w = (r & 1) ? S.z[p][4 * c + 3].y : S.z[p][4 * c + 3].x;
      *(AS1 fx4*)(o + 4 * c) = a;
    }
  }
}

struct Q2Plan {
  Q2Mat* d_mats = nullptr;
  int* d_offs = nullptr;
  int count = 0, grid = 0;
  hipGraphExec_t exec = nullptr;
};

int enqueue(const Q2Plan& P, hipStream_t s) {
  hipLaunchKernelGGL(q2_kernel, dim3(P.grid), dim3(QT), 0, s, P.d_mats, P.d_offs, P.count);
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, Q2Plan> g_plans;

}  // namespace

struct KfacQ2Record { float* Z; const float* v2; long long ldz, ldv2, n; };

KFAC_API int kfac_q2_nmax() { return 16 * (QT - 1) < 5120 ? 16 * (QT - 1) : 5120; }

// Z (n rows of ldz floats: eigenvectors as rows) <- rows of (Q2 Z^T)^T for
// `count` matrices; v2 ((n-1) x ldv2, segment layout) from kfac_sb2st_batched.
// ldz >= 16 * (ceil(n / 16) + 1) (the sliding windows read/write up to there
// as zero padding), ldv2 >= 16 * (ceil(n / 16) + 1).
KFAC_API int kfac_q2_batched(const KfacQ2Record* recs, int count, int use_graph,
                             hipStream_t stream) {
  if (count <= 0) return 0;
  std::vector<Q2Mat> mats(count);
  std::vector<int> offs(count + 1, 0);
  for (int i = 0; i < count; ++i) {
    const KfacQ2Record& r = recs[i];
    const long long need = 16LL * ((r.n + 15) / 16 + 1);
    if (r.n < 2 || r.n > 5120 || r.ldz % 16 || r.ldz < r.n || r.ldv2 % 16 || r.ldv2 < need)
      return -2;
    Q2Mat& M = mats[i];
    memset(&M, 0, sizeof(M));
    M.Z = r.Z; M.v2 = r.v2; M.ldz = r.ldz; M.ldv2 = r.ldv2; M.n = (int)r.n;
    offs[i + 1] = offs[i] + (int)((r.n + QR - 1) / QR);
  }
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  const std::string key((const char*)mats.data(), sizeof(Q2Mat) * mats.size());
  Q2Plan* plan;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      Q2Plan P;
      P.count = count;
      P.grid = offs[count];
      int err;
      if ((err = (int)hipMalloc(&P.d_mats, sizeof(Q2Mat) * count)) != 0) return err;
      if ((err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(Q2Mat) * count,
                                hipMemcpyHostToDevice)) != 0)
        return err;
      if ((err = (int)hipMalloc(&P.d_offs, sizeof(int) * (count + 1))) != 0) return err;
      if ((err = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * (count + 1),
                                hipMemcpyHostToDevice)) != 0)
        return err;
      it = g_plans.emplace(key, P).first;
    }
    plan = &it->second;
    if (graph && !plan->exec) {
      static hipStream_t cap = nullptr;
      if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
      hipGraph_t gr = nullptr;
      if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
        const int e1 = enqueue(*plan, cap);
        const hipError_t e2 = hipStreamEndCapture(cap, &gr);
        if (!e1 && e2 == hipSuccess && gr &&
            hipGraphInstantiate(&plan->exec, gr, nullptr, nullptr, 0) != hipSuccess)
          plan->exec = nullptr;
        if (gr) (void)hipGraphDestroy(gr);
      }
      (void)hipGetLastError();
    }
  }
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}
