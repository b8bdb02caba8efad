// Band -> tridiagonal reduction (stage 2 of the two-stage symmetric
// eigensolver; reference: kfac/layers/utils.py:45-74 calls
// torch.symeig per factor).  Stage 1 (csrc/eig_sy2sb.hip) leaves a band of
// half-bandwidth BW = 16; here every sweep s annihilates column s below the
// subdiagonal with a Householder reflector of length <= BW and chases the
// bulge it creates down the band, one task (s, j) per step j:
//
//   task (s, j):  c = s (j = 0) or s + 1 + (j-1) BW,  rows R = s+1+j BW ..
//                 s+(j+1) BW.  x = B[R, c] -> reflector (v, tau); B <- H B H
//                 on the stored lower band: column c, the bulge block
//                 B[R, c+1 .. r0-1] (left), the diagonal block B[R, R] (both
//                 sides), the block below B[r1+1 .. r1+BW, R] (right: the next
//                 bulge).
//
// Task (s+1, j) may run once (s, j+2) is done: at tick 3 s + j every task
// touches a disjoint region (scripts/models/two_stage_model.py checks the
// wavefront order against the sweep-by-sweep order in fp64).
//
// MI355X mapping: one 1024-thread workgroup runs 16 consecutive sweeps, one
// per wave, in lockstep ticks (wave w runs step t - 3w at tick t, one
// workgroup barrier per tick) on an LDS-resident window of the band: 1024
// columns x 2 BW diagonals, circular, 128 KB of the 160 KB LDS.  Block t+4
// of the band streams in from global memory while tick t computes (two
// register sets: the loads have a tick to land); columns no sweep of the
// workgroup will touch again are written back and published with an
// agent-scope release.  Workgroup g+1 (the next 16 sweeps) trails g by ~48
// ticks and waits (acquire, bounded spin) for the columns it needs: a
// pipeline of workgroups down each matrix, every matrix of the batch at
// once.  A workgroup only ever waits on the previous workgroup of its own
// matrix, and the launch table orders workgroups by their start tick, so
// in-order dispatch always makes progress; every spin is bounded (error flag
// + release of the successor) so a fault cannot leave waves running.
//
// Output: d, e of the tridiagonal matrix and the reflectors for the
// back-transformation (csrc/eig_q2.hip): row s of V2 holds sweep s's steps,
// step j at [j BW, (j+1) BW): tau in slot 0 (v[0] = 1 is implicit), v[1..].
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int BW = 16;             // half-bandwidth of the stage-1 band
constexpr int ND = 2 * BW;         // stored diagonals per column (band + bulge room)
constexpr int NSW = 16;            // sweeps (waves) per workgroup
constexpr int WIN = 1024;          // LDS window columns (circular)
constexpr int PD = 6;              // prefetch register sets: a band block is in flight PD-1 ticks
constexpr int LAG = PD + 1;        // band block prefetched LAG ticks ahead
constexpr int RET = 8;             // columns retired / published every RET ticks
constexpr int SPIN_MAX = 1 << 22;  // bounded waits (~1 s): a lost predecessor cannot hang the GPU

struct SbMat {
  float* band;   // n x ND, column-major band: band[c * ND + (r - c)]
  float* v2;     // n x ldv2 reflector rows
  float* d;
  float* e;
  int* prog;     // [nwg] published retire boundary (columns < prog[g] final)
  int n, ldv2, nwg, pad;
};
struct SbWg { int mat, g; };

// debug: phase stamps (s_memrealtime, 100 MHz) of one workgroup's first ticks
__device__ unsigned long long* g_sb_stamps = nullptr;
__device__ int g_sb_stamp_wg = 0;
#define SB_STAMP(k)                                                                 \
  do {                                                                              \
    if (stamps && tid == 0 && t < 512) stamps[t * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__device__ __forceinline__ float& LB(float* Lb, int r, int c) {
  return Lb[((c & (WIN - 1)) * ND) + (r - c)];
}

// sum over the 16-lane row of the wave (DPP only; every lane of the row ends
// with the row's sum)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);    // row_half_mirror
  v += dpp_f<0x140>(v);    // row_mirror
  return v;
}

// one bulge-chasing step of sweep s, by one wave; false when the sweep has
// run off the end of the matrix.  After the reflector (lanes 0..15), the
// three independent updates run side by side on the wave's 16-lane rows:
// lanes 0..15 the diagonal block (both sides), 16..31 the bulge block
// (left), 32..47 the block below (right) -- one pass of 16 LDS loads and
// stores instead of three.
__device__ bool sb_task(float* Lb, int n, int s, int j, AS1 float* v2row, int lane) {
  const int c = j == 0 ? s : s + 1 + (j - 1) * BW;
  const int r0 = s + 1 + j * BW;
  const int r1 = min(s + (j + 1) * BW, n - 1);
  const int L = r1 - r0 + 1;
  if (r0 > n - 1 || L < 2) return false;
  const float xl = Lb[lane < L ? ((c & (WIN - 1)) * ND + (r0 + lane - c)) : 0];
  const float x = lane < L ? xl : 0.f;
  const float alpha = __shfl(x, 0, 64);
  const float sig = wave_sum(lane >= 1 && lane < L ? x * x : 0.f);
  float tau = 0.f, beta = alpha, scal = 0.f;
  if (sig != 0.f) {
    beta = -copysignf(sqrtf(alpha * alpha + sig), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.f / (alpha - beta);
  }
  const float v = lane == 0 ? 1.f : (lane < L ? x * scal : 0.f);
  if (lane < L) LB(Lb, r0 + lane, c) = lane == 0 ? beta : 0.f;
  if (lane < BW) v2row[j * BW + lane] = lane == 0 ? tau : v;
  if (tau == 0.f) return true;
  float vl[BW];
#pragma unroll
  for (int l = 0; l < BW; ++l) vl[l] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
  const int grp = lane >> 4, li = lane & 15;
  const int nq = r0 - 1 - c;                     // bulge block columns (BW-1 for j >= 1)
  const int nE = min(BW, n - 1 - r1);            // rows below R in the band
  // per-lane element (row, col) of entry l, and whether this lane is active
  bool act;
  if (grp == 0) act = li < L;
  else if (grp == 1) act = li < nq;
  else if (grp == 2) act = li < nE;
  else act = false;
  float val[BW];
  float acc = 0.f;
#pragma unroll
  for (int l = 0; l < BW; ++l) {
    // element of entry l for this lane's group, as selects (no divergent branch)
    const int rr = grp == 0 ? r0 + max(li, l) : (grp == 1 ? r0 + l : r1 + 1 + li);
    const int cc = grp == 0 ? r0 + min(li, l) : (grp == 1 ? c + 1 + li : r0 + l);
    const bool ok = act && l < L;
    // branch-free: inactive lanes read slot 0 (a conditional load becomes a
    // branch with its own LDS wait, serialising the 16 loads)
    const int ad = ok ? (((cc & (WIN - 1)) * ND) + (rr - cc)) : 0;
    const float ld = Lb[ad];
    val[l] = ok ? ld : 0.f;
    acc += val[l] * vl[l];
  }
  acc *= tau;                                    // p (diag lanes), y (bulge), z (below)
  // diagonal block: w = p - tau/2 (p . v) v over the 16-lane row
  const float va = (grp == 0 && li < L) ? v : 0.f;
  const float pv = row_sum16(acc * va);
  const float w = (grp == 0 && li < L) ? acc - 0.5f * tau * pv * va : 0.f;
  float wl[BW];
#pragma unroll
  for (int l = 0; l < BW; ++l) wl[l] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), l));
  // new = val - c1 X[l] - c2 v[l]:  diag: c1 = v_a, X = w, c2 = w_a;  others: c1 = 0, c2 = acc
  const float c1 = grp == 0 ? va : 0.f;
  const float c2 = grp == 0 ? w : acc;
#pragma unroll
  for (int l = 0; l < BW; ++l) {
    // diagonal group: lower entry (li, l), l <= li
    const int rr = grp == 0 ? r0 + li : (grp == 1 ? r0 + l : r1 + 1 + li);
    const int cc = grp == 0 ? r0 + l : (grp == 1 ? c + 1 + li : r0 + l);
    const bool ok = act && l < L && (grp != 0 || l <= li);
    const float nv = val[l] - c1 * wl[l] - c2 * vl[l];
    if (ok) Lb[((cc & (WIN - 1)) * ND) + (rr - cc)] = nv;
  }
  return true;
}

// Cross-workgroup data (band columns, progress counters) moves through
// agent-scope RELAXED atomics: on gfx950 these are plain loads / stores with
// the coherence bit, which write through / read around the per-XCD L2, so no
// L2 writeback or invalidate (what agent-scope acquire / release fences cost,
// every tick, for every workgroup) is needed.  Ordering: the writer waits for
// its band stores to complete (s_waitcnt) before the barrier that precedes
// the counter store; the reader loads band columns only after the barrier
// that follows its counter load.
// Global (not flat) address space: a flat load also counts in lgkmcnt, so
// every LDS wait of the tick would wait for the band prefetches too.
__device__ __forceinline__ float band_ld(const float* p) {
  return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void band_st(float* p, float v) {
  __hip_atomic_store(gptr(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int task_min_col(int s, int j) {
  return j == 0 ? s : s + 1 + (j - 1) * BW;
}

// wait (thread 0 only) until the previous workgroup of this matrix has
// published columns < need; the published value, or -1 on timeout
__device__ int wait_prog(const int* prog, int need) {
  for (int it = 0; it < SPIN_MAX; ++it) {
    const int v = __hip_atomic_load(gptr(prog), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v >= need) return v;
    __builtin_amdgcn_s_sleep(4);
  }
  return -1;
}

__global__ __launch_bounds__(1024) void sb2st_kernel(const SbMat* __restrict__ mats,
                                                     const SbWg* __restrict__ wgs,
                                                     int* __restrict__ err) {
  extern __shared__ float Lb[];                 // WIN x ND
  __shared__ int s_done[NSW];
  __shared__ int s_flag;
  __shared__ int s_pc;                          // last seen progress of the previous workgroup
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const SbWg W = wgs[blockIdx.x];
  const SbMat M = mats[W.mat];
  unsigned long long* const stamps = ((int)blockIdx.x == g_sb_stamp_wg) ? g_sb_stamps : nullptr;
  const int n = M.n, g = W.g, s0 = g * NSW;
  const int* prev = g > 0 ? M.prog + g - 1 : nullptr;
  int* const mine = M.prog + g;
  if (tid < NSW) s_done[tid] = (s0 + tid > n - 2) ? 1 : 0;
  if (tid == 0) {
    s_flag = 0;
    s_pc = n;
    if (prev) {
      s_pc = wait_prog(prev, min(n, s0 + LAG * BW));
      if (s_pc < 0) {
        s_flag = 1;
        atomicOr(err, 1);
      }
    }
  }
  const int cl = tid >> 5, dl = tid & 31;       // thread's (column, diagonal) in a 32-column slab
  __syncthreads();
  if (s_flag) {
    if (tid == 0) __hip_atomic_store(gptr(mine), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // Band block b (columns s0 + 16 b ..) is loaded at tick b - LAG into
  // register set (b - LAG) mod PD and committed to LDS at the end of tick
  // b - LAG + PD - 1; wave 0 needs it at tick b - 1.  Blocks 0 .. LAG-PD load
  // synchronously, LAG-PD+1 .. LAG-1 are issued before tick 0.
  const bool pth = tid < BW * ND;               // threads that move band data (16 columns x 32)
  for (int c = s0 + cl; c < min(n, s0 + (LAG - PD + 1) * BW); c += 32)
    LB(Lb, c + dl, c) = band_ld(M.band + (long long)c * ND + dl);
  float pre[PD];
#pragma unroll
  for (int u = 0; u < PD; ++u) pre[u] = 0.f;
#pragma unroll
  for (int u = 1; u < PD; ++u) {                // set u <- block LAG - PD + u
    const int c = s0 + (LAG - PD + u) * BW + (tid >> 5);
    if (pth && c < n) pre[u] = band_ld(M.band + (long long)c * ND + dl);
  }
  int retired = s0;
  __syncthreads();
  for (int t0 = 0;; t0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {              // t = t0 + u, register set u is t mod PD
      const int t = t0 + u;
      SB_STAMP(0);
      // (1) issue block t + LAG (published by the previous workgroup)
      const int pc0 = s0 + (t + LAG) * BW;
      if (pc0 < n) {
        const int need = min(n, pc0 + BW);
        if (need > s_pc) {             // uniform: s_pc changes only here, between barriers
          if (tid == 0) {
            const int v = wait_prog(prev, need);
            if (v < 0) {
              s_flag = 1;
              atomicOr(err, 1);
            } else {
              s_pc = v;
            }
          }
          __syncthreads();
          if (s_flag) goto abort;
        }
        const int c = pc0 + (tid >> 5);
        if (pth && c < n) pre[u] = band_ld(M.band + (long long)c * ND + dl);
      }
      SB_STAMP(1);
      // (2) one step of every active sweep (disjoint regions within the tick)
      {
        const int s = s0 + wave, j = t - 3 * wave;
        if (!s_done[wave] && j >= 0) {
          const bool more = sb_task(Lb, n, s, j, gptr(M.v2) + (long long)s * M.ldv2, lane);
          if (!more && lane == 0) s_done[wave] = 1;
        }
      }
      kfac_lds_barrier();
      SB_STAMP(2);
      // (3) commit block t + LAG - PD + 1 (issued PD - 1 ticks ago, set (u + 1) mod PD)
      {
        const int cc0 = s0 + (t + LAG - PD + 1) * BW;
        const int c = cc0 + (tid >> 5);
        if (pth && c < n) LB(Lb, c + dl, c) = pre[(u + 1) % PD];
      }
      kfac_lds_barrier();
      SB_STAMP(3);
      // (4) retire: columns below every unfinished sweep's next task
      int all_done = 1, bound = n;
#pragma unroll
      for (int w = 0; w < NSW; ++w) {
        if (!s_done[w]) {
          all_done = 0;
          const int jn = max(t + 1 - 3 * w, 0);
          bound = min(bound, task_min_col(s0 + w, jn));
        }
      }
      bound = min(bound, min(n, s0 + (t + LAG - PD + 2) * BW));   // never past the committed columns
      if (all_done) bound = n;
      if (bound > retired && ((t % RET) == RET - 1 || all_done)) {
        for (int c = retired + cl; c < bound; c += 32)
          band_st(M.band + (long long)c * ND + dl, LB(Lb, c + dl, c));
        retired = bound;
        __builtin_amdgcn_s_waitcnt(0);     // this wave's band stores have completed
        __syncthreads();
        if (tid == 0) __hip_atomic_store(gptr(mine), retired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      SB_STAMP(4);
      if (all_done) return;
      kfac_lds_barrier();
    }
  }
abort:
  // release the successor (its results are garbage, err is set)
  if (tid == 0) __hip_atomic_store(gptr(mine), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void sb2st_prep_kernel(const SbMat* __restrict__ mats) {
  const SbMat M = mats[blockIdx.y];
  for (int g = blockIdx.x * 256 + threadIdx.x; g < M.nwg; g += gridDim.x * 256) M.prog[g] = 0;
}

__global__ __launch_bounds__(256) void sb2st_de_kernel(const SbMat* __restrict__ mats) {
  const SbMat M = mats[blockIdx.y];
  for (int c = blockIdx.x * 256 + threadIdx.x; c < M.n; c += gridDim.x * 256) {
    M.d[c] = M.band[(long long)c * ND];
    M.e[c] = c + 1 < M.n ? M.band[(long long)c * ND + 1] : 0.f;
  }
}

struct SbPlan {
  SbMat* d_mats = nullptr;
  SbWg* d_wgs = nullptr;
  int count = 0, nwg = 0, maxn = 0;
};
std::mutex g_mu;
std::map<std::string, SbPlan> g_plans;

}  // namespace

struct KfacSbRecord {
  float* band; float* v2; float* d; float* e; int* prog; long long n; long long ldv2;
};

KFAC_API int kfac_sb2st_bw() { return BW; }

// debug: stamps of workgroup `wg` (launch order) into buf (512 ticks x 8), or off
KFAC_API int kfac_sb2st_stamps(unsigned long long* buf, int wg) {
  int e = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sb_stamps), &buf, sizeof(buf));
  if (!e) e = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sb_stamp_wg), &wg, sizeof(wg));
  return e;
}
KFAC_API long long kfac_sb2st_ldv2(int n) { return ((long long)n + 2 * BW + 15) / 16 * 16; }
KFAC_API int kfac_sb2st_nwg(int n) { return (n - 1 + NSW - 1) / NSW; }

// Band (n x 2BW column-major, lower band in diagonals 0..BW, zeros above)
// -> d, e and the bulge-chasing reflectors, every matrix of the batch in one
// persistent launch.  err: device int, OR-ed with 1 if a wait timed out.
KFAC_API int kfac_sb2st_batched(const KfacSbRecord* recs, int count, int* err,
                                hipStream_t stream) {
  if (count <= 0) return 0;
  std::vector<SbMat> mats(count);
  for (int i = 0; i < count; ++i) {
    const KfacSbRecord& r = recs[i];
    if (r.n < 2 || r.ldv2 < kfac_sb2st_ldv2((int)r.n)) return -2;
    SbMat& M = mats[i];
    memset(&M, 0, sizeof(M));
    M.band = r.band; M.v2 = r.v2; M.d = r.d; M.e = r.e; M.prog = r.prog;
    M.n = (int)r.n; M.ldv2 = (int)r.ldv2; M.nwg = kfac_sb2st_nwg((int)r.n);
  }
  const std::string key((const char*)mats.data(), sizeof(SbMat) * mats.size());
  SbPlan* P;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      SbPlan p;
      p.count = count;
      std::vector<SbWg> wgs;
      int gmax = 0;
      for (auto& M : mats) { gmax = std::max(gmax, M.nwg); p.maxn = std::max(p.maxn, M.n); }
      for (int g = 0; g < gmax; ++g)          // start-tick order: g major
        for (int i = 0; i < count; ++i)
          if (g < mats[i].nwg) wgs.push_back(SbWg{i, g});
      p.nwg = (int)wgs.size();
      int e1 = (int)hipMalloc(&p.d_mats, sizeof(SbMat) * count);
      if (!e1) e1 = (int)hipMemcpy(p.d_mats, mats.data(), sizeof(SbMat) * count, hipMemcpyHostToDevice);
      if (!e1) e1 = (int)hipMalloc(&p.d_wgs, sizeof(SbWg) * wgs.size());
      if (!e1) e1 = (int)hipMemcpy(p.d_wgs, wgs.data(), sizeof(SbWg) * wgs.size(), hipMemcpyHostToDevice);
      if (e1) return e1;
      static bool attr = false;
      if (!attr) {
        e1 = (int)hipFuncSetAttribute((const void*)sb2st_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      WIN * ND * (int)sizeof(float));
        if (e1) return e1;
        attr = true;
      }
      it = g_plans.emplace(key, p).first;
    }
    P = &it->second;
  }
  int gmax = 0;
  for (auto& M : mats) gmax = std::max(gmax, M.nwg);
  hipLaunchKernelGGL(sb2st_prep_kernel, dim3((gmax + 255) / 256, count), dim3(256), 0, stream,
                     P->d_mats);
  hipLaunchKernelGGL(sb2st_kernel, dim3(P->nwg), dim3(1024), WIN * ND * sizeof(float), stream,
                     P->d_mats, P->d_wgs, err);
  hipLaunchKernelGGL(sb2st_de_kernel, dim3((P->maxn + 255) / 256, count), dim3(256), 0, stream,
                     P->d_mats);
  return (int)hipGetLastError();
}
