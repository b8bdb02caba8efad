// Stage 1 of the two-stage symmetric eigensolver: dense -> band of
// half-bandwidth SB = 16 (reference semantics
// kfac/layers/utils.py:45-74, the factor's eigendecomposition).
//
// Why two stages on MI355X: the one-stage reduction (csrc/eig_reduce.hip)
// reads the whole trailing matrix once per COLUMN (a symmetric mat-vec per
// column, ~196 GB for ResNet-50's three 4608 factors) and pays two dependent
// launches per column.  Here the trailing matrix is read / written three
// times per PANEL of 16 columns (a 16-wide GEMM and a rank-32 update): 16x
// fewer passes, and the dependent chain is 288 panels long instead of 4608
// columns.  The band is finished by bulge chasing (csrc/eig_sb2st.hip).
//
// Storage (row-major, every matrix of the batch):  A lda x lda, FULL
// symmetric (both triangles maintained), zero outside n x n; lda a multiple of
// 128.  Panel p = rows j0 = 16 p .. j0 + 15; its columns j0 + 16 .. n - 1 are
// QR-factorised as 16 row vectors (the transpose of LAPACK's column panel).
// Reflector j = j0 + c stays in row j: beta at column j + 16, v[1:] after it
// -- exactly the layout the compact-WY back-transformation reads with shift
// 16 (csrc/eig_backtransform.hip) -- and tau[j].  The exact operation order is
// modelled in fp64 by scripts/models/two_stage_model.py (sy2sb).
//
// Per panel, one launch each (all matrices of the batch in every launch):
//   P  one 512-thread workgroup per matrix: the 16 x m panel in registers
//      (10 columns per thread), Householder QR with ONE workgroup reduction
//      per reflector (the dots of row c's tail with every panel row: its norm,
//      the trailing rows' update coefficients and the new column of V^T V
//      for T), T (larft) built alongside; V rows -> Vr
//   Y  X = A22 V T, 16 rows per workgroup on v_mfma_f32_16x16x4_f32 (exact
//      f32), 4 waves split K; per-workgroup partial M = V^T X
//   N  N = T^T (sum of the partial M) -- one small workgroup per matrix
//   U  A22 -= Zm V^T + V Zm^T with Zm = X - V N / 2 computed per tile from
//      X, V, N (64 x 64 tiles, both triangles)
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int SB = 16;             // half-bandwidth of the band
constexpr int PT = 512;            // panel workgroup threads
constexpr int PQ = 10;             // panel columns per thread: m <= PT * PQ
constexpr int NMAX2 = PT * PQ;       // largest n of the two-stage path (5120; Q2 holds 16 components per thread)
constexpr int UT = 64;             // update tile
constexpr int MAXM2 = 64;          // matrices per launch sequence

struct SyMat {
  float* A; float* tau; float* band;
  float* Vr;   // SB x lda: reflector rows of the current panel (v[0] = 1 explicit, 0 before)
  float* X;    // lda x SB
  float* Mp;   // (lda / 16) x 256 partial V^T X
  float* T;    // 16 x 16
  float* N;    // 16 x 16
  long long lda;
  int n, pad;
};

inline long long a64(long long x) { return (x + 63) / 64 * 64; }

struct SyWs { long long Vr, X, Mp, T, N, total; };
SyWs ws_layout(long long lda) {
  SyWs L;
  long long o = 0;
  L.Vr = o; o += a64(SB * lda);
  L.X = o; o += a64(lda * SB);
  L.Mp = o; o += a64((lda / 16 + 1) * 256);
  L.T = o; o += 256;
  L.N = o; o += 256;
  L.total = o;
  return L;
}

// matrix of this workgroup from a launch's ascending offsets (count + 1)
// (the matrices are sorted by descending n, so the active ones of a panel are
// a prefix: the active index is the matrix index)
__device__ __forceinline__ bool r_ok(int r, int nr) { return r < nr; }

__device__ __forceinline__ int find_mat(const int* __restrict__ offs, int count, int wg,
                                        int* local) {
  int lo = 0;
  for (int i = 1; i < count; ++i)
    if (offs[i] <= wg) lo = i;
  *local = wg - offs[lo];
  return lo;
}

// ------------------------------------------------------------------- P
__global__ __launch_bounds__(PT) __attribute__((amdgpu_waves_per_eu(1, 2))) void sy2sb_panel_kernel(const SyMat* __restrict__ mats,
                                                         const int* __restrict__ act, int p) {
  const SyMat M = mats[act[blockIdx.x]];
  const int n = M.n;
  const long long lda = M.lda;
  const int j0 = p * SB, m = n - j0 - SB;
  if (m < 1) return;
  const int kb = m < SB ? m : SB;
  const int nr = (n - j0) < SB ? (n - j0) : SB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NW = PT / 64;
  AS1 float* A = gptr(M.A);
  AS1 float* Vr = gptr(M.Vr);
  __shared__ __attribute__((aligned(16))) float red16[2][NW][SB];
  __shared__ __attribute__((aligned(16))) float colc[2][SB];
  __shared__ float sT[SB][SB + 1];
  for (int e = tid; e < SB * (SB + 1); e += PT) (&sT[0][0])[e] = 0.f;

  // buffer addressing (one voffset per thread, uniform row / column offsets):
  // 64-bit per-element addresses, shared by the loads and the final stores,
  // kept ~100 VGPRs live and spilled the panel
  const long long base = (long long)j0 * lda + j0 + SB;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      M.A + base, 0, (int)(((long long)(nr - 1) * lda + m) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc(
      M.Vr, 0, (int)((long long)SB * lda * 4), 0x00020000);
  const int vo = tid * 4, ldi = (int)lda;
  float P[SB][PQ];
#pragma unroll
  for (int c = 0; c < SB; ++c)
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int k = tid + PT * q;
      const bool ok = c < nr && k < m;
      const float x = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(rsA, vo, (int)((c * lda + PT * q) * 4), 0));
      P[c][q] = ok ? x : 0.f;
    }
  __syncthreads();     // sT zeroed

  // fully unrolled over the panel rows: every P[c][q] index is static, so the
  // panel stays in registers (a runtime row index puts it in scratch).
  // ONE workgroup reduction (and one barrier) per reflector: the dots
  // e_r = sum_{k > c} P[c][k] P[r][k] of row c's tail with every panel row,
  // plus column c (thread c) through LDS, give
  //   sig = e_c,  alpha = P[c][c],  and for r != c
  //   d_r = sum_{k >= c} v[k] P[r][k] = P[r][c] + scal e_r
  // -- the update coefficients (r > c) and V^T v for T (r < c), as before.
#pragma clang loop unroll(full)
  for (int c = 0; c < SB; ++c) {
    if (c < kb) {                             // kb is uniform
    const int b = c & 1;
    float e[SB];
#pragma unroll
    for (int r = 0; r < SB; ++r) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const float x = (q == 0 && tid <= c) ? 0.f : P[c][q];   // k > c
        s = __builtin_fmaf(x, P[r][q], s);
      }
      e[r] = r < nr ? s : 0.f;
    }
    const float esum = kfac_butterfly16(e);   // lanes with (lane & 15) == x: wave sum of e[x]
    if (lane < SB) red16[b][wid][lane] = esum;
    if (tid == c) {                           // column c: thread c, q = 0
#pragma unroll
      for (int r = 0; r < SB; ++r) colc[b][r] = P[r][0];
    }
    kfac_lds_barrier();      // LDS only: the Vr stores stay in flight
    // lane l (every wave) sums the 8 wave partials of e_{l & 15}; the row
    // coefficients then go to scalar registers by readlane
    float el = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) el += red16[b][w][lane & 15];
    const float pl = colc[b][lane & 15];
    const float sig = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(el), c));
    const float alpha = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), c));
    float tau = 0.f, beta = alpha, scal = 0.f;
    if (sig != 0.f) {
      beta = -copysignf(sqrtf(alpha * alpha + sig), alpha);
      tau = (beta - alpha) / beta;
      scal = 1.f / (alpha - beta);
    }
    // d_l = P[l][c] + scal e_l: update coefficient of row l > c, (V^T v)_l for l < c
    const float dl = pl + scal * el;
    float v[PQ];
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int k = tid + PT * q;
      v[q] = k < c ? 0.f : (k == c ? 1.f : P[c][q] * scal);
    }
    // -- update the rows below
#pragma unroll
    for (int r = 0; r < SB; ++r) {
      if (r > c) {
        const float f = tau * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dl), r));
#pragma unroll
        for (int q = 0; q < PQ; ++q) P[r][q] = __builtin_fmaf(-f, v[q], P[r][q]);
      }
    }
    // -- finish row c (R before, beta, v after)
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int k = tid + PT * q;
      P[c][q] = k == c ? beta : (k > c ? v[q] : P[c][q]);
      if (k < ldi)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[q]), rsV, vo,
                                              (int)((c * lda + PT * q) * 4), 0);
    }
    // -- T column c (larft, forward columnwise): T[0:c, c] = -tau T[0:c, 0:c] (V^T v),
    // (V^T v)_a = d_a for a < c; wave 0, lane a computes d_a (lane tid owns row
    // tid of sT: written and read by the same lane)
    if (wid == 0 && c > 0) {
      float s = 0.f;
#pragma unroll
      for (int a = 0; a < SB; ++a) {
        if (a < c) {
          const float x = (r_ok(a, nr)) ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dl), a)) : 0.f;
          s += (a >= lane) ? sT[lane & 15][a] * x : 0.f;
        }
      }
      if (lane < c) sT[lane][c] = -tau * s;
    }
    if (tid == c) sT[c][c] = tau;
    if (tid == 0) M.tau[j0 + c] = tau;
    }
  }
  // rows without a reflector (short last panel): tau 0, V rows 0
  for (int c = kb; c < SB; ++c) {
    if (tid == 0 && j0 + c < n) M.tau[j0 + c] = 0.f;
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int k = tid + PT * q;
      if (k < ldi)
        __builtin_amdgcn_raw_buffer_store_b32(0u, rsV, vo, (int)((c * lda + PT * q) * 4), 0);
    }
  }
#pragma unroll
  for (int c = 0; c < SB; ++c)
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int k = tid + PT * q;
      if (c < nr && k < m)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(P[c][q]), rsA, vo,
                                              (int)((c * lda + PT * q) * 4), 0);
    }
  __syncthreads();
  if (tid < SB * SB) M.T[tid] = sT[tid / SB][tid % SB];
}

// ------------------------------------------------------------------- Y
// X = A22 V T for 16 rows of A22 per workgroup (exact f32 MFMA 16x16x4; the
// 4 waves take quarters of K), and this block's partial M = V^T X.
// v_mfma_f32_16x16x4_f32: lane l supplies A[l % 16][l / 16] and
// B[l / 16][l % 16] and holds D[4 (l / 16) + t][l % 16], t = 0..3.  Each lane
// loads 4 consecutive k of its row (a float4) and feeds them to 4 MFMAs: the
// k <-> (lane, instruction) assignment is the same for A and B, so the sum is
// the plain dot product.
__global__ __launch_bounds__(256) void sy2sb_yx_kernel(const SyMat* __restrict__ mats,
                                                       const int* __restrict__ offs, int count,
                                                       int p) {
  int blk;
  const SyMat M = mats[find_mat(offs, count, blockIdx.x, &blk)];
  const int n = M.n;
  const long long lda = M.lda;
  const int j0 = p * SB, m = n - j0 - SB;
  const int mk = (m + 15) / 16 * 16;
  const int row0 = blk * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  __shared__ float sY[4][16][17];
  __shared__ float sYt[16][17];
  __shared__ float sX[16][17];
  __shared__ float sTT[16][17];
  const AS1 float* Arow = gptr(M.A) + (long long)(j0 + SB + row0 + i) * lda + j0 + SB;
  const AS1 float* Vrow = gptr(M.Vr) + (long long)i * lda;
  const int chunk = ((mk / 16 + 3) / 4) * 16;
  const int kbeg = wid * chunk, kend = min(mk, kbeg + chunk);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  int k0 = kbeg;
  // 4 k-steps per iteration: 8 float4 loads in flight before the MFMAs
  for (; k0 + 64 <= kend; k0 += 64) {
    fx4 a4[4], b4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a4[u] = *(const AS1 fx4*)(Arow + k0 + 16 * u + 4 * q);
      b4[u] = *(const AS1 fx4*)(Vrow + k0 + 16 * u + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].x, b4[u].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].y, b4[u].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].z, b4[u].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[u].w, b4[u].w, acc, 0, 0, 0);
    }
  }
  for (; k0 < kend; k0 += 16) {
    const fx4 a4 = *(const AS1 fx4*)(Arow + k0 + 4 * q);
    const fx4 b4 = *(const AS1 fx4*)(Vrow + k0 + 4 * q);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc, 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) sY[wid][4 * q + t][i] = acc[t];
  sTT[tid / 16][tid % 16] = M.T[tid];
  __syncthreads();
  const int r = tid / 16, c = tid % 16;
  sYt[r][c] = sY[0][r][c] + sY[1][r][c] + sY[2][r][c] + sY[3][r][c];
  __syncthreads();
  float x = 0.f;
#pragma unroll
  for (int a = 0; a < SB; ++a) x += sYt[r][a] * sTT[a][c];
  sX[r][c] = x;
  gptr(M.X)[(long long)(row0 + r) * SB + c] = x;
  __syncthreads();
  // partial M[c][c'] = sum_r V[row0 + r][c] X[r][c'] (V[k][c] = Vr[c][k])
  const int cc = tid / 16, c2 = tid % 16;
  float s = 0.f;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) s += gptr(M.Vr)[(long long)cc * lda + row0 + rr] * sX[rr][c2];
  gptr(M.Mp)[(long long)blk * 256 + tid] = s;
}

// ------------------------------------------------------------------- N
// 1024 threads: quarter `part` of the partials of entry `e`, 8 loads in
// flight per thread (a serial 288-long sum took 34 us), then a fixed-order
// combine: deterministic.
__global__ __launch_bounds__(1024) void sy2sb_n_kernel(const SyMat* __restrict__ mats,
                                                       const int* __restrict__ act, int p) {
  const SyMat M = mats[act[blockIdx.x]];
  const int m = M.n - p * SB - SB;
  if (m < 1) return;
  const int nblk = (m + 15) / 16, tid = threadIdx.x;
  const int e = tid & 255, part = tid >> 8;
  __shared__ float sP[4][256];
  __shared__ float sM[16][17];
  const AS1 float* Mp = gptr(M.Mp);
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  for (int b0 = part * 8; b0 < nblk; b0 += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = b0 + u;
      acc[u] += gld_if(Mp, (long long)b * 256 + e, b < nblk, 0.f);
    }
  }
  sP[part][e] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (tid < 256) sM[tid / 16][tid % 16] = (sP[0][tid] + sP[1][tid]) + (sP[2][tid] + sP[3][tid]);
  __syncthreads();
  if (tid < 256) {
    const int c = tid / 16, c2 = tid % 16;
    float nn = 0.f;
#pragma unroll
    for (int a = 0; a < SB; ++a) nn += M.T[a * SB + c] * sM[a][c2];
    M.N[tid] = nn;
  }
}

// ------------------------------------------------------------------- U
// A22[I][J] -= Zm_I V_J^T + V_I Zm_J^T, Zm = X - V N / 2, one 64 x 64 tile
// per workgroup (both triangles: the next panel and the Y stage read rows)
__global__ __launch_bounds__(256) void sy2sb_upd_kernel(const SyMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int count,
                                                        int p) {
  int t;
  const SyMat M = mats[find_mat(offs, count, blockIdx.x, &t)];
  const int n = M.n;
  const long long lda = M.lda;
  const int j0 = p * SB, m = n - j0 - SB;
  const int nt = (m + UT - 1) / UT;
  const int I0 = (t / nt) * UT, J0 = (t % nt) * UT;
  const int tid = threadIdx.x;
  const int ty = tid >> 4, tx = tid & 15;
  // the tile's old values first: their latency hides under the V / Zm staging
  AS1 float* A = gptr(M.A) + (long long)(j0 + SB) * lda + j0 + SB;
  const int c0 = J0 + 4 * tx;
  fx4 old[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = I0 + 4 * ty + a;
    const fx4 z4 = {0.f, 0.f, 0.f, 0.f};
    old[a] = (row < m && c0 + 3 < m) ? *(const AS1 fx4*)(A + (long long)row * lda + c0) : z4;
  }
  __shared__ float sN[SB][SB + 1];
  __shared__ float sV[2][UT][SB + 1];
  __shared__ float sZ[2][UT][SB + 1];
  sN[tid / 16][tid % 16] = M.N[tid];
  const AS1 float* Vr = gptr(M.Vr);
  const AS1 float* X = gptr(M.X);
  // V rows of I and J (V[k][c] = Vr[c][k]); 2 x 64 x 16 values, 8 per thread
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int idx = tid + 256 * e;            // 0 .. 2047
    const int h = idx >> 10, rem = idx & 1023, c = rem >> 6, rr = rem & 63;
    const int row = (h ? J0 : I0) + rr;
    sV[h][rr][c] = gld_if(Vr, (long long)c * lda + row, row < m, 0.f);   // rows past m: 0
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int idx = tid + 256 * e;
    const int h = idx >> 10, rem = idx & 1023, rr = rem >> 4, c = rem & 15;
    const int row = (h ? J0 : I0) + rr;
    const float z = gld_if(X, (long long)row * SB + c, row < m, 0.f);
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < SB; ++a) s += sV[h][rr][a] * sN[a][c];
    sZ[h][rr][c] = z - 0.5f * s;
  }
  __syncthreads();
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
#pragma unroll 2
  for (int c = 0; c < SB; ++c) {
    float zi[4], vi[4], zj[4], vj[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      zi[a] = sZ[0][4 * ty + a][c]; vi[a] = sV[0][4 * ty + a][c];
      zj[a] = sZ[1][4 * tx + a][c]; vj[a] = sV[1][4 * tx + a][c];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] += zi[a] * vj[b] + vi[a] * zj[b];
  }
  // tiles run past m up to a multiple of 64 (and past lda): only rows and
  // columns < m are read or written
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = I0 + 4 * ty + a;
    if (row >= m) continue;
    AS1 float* pr = A + (long long)row * lda + c0;
    if (c0 + 3 < m) {
      fx4 x = old[a];
      x.x -= acc[a][0]; x.y -= acc[a][1]; x.z -= acc[a][2]; x.w -= acc[a][3];
      *(AS1 fx4*)pr = x;
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (c0 + b < m) pr[b] -= acc[a][b];
    }
  }
}

// ------------------------------------------------------------------- band
// Bs[r][o] = B[r][r - 2 SB + 1 + o] (lower band with room for the stage-2
// bulge) from the upper band of A; rows n .. n + 2 SB - 1 zero.
__global__ __launch_bounds__(256) void sy2sb_band_kernel(const SyMat* __restrict__ mats) {
  const SyMat M = mats[blockIdx.y];
  const int n = M.n;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(e / (2 * SB)), o = (int)(e % (2 * SB));
  if (r >= n + 2 * SB) return;
  const int c = r - 2 * SB + 1 + o;
  float v = 0.f;
  if (r < n && c >= 0 && c <= r && r - c <= SB) v = M.A[(long long)c * M.lda + r];
  M.band[(long long)r * (2 * SB) + o] = v;
}

__global__ __launch_bounds__(256) void sy2sb_zero_kernel(const SyMat* __restrict__ mats) {
  const SyMat M = mats[blockIdx.y];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < M.n; i += gridDim.x * 256) M.tau[i] = 0.f;
}

// ------------------------------------------------------------------ host
struct SyPlan {
  SyMat* d_mats = nullptr;
  int* d_offs = nullptr;      // per panel: act (count) | Y offsets (count+1) | U offsets (count+1)
  int count = 0, npan = 0, nmax = 0, band_grid = 0;
  std::vector<int> nact, gy, gu;
  hipGraphExec_t exec = nullptr;
};

int enqueue(const SyPlan& P, hipStream_t s) {
  const int stride = 3 * P.count + 2;
  hipLaunchKernelGGL(sy2sb_zero_kernel, dim3(8, P.count), dim3(256), 0, s, P.d_mats);
  for (int p = 0; p < P.npan; ++p) {
    if (P.nact[p] == 0) break;
    const int* act = P.d_offs + (size_t)p * stride;
    const int* oy = act + P.count;
    const int* ou = oy + P.count + 1;
    hipLaunchKernelGGL(sy2sb_panel_kernel, dim3(P.nact[p]), dim3(PT), 0, s, P.d_mats, act, p);
    hipLaunchKernelGGL(sy2sb_yx_kernel, dim3(P.gy[p]), dim3(256), 0, s, P.d_mats, oy, P.nact[p], p);
    hipLaunchKernelGGL(sy2sb_n_kernel, dim3(P.nact[p]), dim3(1024), 0, s, P.d_mats, act, p);
    hipLaunchKernelGGL(sy2sb_upd_kernel, dim3(P.gu[p]), dim3(256), 0, s, P.d_mats, ou, P.nact[p], p);
  }
  hipLaunchKernelGGL(sy2sb_band_kernel, dim3(P.band_grid, P.count), dim3(256), 0, s, P.d_mats);
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, SyPlan> g_plans;

}  // namespace

struct KfacSy2sbRecord {
  float* A; long long lda; float* tau; float* band; float* ws; long long n;
};

KFAC_API long long kfac_sy2sb_ws_floats(long long lda) { return ws_layout(lda).total; }
KFAC_API int kfac_sy2sb_nmax() { return NMAX2; }

namespace {
SyPlan* plan_for(const KfacSy2sbRecord* recs, int count, bool capture, int* err) {
  std::vector<int> order(count);
  for (int i = 0; i < count; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return recs[a].n > recs[b].n; });
  std::vector<SyMat> mats;
  for (int oi : order) {
    const KfacSy2sbRecord& r = recs[oi];
    if (r.n < 2 || r.n > NMAX2 || r.lda % 128 || r.lda < r.n) { *err = -2; return nullptr; }
    const SyWs L = ws_layout(r.lda);
    SyMat M;
    memset(&M, 0, sizeof(M));
    M.A = r.A; M.tau = r.tau; M.band = r.band; M.lda = r.lda; M.n = (int)r.n;
    M.Vr = r.ws + L.Vr; M.X = r.ws + L.X; M.Mp = r.ws + L.Mp; M.T = r.ws + L.T; M.N = r.ws + L.N;
    mats.push_back(M);
  }
  const std::string key((const char*)mats.data(), sizeof(SyMat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    SyPlan P;
    P.count = count;
    P.nmax = mats[0].n;
    P.npan = (P.nmax + SB - 1) / SB;
    const int stride = 3 * count + 2;
    std::vector<int> offs((size_t)P.npan * stride, 0);
    P.nact.assign(P.npan, 0); P.gy.assign(P.npan, 0); P.gu.assign(P.npan, 0);
    for (int p = 0; p < P.npan; ++p) {
      int* act = offs.data() + (size_t)p * stride;
      int* oy = act + count;
      int* ou = oy + count + 1;
      int na = 0, accy = 0, accu = 0;
      for (int i = 0; i < count; ++i) {      // descending n: the active matrices come first
        const int m = mats[i].n - p * SB - SB;
        if (m < 1) continue;
        act[na] = i;
        oy[na] = accy; ou[na] = accu;
        accy += (m + 15) / 16;
        const int nt = (m + UT - 1) / UT;
        accu += nt * nt;
        ++na;
      }
      oy[na] = accy; ou[na] = accu;
      P.nact[p] = na; P.gy[p] = accy; P.gu[p] = accu;
    }
    P.band_grid = (int)(((long long)(P.nmax + 2 * SB) * 2 * SB + 255) / 256);
    if ((*err = (int)hipMalloc(&P.d_mats, sizeof(SyMat) * mats.size())) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(SyMat) * mats.size(),
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    if ((*err = (int)hipMalloc(&P.d_offs, sizeof(int) * offs.size())) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * offs.size(),
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    it = g_plans.emplace(key, P).first;
  }
  SyPlan* plan = &it->second;
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

// Reduce `count` full symmetric matrices (2 <= n <= kfac_sy2sb_nmax(), lda a
// multiple of 128 >= n, zero outside n x n) to band form: A's rows keep the
// stage-1 reflectors, tau (n floats), band ((n + 32) x 32 floats, the lower
// band of stage 2), ws (kfac_sy2sb_ws_floats(lda) floats, zeroed once).
KFAC_API int kfac_sy2sb_batched(const KfacSy2sbRecord* recs, int count, int use_graph,
                                hipStream_t stream) {
  if (count <= 0 || count > MAXM2) return count <= 0 ? 0 : -5;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  int err = 0;
  SyPlan* plan = plan_for(recs, count, graph, &err);
  if (!plan) return err ? err : -4;
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}
