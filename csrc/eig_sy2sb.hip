// Dense -> band reduction (stage 1 of the two-stage symmetric eigensolver,
// SURVEY.md K6; reference: kfac/layers/utils.py:45-74, torch.symeig per
// factor).  Panels of BW = 16 columns; for the panel at columns k .. k+15
// (m = n - k - 16 rows below the band):
//
//   panel  one 512-thread workgroup per matrix: Householder QR of
//          A[k+16:, k:k+16] held in registers (<= 10 rows x 16 per thread),
//          one block reduction per column (the column's |x|^2 and its dots
//          with the later columns together), Gram V^T V, T (larft) and
//          U^T = (V T)^T; R to the band, v[1:] of reflector k+c to row k+c
//          of the upper triangle (the back-transformation's layout, offset 16)
//   x      X = A22 U, v_mfma_f32_16x16x4f32 (exact f32), one wave per 16 rows
//   w      W = X - V (T^T (V^T X)) / 2, one workgroup per matrix
//   upd    A22 -= V W^T + W V^T, 128 x 128 tiles, v_mfma_f32_32x32x2f32
//
// A is stored full (both triangles, row-major, lda % 64 == 0); every matrix
// of the batch advances through the same launch sequence (ragged: a launch's
// workgroups map to matrices through a host-built offset table).  The band
// (n x 32 column-major, diagonals 0..16, zeros for the bulge room) is then
// extracted for stage 2 (csrc/eig_sb2st.hip).  Model of the exact operation
// order in fp64: scripts/models/two_stage_model.py (sy2sb).
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int BW = 16;
constexpr int ND = 2 * BW;
constexpr int PT = 1024;        // panel workgroup
constexpr int RQ = 5;           // panel rows per thread: m <= 5120
constexpr int NWV = PT / 64;
constexpr int TB = 128;         // update tile
constexpr int MAXM = 255;

struct S1Mat {
  float* A; long long lda; int n, pad;
  float* tau;                   // n (zeroed up front: rows without a reflector)
  float* V; float* W; float* X; // n x 16 each (panel rows)
  float* Ut;                    // 16 x ldu
  float* T;                     // 16 x 16
  float* band;                  // n x ND
  long long ldu;
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



// -------------------------------------------------------------- panel
__global__ __launch_bounds__(PT) void sy2sb_panel_kernel(const S1Mat* __restrict__ mats,
                                                         const int* __restrict__ offs, int nact,
                                                         int k) {
  __shared__ int soff[MAXM + 1];
  __shared__ float red16[NWV][BW];
  __shared__ float red[BW];
  __shared__ float rowc[BW];
  __shared__ float taus[BW];
  __shared__ float G[BW][BW + 1];
  __shared__ float sT[BW][BW + 1];
  __shared__ float gred[NWV][BW * BW];
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const S1Mat M = mats[mi];
  const int n = M.n, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long lda = M.lda;
  const int m = n - k - BW;
  AS1 float* const A = gptr(M.A);
  float P[RQ][BW];
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int i = tid + PT * q;
    const bool ok = i < m;
    const AS1 fx4* src = (const AS1 fx4*)(A + (long long)(k + BW + (ok ? i : 0)) * lda + k);
#pragma unroll
    for (int x = 0; x < BW / 4; ++x) {
      const fx4 t = src[x];
      P[q][4 * x] = ok ? t.x : 0.f; P[q][4 * x + 1] = ok ? t.y : 0.f;
      P[q][4 * x + 2] = ok ? t.z : 0.f; P[q][4 * x + 3] = ok ? t.w : 0.f;
    }
  }
  // column loop NOT unrolled: P is indexed only with literal x, the runtime
  // column c enters through compares (selects), so P stays in VGPRs
#pragma unroll 1
  for (int c = 0; c < BW; ++c) {
    float part[BW];
#pragma unroll
    for (int x = 0; x < BW; ++x) part[x] = 0.f;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int i = tid + PT * q;
      float xc = 0.f;
#pragma unroll
      for (int x = 0; x < BW; ++x) xc = (x == c) ? P[q][x] : xc;
      xc = (i > c && i < m) ? xc : 0.f;
#pragma unroll
      for (int x = 0; x < BW; ++x) part[x] += xc * P[q][x];
    }
    if (tid == c) {
#pragma unroll
      for (int x = 0; x < BW; ++x) rowc[x] = P[0][x];
    }
    {
      const float s_ = kfac_butterfly16(part);       // lane x (< 16): value x
      if (lane < BW) red16[wave][lane] = s_;
    }
    __syncthreads();
    if (tid < BW) {
      float s_ = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) s_ += red16[w][tid];
      red[tid] = s_;
    }
    __syncthreads();
    const float sig = red[c];
    const float alpha = rowc[c];
    float tau = 0.f, beta = alpha, scal = 0.f;
    if (c < m - 1 && sig != 0.f) {
      beta = -copysignf(sqrtf(alpha * alpha + sig), alpha);
      tau = (beta - alpha) / beta;
      scal = 1.f / (alpha - beta);
    }
    if (tid == 0) taus[c] = tau;
    float wc[BW];
#pragma unroll
    for (int x = 0; x < BW; ++x) wc[x] = (x > c) ? tau * (rowc[x] + scal * red[x]) : 0.f;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int i = tid + PT * q;
      float xc = 0.f;
#pragma unroll
      for (int x = 0; x < BW; ++x) xc = (x == c) ? P[q][x] : xc;
      const bool below = i > c && i < m;
      const float vi = below ? scal * xc : (i == c ? 1.f : 0.f);
      const float nc = below ? vi : (i == c ? beta : xc);
#pragma unroll
      for (int x = 0; x < BW; ++x) P[q][x] = (x == c) ? nc : P[q][x] - vi * wc[x];
    }
    __syncthreads();   // red / rowc reused by the next column
  }
  // explicit v (1 at row c, zero above) for the Gram and U
#define vval(q, c) ((tid + PT * (q) < m) ? (tid + PT * (q) == (c) ? 1.f : (tid + PT * (q) > (c) ? P[q][c] : 0.f)) : 0.f)
  // v[1:] of reflector k+c to row k+c (upper triangle, component k+16+i),
  // R (rows i < 16, columns c >= i) to the lower band; then P -> explicit V
  {
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int i = tid + PT * q;
      if (i >= m) continue;
#pragma unroll
      for (int c = 0; c < BW; ++c)
        if (i > c) A[(long long)(k + c) * lda + k + BW + i] = P[q][c];
      if (q == 0 && i < BW) {
        AS1 float* const arow = A + (long long)(k + BW + i) * lda + k;
#pragma unroll
        for (int c = 0; c < BW; ++c) arow[c] = (c >= i) ? P[q][c] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
      for (int c = 0; c < BW; ++c) P[q][c] = vval(q, c);
  }
#undef vval
  // Gram V^T V: one row a of G per pass (<= 16 wave sums), upper half
#pragma unroll
  for (int a = 0; a < BW; ++a) {
    float gp[BW];
#pragma unroll
    for (int b = 0; b < BW; ++b) gp[b] = 0.f;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const float va = P[q][a];
#pragma unroll
      for (int b = a; b < BW; ++b) gp[b] += va * P[q][b];
    }
    {
      const float s = kfac_butterfly16(gp);
      if (lane < BW) gred[wave][a * BW + lane] = s;
    }
  }
  __syncthreads();
  if (tid < BW * BW) {
    const int a = tid / BW, b = tid % BW;
    if (b >= a) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) s += gred[w][tid];
      G[a][b] = s;
      G[b][a] = s;
    }
  }
  __syncthreads();
  // T (upper): T(i,i) = tau_i, T(0:i, i) = -tau_i T(0:i, 0:i) G(0:i, i)
  if (wave == 0) {
    const int r = lane;
    if (r < BW) {
#pragma unroll
      for (int x = 0; x < BW; ++x) sT[r][x] = 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = 0; i < BW; ++i) {
      const float ti = taus[i];
      float acc = 0.f;
      if (r < i)
        for (int q = r; q < i; ++q) acc += sT[r][q] * G[q][i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (r < i) sT[r][i] = -ti * acc;
      else if (r == i) sT[r][i] = ti;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  // outputs: R into the lower band, v[1:] into the upper rows k+c, V, U^T, T, tau
  AS1 float* const gV = gptr(M.V);
  AS1 float* const gUt = gptr(M.Ut);
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int i = tid + PT * q;
    if (i >= m) continue;
    float u[BW];
#pragma unroll
    for (int b = 0; b < BW; ++b) {
      float s = 0.f;
#pragma unroll
      for (int a = 0; a <= b; ++a) s += P[q][a] * sT[a][b];
      u[b] = s;
    }
#pragma unroll
    for (int b = 0; b < BW; ++b) gUt[(long long)b * M.ldu + i] = u[b];
    AS1 fx4* vrow = (AS1 fx4*)(gV + (long long)i * BW);
#pragma unroll
    for (int x = 0; x < BW / 4; ++x) {
      fx4 t;
      t.x = P[q][4 * x]; t.y = P[q][4 * x + 1]; t.z = P[q][4 * x + 2]; t.w = P[q][4 * x + 3];
      vrow[x] = t;
    }
  }
  if (tid < BW) M.tau[k + tid] = taus[tid];
  if (tid < BW * BW) gptr(M.T)[tid] = sT[tid / BW][tid % BW];
  // pad U^T to a multiple of 16 columns (the X kernel's k-steps)
  if (tid < BW * 16) {
    const int b = tid / 16, i = m + (tid % 16);
    if (i < ((m + 15) & ~15)) gUt[(long long)b * M.ldu + i] = 0.f;
  }
}

// -------------------------------------------------------------- x
// X = A22 U: wave per 16 rows, 16x16x4 f32 MFMA; lane (r, g): A22 row r,
// k-quad g of every 16-wide k step (the same k permutation on both operands)
__global__ __launch_bounds__(256) void sy2sb_x_kernel(const S1Mat* __restrict__ mats,
                                                      const int* __restrict__ offs, int nact,
                                                      int k) {
  __shared__ int soff[MAXM + 1];
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const S1Mat M = mats[mi];
  const int n = M.n, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = n - k - BW;
  const int i0 = (local * 4 + wave) * 16;
  if (i0 >= m) return;
  const long long lda = M.lda;
  const int r = lane & 15, g = lane >> 4;
  const int row = min(i0 + r, m - 1);
  const AS1 float* arow = gptr(M.A) + (long long)(k + BW + row) * lda + k + BW;
  const AS1 float* urow = gptr(M.Ut) + (long long)r * M.ldu;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int mk = m & ~15;
  int kk = 0;
  for (; kk < mk; kk += 16) {
    const fx4 a = *(const AS1 fx4*)(arow + kk + 4 * g);
    const fx4 b = *(const AS1 fx4*)(urow + kk + 4 * g);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
  if (kk < m) {     // tail: U^T is zero-padded; A columns past m read as zero
    float a4[4], b4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = kk + 4 * g + t;
      a4[t] = gld_if(arow, c, c < m, 0.f);
      b4[t] = urow[c];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t], b4[t], acc, 0, 0, 0);
  }
  // C map: col = lane & 15, rows 4 g + v
  AS1 float* const X = gptr(M.X);
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int i = i0 + 4 * g + v;
    if (i < m) X[(long long)i * BW + r] = acc[v];
  }
}

// -------------------------------------------------------------- w
// W = X - V (T^T (V^T X)) / 2: one workgroup per matrix
constexpr int PTW = 512;
__global__ __launch_bounds__(PTW) void sy2sb_w_kernel(const S1Mat* __restrict__ mats,
                                                     const int* __restrict__ offs, int nact,
                                                     int k) {
  __shared__ int soff[MAXM + 1];
  __shared__ float yred[PTW / 64][BW * BW];
  __shared__ float Y[BW][BW + 1];
  __shared__ float Z[BW][BW + 1];
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const S1Mat M = mats[mi];
  const int n = M.n, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = n - k - BW;
  const AS1 float* gV = gptr(M.V);
  const AS1 float* gX = gptr(M.X);
  // Y = V^T X in 4 blocks of 4 rows of Y (64 partials per thread), rows of
  // V / X streamed from L2 per block; transposed butterfly per wave
  for (int blk = 0; blk < 4; ++blk) {
    float pv[64];
#pragma unroll
    for (int e = 0; e < 64; ++e) pv[e] = 0.f;
    for (int i = tid; i < m; i += PTW) {
      const fx4 va = *(const AS1 fx4*)(gV + (long long)i * BW + 4 * blk);
      const float vv[4] = {va.x, va.y, va.z, va.w};
      float xr[BW];
#pragma unroll
      for (int e = 0; e < BW / 4; ++e) {
        const fx4 xb = *(const AS1 fx4*)(gX + (long long)i * BW + 4 * e);
        xr[4 * e] = xb.x; xr[4 * e + 1] = xb.y; xr[4 * e + 2] = xb.z; xr[4 * e + 3] = xb.w;
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b2 = 0; b2 < BW; ++b2) pv[a * BW + b2] += vv[a] * xr[b2];
    }
    kfac_butterfly64(pv);
    yred[wave][blk * 64 + lane] = pv[0];
  }
  __syncthreads();
  if (tid < BW * BW) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < PTW / 64; ++w) s += yred[w][tid];
    Y[tid / BW][tid % BW] = s;
  }
  __syncthreads();
  if (tid < BW * BW) {    // Z = T^T Y / 2 (T upper: T^T lower)
    const int a = tid / BW, b = tid % BW;
    const AS1 float* T = gptr(M.T);
    float s = 0.f;
    for (int q = 0; q <= a; ++q) s += T[q * BW + a] * Y[q][b];
    Z[a][b] = 0.5f * s;
  }
  __syncthreads();
  AS1 float* const gW = gptr(M.W);
  for (int i = tid; i < m; i += PTW) {
    float vr[BW], xr[BW];
#pragma unroll
    for (int e = 0; e < BW / 4; ++e) {
      const fx4 a4 = *(const AS1 fx4*)(gV + (long long)i * BW + 4 * e);
      const fx4 b4 = *(const AS1 fx4*)(gX + (long long)i * BW + 4 * e);
      vr[4 * e] = a4.x; vr[4 * e + 1] = a4.y; vr[4 * e + 2] = a4.z; vr[4 * e + 3] = a4.w;
      xr[4 * e] = b4.x; xr[4 * e + 1] = b4.y; xr[4 * e + 2] = b4.z; xr[4 * e + 3] = b4.w;
    }
#pragma unroll
    for (int e = 0; e < BW / 4; ++e) {
      float o[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int b2 = 4 * e + t;
        float s = xr[b2];
#pragma unroll
        for (int a = 0; a < BW; ++a) s -= vr[a] * Z[a][b2];
        o[t] = s;
      }
      fx4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
      *(AS1 fx4*)(gW + (long long)i * BW + 4 * e) = ov;
    }
  }
}

// -------------------------------------------------------------- upd
// A22[I][K] -= L_I R_K^T, L = [V | W], R = [W | V] (32 wide), every tile of
// the trailing square (both triangles kept), 4 waves of 64 x 64
__global__ __launch_bounds__(256) void sy2sb_upd_kernel(const S1Mat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int k) {
  __shared__ float sL[TB][2 * BW + 1];
  __shared__ float sR[TB][2 * BW + 1];
  __shared__ int soff[MAXM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const S1Mat M = mats[mi];
  const int n = M.n;
  const int m = n - k - BW;
  const int mt = (m + TB - 1) / TB;
  const int I = local / mt, K = local % mt;
  const AS1 float* gV = gptr(M.V);
  const AS1 float* gW = gptr(M.W);
#pragma unroll
  for (int e0 = 0; e0 < TB * BW; e0 += 256) {
    const int e = e0 + tid;
    const int rr = e / BW, x = e - rr * BW;
    const int ri = I * TB + rr, rk = K * TB + rr;
    const float vi = gld_if(gV, (long long)ri * BW + x, ri < m, 0.f);
    const float wi = gld_if(gW, (long long)ri * BW + x, ri < m, 0.f);
    const float vk = gld_if(gV, (long long)rk * BW + x, rk < m, 0.f);
    const float wk = gld_if(gW, (long long)rk * BW + x, rk < m, 0.f);
    sL[rr][x] = vi; sL[rr][BW + x] = wi;
    sR[rr][x] = wk; sR[rr][BW + x] = vk;
  }
  __syncthreads();
  const int wr = wave >> 1, wc = wave & 1;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[a][b][x] = 0.f;
#pragma unroll
  for (int kk = 0; kk < BW; ++kk) {            // k = 2 kk + lh over 2 BW
    const int kx = 2 * kk + lh;
    float av[2], bv[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) av[a] = sL[wr * 64 + a * 32 + l31][kx];
#pragma unroll
    for (int b = 0; b < 2; ++b) bv[b] = sR[wc * 64 + b * 32 + l31][kx];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
  AS1 float* const A = gptr(M.A) + (long long)(k + BW) * M.lda + k + BW;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float old[16];
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh;
        const int gc = K * TB + wc * 64 + b * 32 + l31;
        old[x] = gld_if(A, (long long)gr * M.lda + gc, gr < m && gc < m, 0.f);
      }
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh;
        const int gc = K * TB + wc * 64 + b * 32 + l31;
        if (gr < m && gc < m) A[(long long)gr * M.lda + gc] = old[x] - acc[a][b][x];
      }
    }
}

// ------------------------------------------------------------ band, tau
__global__ __launch_bounds__(256) void sy2sb_init_kernel(const S1Mat* __restrict__ mats) {
  const S1Mat M = mats[blockIdx.y];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < M.n; i += gridDim.x * 256) M.tau[i] = 0.f;
}

__global__ __launch_bounds__(256) void sy2sb_band_kernel(const S1Mat* __restrict__ mats) {
  const S1Mat M = mats[blockIdx.y];
  const long long tot = (long long)M.n * ND;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < tot; e += (long long)gridDim.x * 256) {
    const int c = (int)(e / ND), d = (int)(e % ND);
    const int r = c + d;
    M.band[e] = (d <= BW && r < M.n) ? M.A[(long long)r * M.lda + c] : 0.f;
  }
}

struct S1Plan {
  S1Mat* d_mats = nullptr;
  int* d_offs = nullptr;
  int count = 0, maxn = 0, np = 0;
  std::vector<int> grid[4], nact[4];      // [panel] per kind: panel, x, w, upd
  hipGraphExec_t exec = nullptr;
};

void counts(int n, int p, int out[4]) {
  const int k = p * BW, m = n - k - BW;
  if (m < 2) { out[0] = out[1] = out[2] = out[3] = 0; return; }
  const int mt = (m + TB - 1) / TB;
  out[0] = 1;
  out[1] = (m + 63) / 64;
  out[2] = 1;
  out[3] = mt * mt;
}

int enqueue(const S1Plan& P, hipStream_t stream) {
  const int nm = P.count;
  hipLaunchKernelGGL(sy2sb_init_kernel, dim3((P.maxn + 255) / 256, nm), dim3(256), 0, stream,
                     P.d_mats);
  for (int p = 0; p < P.np; ++p) {
    const int k = p * BW;
    const int* of = P.d_offs + (size_t)p * 4 * (nm + 1);
    if (P.grid[0][p] == 0) continue;
    hipLaunchKernelGGL(sy2sb_panel_kernel, dim3(P.grid[0][p]), dim3(PT), 0, stream, P.d_mats,
                       of, P.nact[0][p], k);
    hipLaunchKernelGGL(sy2sb_x_kernel, dim3(P.grid[1][p]), dim3(256), 0, stream, P.d_mats,
                       of + (nm + 1), P.nact[1][p], k);
    hipLaunchKernelGGL(sy2sb_w_kernel, dim3(P.grid[2][p]), dim3(PTW), 0, stream, P.d_mats,
                       of + 2 * (nm + 1), P.nact[2][p], k);
    hipLaunchKernelGGL(sy2sb_upd_kernel, dim3(P.grid[3][p]), dim3(256), 0, stream, P.d_mats,
                       of + 3 * (nm + 1), P.nact[3][p], k);
  }
  hipLaunchKernelGGL(sy2sb_band_kernel, dim3(512, nm), dim3(256), 0, stream, P.d_mats);
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, S1Plan> g_plans;

}  // namespace

struct KfacS1Record {
  float* A; long long lda; float* tau; float* ws; float* band; long long n;
};

// workspace floats per matrix: V, W, X (n x 16), U^T (16 x ldu), T
KFAC_API long long kfac_sy2sb_ws_floats(int n) {
  const long long ldu = ((long long)n + 16 + 63) / 64 * 64;
  return 3LL * n * BW + BW * ldu + BW * BW + 64;
}

// Dense symmetric (both triangles, row-major) -> band + Q1 reflectors for a
// ragged batch (n <= 5136 each): band (n x 32), tau (n), reflector k+c in row
// k+c of A from column k+c+16 on (v[0] = 1 implicit).
KFAC_API int kfac_sy2sb_batched(const KfacS1Record* recs, int count, int use_graph,
                                hipStream_t stream) {
  if (count <= 0) return 0;
  if (count > MAXM) return -5;
  std::vector<S1Mat> mats(count);
  int maxn = 0;
  for (int i = 0; i < count; ++i) {
    const KfacS1Record& r = recs[i];
    if (r.n < 2 || r.lda < r.n || (r.lda & 63)) return -2;
    if (r.n - BW > PT * RQ) return -6;
    S1Mat& M = mats[i];
    memset(&M, 0, sizeof(M));
    M.A = r.A; M.lda = r.lda; M.n = (int)r.n; M.tau = r.tau; M.band = r.band;
    M.ldu = ((long long)r.n + 16 + 63) / 64 * 64;
    float* p = r.ws;
    M.V = p; p += (long long)r.n * BW;
    M.W = p; p += (long long)r.n * BW;
    M.X = p; p += (long long)r.n * BW;
    M.Ut = p; p += BW * M.ldu;
    M.T = p;
    maxn = std::max(maxn, M.n);
  }
  const std::string key((const char*)mats.data(), sizeof(S1Mat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    S1Plan P;
    P.count = count;
    P.maxn = maxn;
    P.np = (maxn + BW - 1) / BW;
    const int nm = count;
    std::vector<int> offs((size_t)P.np * 4 * (nm + 1), 0);
    for (int q = 0; q < 4; ++q) { P.grid[q].assign(P.np, 0); P.nact[q].assign(P.np, 0); }
    for (int p = 0; p < P.np; ++p) {
      int acc[4] = {0, 0, 0, 0};
      for (int i = 0; i < nm; ++i) {
        int c[4];
        counts(mats[i].n, p, c);
        for (int q = 0; q < 4; ++q) {
          offs[((size_t)p * 4 + q) * (nm + 1) + i] = acc[q];
          if (c[q] > 0) P.nact[q][p] = i + 1;
          acc[q] += c[q];
        }
      }
      for (int q = 0; q < 4; ++q) {
        offs[((size_t)p * 4 + q) * (nm + 1) + nm] = acc[q];
        P.grid[q][p] = acc[q];
      }
    }
    int e = (int)hipMalloc(&P.d_mats, sizeof(S1Mat) * nm);
    if (!e) e = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(S1Mat) * nm, hipMemcpyHostToDevice);
    if (!e) e = (int)hipMalloc(&P.d_offs, sizeof(int) * offs.size());
    if (!e) e = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * offs.size(), hipMemcpyHostToDevice);
    if (e) return e;
    it = g_plans.emplace(key, P).first;
  }
  S1Plan& P = it->second;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  if (graph && !P.exec) {
    static hipStream_t cap = nullptr;
    if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
    hipGraph_t g = nullptr;
    if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      const int e1 = enqueue(P, cap);
      const hipError_t e2 = hipStreamEndCapture(cap, &g);
      if (!e1 && e2 == hipSuccess && g && hipGraphInstantiate(&P.exec, g, nullptr, nullptr, 0) != hipSuccess)
        P.exec = nullptr;
      if (g) (void)hipGraphDestroy(g);
    }
    (void)hipGetLastError();
  }
  if (graph && P.exec) return (int)hipGraphLaunch(P.exec, stream);
  return enqueue(P, stream);
}
