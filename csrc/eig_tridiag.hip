// Blocked Householder tridiagonalisation for large K-FAC factors on gfx950.
//
// Replaces rocSOLVER's sytrd, whose per-column chain of ~8 small kernels is
// latency bound on MI355X (15 us per column at n = 1024, 23 us at n = 4608:
// profiles/r1_rocsolver_fill_split.log).  Same algorithm family (LAPACK
// sytrd/latrd, lower), re-shaped for the GPU:
//
//   * every matrix of a size class in one launch (blockIdx.y = matrix)
//   * THREE launches per column:
//       A  symmetric mat-vec y = A22 v over UPPER 128x128 tiles only (each
//          off-diagonal tile feeds y_I and y_K: half the HBM/MALL traffic of a
//          full mat-vec); the Householder vector v is formed on the fly from
//          the previous launch's column and norm partials; the diagonal tiles
//          also produce the panel dot products W^T v, V^T v
//       B  w' = tau (y - V W^T v - W V^T v), partial w'^T v
//       C  W[:, c] = w' + alpha2 v, next column with the panel corrections,
//          its norm partials
//     every cross-workgroup reduction is a per-block partial re-reduced by the
//     next launch (no atomics: deterministic)
//   * per panel of NB = 32 columns one MFMA-free rank-2NB update of the upper
//     triangle of the trailing matrix (VALU, 8x8 outputs per thread)
//   * the whole sequence (3n + 2n/NB launches) is captured into ONE hipGraph
//     per (size class, buffers) and replayed at every inverse update, so the
//     per-launch cost is the graph's kernel boundary, not a host launch.
//
// Storage: row-major, UPPER triangle maintained (== LAPACK lower, column-major);
// row j is "column j".  Output: d, e, tau and the reflectors in row j
// (e_j at j+1, v[1:] from j+2): the layout rocSOLVER's ormtr (lower) reads.
// Reference semantics: kfac/layers/utils.py:45-74 (symeig).  The algorithm is
// modelled phase by phase in scripts/models/sytrd_model.py.
#include "common.h"

#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr int TB = 128;   // symv / update tile
constexpr int NB = 32;    // panel width

struct Ws {
  float* V; float* W; float* X; float* Wp; float* Sc; float* P; float* Dx; double* Ep; double* Np;
};

__host__ __device__ inline long long ws_floats(int n) {
  const int nt = (n + TB - 1) / TB;
  const long long n4 = (n + 3) / 4 * 4;
  long long s = 2LL * n * NB + 3 * n4 + (long long)nt * nt * TB + (long long)nt * 2 * NB +
                4LL * nt;
  return (s + 63) / 64 * 64;
}

__device__ inline Ws ws_at(float* base, int n) {
  const int nt = (n + TB - 1) / TB;
  const long long n4 = (n + 3) / 4 * 4;
  Ws w;
  w.V = base;
  w.W = w.V + (long long)n * NB;
  w.X = w.W + (long long)n * NB;
  w.Wp = w.X + n4;
  w.Sc = w.Wp + n4;
  w.P = w.Sc + n4;
  w.Dx = w.P + (long long)nt * nt * TB;
  w.Ep = (double*)(w.Dx + (long long)nt * 2 * NB);
  w.Np = w.Ep + nt;
  return w;
}

__device__ inline void tri_index(int t, int mb, int& I, int& K) {
  int i = 0;
  while (t >= mb - i) { t -= mb - i; ++i; }
  I = i; K = i + t;
}

struct Args {
  float* A; long long sA; int lda; int n; int nt;
  float* ws; long long sW;
  float* d; float* e; float* tau;
};

// 256-thread block reduction of one double (result valid in thread 0)
__device__ inline double block_sum_d(double v, double* red8) {
  v = wave_reduce_sum_d(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red8[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < 4; ++w) s += red8[w];
  return s;
}

// ------------------------------------------------------------------ phase A
__global__ __launch_bounds__(256) void sytrd_symv_kernel(Args a, int j, int s0, int sh) {
  const int mat = blockIdx.y;
  float* A = a.A + mat * a.sA;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const int n = a.n, nt = a.nt, lda = a.lda;
  __shared__ float sv[2][TB];
  __shared__ float red[TB][33];
  __shared__ float colred[4][TB];
  __shared__ float sc[4];
  int I, K;
  tri_index(blockIdx.x, nt - s0, I, K);
  I += s0; K += s0;
  const int tid = threadIdx.x;
  const bool diag = (I == K);
  const int wave = tid >> 6, lane = tid & 63, half = lane >> 5, cl = lane & 31;
  const int kk0 = cl * 4, k0 = K * TB + kk0;
  // the small loads first (norm partials, alpha, this thread's x element),
  // then all 16 row loads of the lane (64 KB per workgroup in flight): the
  // scalar set-up waits only for the former (in-order vmcnt)
  double npv = 0.0;
  float alpha = 0.f;
  if (wave == 0) {
    for (int s = sh + lane; s < nt; s += 64) npv += w.Np[s];
    alpha = w.X[j + 1];
  }
  const bool lead = (I == s0 && K == s0 && tid == 0);
  const float xj = lead ? w.X[j] : 0.f;
  const int vh = tid >> 7, vt = tid & 127;
  const int vr_idx = (vh ? K : I) * TB + vt;
  const float xv = (vr_idx < n && vr_idx > j + 1) ? w.X[vr_idx] : 0.f;
  float4 q[16];
  const bool full_cols = (k0 + 3 < n);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int r = I * TB + wave * 32 + it * 2 + half;
    q[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < n) {
      const float* row = A + (long long)r * lda;
      if (full_cols) {
        q[it] = *(const float4*)(row + k0);
      } else {
        if (k0 < n) q[it].x = row[k0];
        if (k0 + 1 < n) q[it].y = row[k0 + 1];
        if (k0 + 2 < n) q[it].z = row[k0 + 2];
      }
    }
  }
  if (wave == 0) {
    const double sig = wave_reduce_sum_d(npv);
    if (lane == 0) {
      float beta, tau, scale;
      if (sig == 0.0) {
        tau = 0.f; beta = alpha; scale = 0.f;
      } else {
        const double b = -copysign(sqrt((double)alpha * alpha + sig), (double)alpha);
        beta = (float)b;
        tau = (float)((b - alpha) / b);
        scale = (float)(1.0 / ((double)alpha - b));
      }
      sc[0] = beta; sc[1] = tau; sc[2] = scale;
    }
  }
  __syncthreads();
  sv[vh][vt] = (vr_idx == j + 1) ? 1.f : xv * sc[2];
  __syncthreads();

  float ca[4] = {0.f, 0.f, 0.f, 0.f};
  const float vk0 = sv[1][kk0], vk1 = sv[1][kk0 + 1], vk2 = sv[1][kk0 + 2], vk3 = sv[1][kk0 + 3];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int rr = wave * 32 + it * 2 + half;
    float x0 = q[it].x, x1 = q[it].y, x2 = q[it].z, x3 = q[it].w;
    const float vr = sv[0][rr];
    if (diag) {
      // upper triangle only: row sums take k >= r, column sums k > r
      x0 = (kk0 >= rr) ? x0 : 0.f;
      x1 = (kk0 + 1 >= rr) ? x1 : 0.f;
      x2 = (kk0 + 2 >= rr) ? x2 : 0.f;
      x3 = (kk0 + 3 >= rr) ? x3 : 0.f;
      red[rr][cl] = x0 * vk0 + x1 * vk1 + x2 * vk2 + x3 * vk3;
      ca[0] += (kk0 > rr) ? x0 * vr : 0.f;
      ca[1] += (kk0 + 1 > rr) ? x1 * vr : 0.f;
      ca[2] += (kk0 + 2 > rr) ? x2 * vr : 0.f;
      ca[3] += (kk0 + 3 > rr) ? x3 * vr : 0.f;
    } else {
      red[rr][cl] = x0 * vk0 + x1 * vk1 + x2 * vk2 + x3 * vk3;
      ca[0] += x0 * vr; ca[1] += x1 * vr; ca[2] += x2 * vr; ca[3] += x3 * vr;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) ca[i] += __shfl_xor(ca[i], 32, 64);
  if (half == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) colred[wave][kk0 + i] = ca[i];
  }
  __syncthreads();
  if (tid < TB) {
    float rs = 0.f;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) rs += red[tid][l];
    const float cs = colred[0][tid] + colred[1][tid] + colred[2][tid] + colred[3][tid];
    if (diag) {
      w.P[((long long)I * nt + K) * TB + tid] = rs + cs;
    } else {
      w.P[((long long)I * nt + K) * TB + tid] = rs;
      w.P[((long long)K * nt + I) * TB + tid] = cs;
    }
  }
  if (lead) {
    a.tau[(long long)mat * n + j] = sc[1];
    a.e[(long long)mat * n + j] = sc[0];
    a.d[(long long)mat * n + j] = xj;
    w.Sc[j] = sc[2];
  }
}

// ------------------------------------------------------------------ phase B
// w' = tau (y - V s1 - W s2) with s1 = W^T v, s2 = V^T v assembled from the
// x-dot partials of the previous launch (v = e_{j+1} + scale x), the column's
// v materialised into V[:, c] and row j of A.  Every partial and row load is
// issued up front (latency bound: no serial load-accumulate chains).
__global__ __launch_bounds__(256) void sytrd_w_kernel(Args a, int j, int c, int s0) {
  const int mat = blockIdx.y;
  float* A = a.A + mat * a.sA;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const int n = a.n, nt = a.nt, lda = a.lda;
  const int J = s0 + blockIdx.x;
  __shared__ double s4[4][2 * NB];
  __shared__ float s12[2 * NB];
  __shared__ float row1[2 * NB];
  __shared__ float ys[2][TB];
  __shared__ double red8[4];
  const int tid = threadIdx.x;
  const int r = J * TB + (tid & (TB - 1));
  const bool row_ok = tid < TB && r < n;
  float4 vr4[NB / 4], wr4[NB / 4];
  float xr = 0.f;
  if (row_ok) {
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) {
      vr4[i] = *(const float4*)(w.V + (long long)r * NB + 4 * i);
      wr4[i] = *(const float4*)(w.W + (long long)r * NB + 4 * i);
    }
    xr = w.X[r];
  }
  const float tau = a.tau[(long long)mat * n + j];
  const float beta = a.e[(long long)mat * n + j];
  const float scale = w.Sc[j];
  if (tid < 2 * NB) {   // row j+1 of W (cols 0..31) and V (32..63)
    const int cc = tid & (NB - 1);
    row1[tid] = (cc < c) ? (tid < NB ? w.W : w.V)[(long long)(j + 1) * NB + cc] : 0.f;
  }
  {  // x-dot partials: 64 columns x 4 groups of blocks
    const int col = tid & 63, g = tid >> 6;
    double acc = 0.0;
    if ((col & (NB - 1)) < c) {
#pragma unroll 4
      for (int q = s0 + g; q < nt; q += 4) acc += w.Dx[(long long)q * 2 * NB + col];
    }
    s4[g][col] = acc;
  }
  {  // y: two halves of the partial range, 8 loads in flight
    const int h = tid >> 7, t = tid & 127;
    const int mid = s0 + (nt - s0) / 2;
    const int lo = h ? mid : s0, hi = h ? nt : mid;
    float y = 0.f;
#pragma unroll 8
    for (int q = lo; q < hi; ++q) y += w.P[((long long)J * nt + q) * TB + t];
    ys[h][t] = y;
  }
  __syncthreads();
  if (tid < 2 * NB)
    s12[tid] = (float)((double)scale * (s4[0][tid] + s4[1][tid] + s4[2][tid] + s4[3][tid])) +
               row1[tid];
  __syncthreads();
  double ev = 0.f;
  if (row_ok) {
    float wp = 0.f, v = 0.f;
    if (r > j) {
      v = (r == j + 1) ? 1.f : xr * scale;
      const float y = ys[0][tid] + ys[1][tid];
      float corr = 0.f;
#pragma unroll
      for (int i = 0; i < NB / 4; ++i) {
        corr += vr4[i].x * s12[4 * i] + vr4[i].y * s12[4 * i + 1] + vr4[i].z * s12[4 * i + 2] +
                vr4[i].w * s12[4 * i + 3];
        corr += wr4[i].x * s12[NB + 4 * i] + wr4[i].y * s12[NB + 4 * i + 1] +
                wr4[i].z * s12[NB + 4 * i + 2] + wr4[i].w * s12[NB + 4 * i + 3];
      }
      wp = tau * (y - corr);
      A[(long long)j * lda + r] = (r == j + 1) ? beta : v;
    }
    w.V[(long long)r * NB + c] = v;
    w.Wp[r] = wp;
    ev = (double)wp * v;
  }
  const double sum = block_sum_d(ev, red8);
  if (tid == 0) w.Ep[J] = sum;
}

// ------------------------------------------------------------------ phase C
// W[:, c] = w' + alpha2 v; the next column x (panel corrections applied), its
// norm partials and its dot partials W^T x, V^T x (rows >= j+3) for phase B.
__global__ __launch_bounds__(256) void sytrd_x_kernel(Args a, int j, int c, int s0, int has_next) {
  const int mat = blockIdx.y;
  const float* A = a.A + mat * a.sA;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const int n = a.n, nt = a.nt, lda = a.lda;
  const int J = s0 + blockIdx.x;
  __shared__ float wrow[NB], vrow[NB];
  __shared__ float sal[1];
  __shared__ double red8[4];
  __shared__ float dred[TB][2 * NB + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int jn = j + 1;
  const int r = J * TB + tid;
  const bool row_ok = tid < TB && r < n;
  float4 vr4[NB / 4], wr4[NB / 4];
#pragma unroll
  for (int i = 0; i < NB / 4; ++i) {   // rows past n feed zeros into the dot partials
    vr4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    wr4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float wpr = 0.f, arow = 0.f, vrc = 0.f;
  if (row_ok) {
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) {
      vr4[i] = *(const float4*)(w.V + (long long)r * NB + 4 * i);
      wr4[i] = *(const float4*)(w.W + (long long)r * NB + 4 * i);
    }
    wpr = w.Wp[r];
    vrc = w.V[(long long)r * NB + c];
    if (has_next && r >= jn) arow = A[(long long)jn * lda + r];
  }
  const float tau = a.tau[(long long)mat * n + j];
  double ep = 0.0;
  if (tid < 64)
    for (int q = s0 + lane; q < nt; q += 64) ep += w.Ep[q];
  float wj = 0.f, vj = 0.f, wpj = 0.f;
  if (has_next && tid < NB) {
    wj = w.W[(long long)jn * NB + tid];
    vj = w.V[(long long)jn * NB + tid];
    if (tid == c) wpj = w.Wp[jn];
  }
  if (tid < 64) {
    const double s = wave_reduce_sum_d(ep);
    if (tid == 0) sal[0] = (float)(-0.5 * (double)tau * s);
  }
  __syncthreads();
  const float alpha2 = sal[0];
  if (has_next && tid < NB) {
    // row jn of the panel W/V; column c of W is w' + alpha2 v (this launch
    // writes it), columns beyond c are still zero
    wrow[tid] = (tid < c) ? wj : (tid == c ? wpj + alpha2 * vj : 0.f);
    vrow[tid] = (tid <= c) ? vj : 0.f;
  }
  const float wc = wpr + alpha2 * vrc;
  if (row_ok) w.W[(long long)r * NB + c] = wc;
  if (!has_next) return;
  __syncthreads();
  double nrm = 0.0;
  float x = 0.f;
  if (row_ok && r >= jn) {
    // the W row read above still holds 0 in column c: its final value is wc
    x = arow;
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) {
      x -= vr4[i].x * wrow[4 * i] + vr4[i].y * wrow[4 * i + 1] + vr4[i].z * wrow[4 * i + 2] +
           vr4[i].w * wrow[4 * i + 3];
      x -= wr4[i].x * vrow[4 * i] + wr4[i].y * vrow[4 * i + 1] + wr4[i].z * vrow[4 * i + 2] +
           wr4[i].w * vrow[4 * i + 3];
    }
    x -= wc * vrow[c];
    w.X[r] = x;
    if (r >= jn + 2) nrm = (double)x * x;
  }
  if (tid < TB) {   // x-dot partials for the next column: rows >= jn + 2
    const float xd = (row_ok && r >= jn + 2) ? x : 0.f;
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) {
      dred[tid][4 * i] = wr4[i].x * xd;
      dred[tid][4 * i + 1] = wr4[i].y * xd;
      dred[tid][4 * i + 2] = wr4[i].z * xd;
      dred[tid][4 * i + 3] = wr4[i].w * xd;
      dred[tid][NB + 4 * i] = vr4[i].x * xd;
      dred[tid][NB + 4 * i + 1] = vr4[i].y * xd;
      dred[tid][NB + 4 * i + 2] = vr4[i].z * xd;
      dred[tid][NB + 4 * i + 3] = vr4[i].w * xd;
    }
    dred[tid][c] = wc * xd;
  }
  const double sum = block_sum_d(nrm, red8);   // contains the barrier for dred
  if (tid == 0) w.Np[J] = sum;
  if (tid < 2 * NB) {
    float acc = 0.f;
#pragma unroll 8
    for (int t = 0; t < TB; ++t) acc += dred[t][tid];
    w.Dx[(long long)J * 2 * NB + tid] = acc;
  }
}

// ------------------------------------------------- trailing rank-2w update
__global__ __launch_bounds__(256) void sytrd_trail_kernel(Args a, int q, int wdt, int s0) {
  const int mat = blockIdx.y;
  float* A = a.A + mat * a.sA;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const int n = a.n, nt = a.nt, lda = a.lda;
  __shared__ float vi[TB][NB + 1], wi[TB][NB + 1], vk[TB][NB + 1], wk[TB][NB + 1];
  int I, K;
  tri_index(blockIdx.x, nt - s0, I, K);
  I += s0; K += s0;
  const int tid = threadIdx.x;
  for (int e = tid; e < TB * NB; e += 256) {
    const int rr = e / NB, cc = e - rr * NB;
    const int ri = I * TB + rr, rk = K * TB + rr;
    const bool okc = cc < wdt;
    vi[rr][cc] = (okc && ri < n) ? w.V[(long long)ri * NB + cc] : 0.f;
    wi[rr][cc] = (okc && ri < n) ? w.W[(long long)ri * NB + cc] : 0.f;
    vk[rr][cc] = (okc && rk < n) ? w.V[(long long)rk * NB + cc] : 0.f;
    wk[rr][cc] = (okc && rk < n) ? w.W[(long long)rk * NB + cc] : 0.f;
  }
  __syncthreads();
  const int ty = tid >> 4, tx = tid & 15;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[i][k] = 0.f;
  for (int cc = 0; cc < wdt; ++cc) {
    float av[8], aw[8], bv[8], bw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      av[i] = vi[ty * 8 + i][cc]; aw[i] = wi[ty * 8 + i][cc];
      bv[i] = vk[tx * 8 + i][cc]; bw[i] = wk[tx * 8 + i][cc];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[i][k] += av[i] * bw[k] + aw[i] * bv[k];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = I * TB + ty * 8 + i;
    if (r < q || r >= n) continue;
    float* row = A + (long long)r * lda;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int col = K * TB + tx * 8 + k;
      if (col >= r && col < n) row[col] -= acc[i][k];
    }
  }
}

// ------------------------------------------- panel start: column q's row
__global__ __launch_bounds__(256) void sytrd_prep_kernel(Args a, int q, int s0) {
  const int mat = blockIdx.y;
  const float* A = a.A + mat * a.sA;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const int n = a.n, lda = a.lda;
  const int J = s0 + blockIdx.x;
  __shared__ double red8[4];
  const int tid = threadIdx.x;
  for (int e = tid; e < TB * NB; e += 256) {
    const long long r = (long long)J * TB + e / NB;
    if (r < n) {
      w.V[r * NB + (e % NB)] = 0.f;
      w.W[r * NB + (e % NB)] = 0.f;
    }
  }
  double nrm = 0.0;
  const int r = J * TB + tid;
  if (tid < TB && r < n && r >= q) {
    const float x = A[(long long)q * lda + r];
    w.X[r] = x;
    if (r >= q + 2) nrm = (double)x * x;
  }
  const double s = block_sum_d(nrm, red8);
  if (tid == 0) w.Np[J] = s;
}

__global__ void sytrd_finish_kernel(Args a) {
  const int mat = blockIdx.x;
  const Ws w = ws_at(a.ws + mat * a.sW, a.n);
  const long long o = (long long)mat * a.n + a.n - 1;
  a.d[o] = w.X[a.n - 1];
  a.e[o] = 0.f;
  a.tau[o] = 0.f;
}

int enqueue(const Args& a, int batch, hipStream_t stream) {
  const int n = a.n, nt = a.nt;
  auto blk = [](int r) { return r / TB; };
  auto tri = [](int m) { return m * (m + 1) / 2; };
  hipLaunchKernelGGL(sytrd_prep_kernel, dim3(nt, batch), dim3(256), 0, stream, a, 0, 0);
  int p = 0;
  while (p < n - 1) {
    const int wdt = (n - 1 - p) < NB ? (n - 1 - p) : NB;
    for (int c = 0; c < wdt; ++c) {
      const int j = p + c;
      const int s0 = blk(j + 1), sh = blk(j);
      const int mb = nt - s0;
      hipLaunchKernelGGL(sytrd_symv_kernel, dim3(tri(mb), batch), dim3(256), 0, stream, a, j, s0,
                         sh);
      hipLaunchKernelGGL(sytrd_w_kernel, dim3(mb, batch), dim3(256), 0, stream, a, j, c, s0);
      hipLaunchKernelGGL(sytrd_x_kernel, dim3(mb, batch), dim3(256), 0, stream, a, j, c, s0,
                         (int)(c + 1 < wdt));
    }
    const int q = p + wdt;
    const int s0q = blk(q);
    hipLaunchKernelGGL(sytrd_trail_kernel, dim3(tri(nt - s0q), batch), dim3(256), 0, stream, a, q,
                       wdt, s0q);
    hipLaunchKernelGGL(sytrd_prep_kernel, dim3(nt - s0q, batch), dim3(256), 0, stream, a, q, s0q);
    p = q;
  }
  hipLaunchKernelGGL(sytrd_finish_kernel, dim3(batch), dim3(1), 0, stream, a);
  return (int)hipGetLastError();
}

typedef std::tuple<float*, int, long long, int, int, float*, float*, float*, float*, long long,
                   hipStream_t> GraphKey;
std::mutex g_graph_mu;
std::map<GraphKey, hipGraphExec_t> g_graphs;

}  // namespace

KFAC_API long long kfac_sytrd_ws_floats(int n) { return ws_floats(n); }

namespace {

Args make_args(float* A, int lda, long long strideA, int n, float* d, float* e, float* tau,
               float* ws) {
  Args a;
  a.A = A; a.sA = strideA; a.lda = lda; a.n = n; a.nt = (n + TB - 1) / TB;
  a.ws = ws; a.sW = ws_floats(n);
  a.d = d; a.e = e; a.tau = tau;
  return a;
}

// The cached graph of this argument set, captured (on a private NON-blocking
// stream, under the lock) if missing; nullptr if capture is impossible.
// Capture must not overlap other threads' library calls on the legacy stream
// (hipBLASLt inside rocBLAS refuses them during a capture), so callers build
// the graphs up front (kfac_sytrd_prepare) before concurrent solves start.
hipGraphExec_t graph_for(const Args& a, int batch) {
  const GraphKey key(a.A, a.lda, a.sA, a.n, batch, a.d, a.e, a.tau, a.ws, a.sW, nullptr);
  std::lock_guard<std::mutex> lk(g_graph_mu);
  auto it = g_graphs.find(key);
  if (it != g_graphs.end()) return it->second;
  static hipStream_t cap = nullptr;   // one device per process
  if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  hipGraph_t graph = nullptr;
  if (hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  const int err = enqueue(a, batch, cap);
  hipError_t e2 = hipStreamEndCapture(cap, &graph);
  if (err || e2 != hipSuccess || !graph) {
    if (graph) hipGraphDestroy(graph);
    (void)hipGetLastError();
    return nullptr;
  }
  hipGraphExec_t exec = nullptr;
  e2 = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  if (e2 != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  g_graphs[key] = exec;
  return exec;
}

}  // namespace

// A: batch x n rows of lda floats (row-major, symmetric; the upper triangle is
// read and overwritten), d/e/tau: batch x n, ws: batch x kfac_sytrd_ws_floats(n).
// use_graph: replay the launch sequence as one hipGraph (captured on first use).
KFAC_API int kfac_sytrd_batched(float* A, int lda, long long strideA, int n, int batch, float* d,
                                float* e, float* tau, float* ws, int use_graph,
                                hipStream_t stream) {
  if (n < 2 || batch < 1 || lda < n || (lda & 3) != 0) return -2;
  const Args a = make_args(A, lda, strideA, n, d, e, tau, ws);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return -3;
  // the null stream, or a stream being captured by the caller: plain launches
  if (!use_graph || stream == nullptr || cs != hipStreamCaptureStatusNone)
    return enqueue(a, batch, stream);
  hipGraphExec_t exec = graph_for(a, batch);
  if (!exec) return enqueue(a, batch, stream);
  return (int)hipGraphLaunch(exec, stream);
}

// Build (capture + instantiate) the graph of an argument set without running it.
KFAC_API int kfac_sytrd_prepare(float* A, int lda, long long strideA, int n, int batch, float* d,
                                float* e, float* tau, float* ws) {
  if (n < 2 || batch < 1 || lda < n || (lda & 3) != 0) return -2;
  return graph_for(make_args(A, lda, strideA, n, d, e, tau, ws), batch) ? 0 : -4;
}

// Drop every cached graph that addresses `ws` (the caller frees the buffers).
KFAC_API void kfac_sytrd_forget(float* ws) {
  std::lock_guard<std::mutex> lk(g_graph_mu);
  for (auto it = g_graphs.begin(); it != g_graphs.end();) {
    if (std::get<8>(it->first) == ws) {
      hipGraphExecDestroy(it->second);
      it = g_graphs.erase(it);
    } else {
      ++it;
    }
  }
}
