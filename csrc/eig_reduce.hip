// Batched Householder tridiagonalisation for a ragged batch of K-FAC factors
// (replaces rocSOLVER's sytrd and the round-1 per-class
// csrc/eig_tridiag.hip path).
//
// The reduction is a chain of n dependent columns, so what a column costs in
// launches and per-workgroup latency sets the speed; every matrix of the
// inverse update (all sizes) advances through ONE launch sequence:
//
//   fin(j)   one workgroup per 256 rows (each row's work done once):
//            step 1  Householder scalars of column j-1 from the previous
//                    launches' partial sums (|xh|^2, W^T xh, V^T xh, xh.a,
//                    xh^T yh), re-reduced in a fixed order: deterministic
//            step 2  w_{j-1} = tau (a + s yh - V s1 - W s2) + alpha2 v -> the
//                    panel columns W/V[:, c-1], reflector row j-1, d/e/tau
//            step 3  x_j = A row j - V W[j]^T - W V[j]^T, kept UNNORMALISED
//                    (xh): its Householder scale needs a global norm that
//                    only the next fin knows; y_j = a_j + s_j A22 xh_j is
//                    linear in the scale.  Partial sums for fin(j+1).
//   upd(j)   every NB = 32 columns: A22 -= V W^T + W V^T on the upper 128 x
//            128 tiles, exact-f32 MFMA (v_mfma_f32_32x32x2_f32)
//   symv(j)  yh = A22 xh over the upper tiles (an off-diagonal tile feeds its
//            row and its column block: half the traffic of a full mat-vec),
//            per-tile partials; lean (tile + 256 floats in, no panel data) so
//            the bandwidth-bound early columns run at high occupancy
//
// The recurrence (unnormalised xh, scalars one launch late) is modelled
// exactly in scripts/models/sytrd_fused_model.py (fp64, 1e-15).  Storage:
// row-major, UPPER triangle maintained (== LAPACK lower, column-major); output
// d, e, tau and reflector j in row j (beta at j+1, v[2:] after): the layout
// the compact-WY back-transformation (csrc/eig_library.hip) reads.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int TB = 128;        // symv / update tile
constexpr int FB = 256;        // rows per fin workgroup
constexpr int NB = 32;         // panel width
constexpr int RSW = 64;       // fin partial kinds per block (see K_W / K_V)
constexpr int MAXM = 255;      // matrices per batch
constexpr int NTMAX = 40;      // 128-row blocks (n <= 5120)
constexpr int PQ4 = NTMAX / 4; // float4 loads of a row's yh partials
constexpr int NFMAX = (NTMAX * TB + FB - 1) / FB;   // fin blocks

struct RMat {
  float* A; long long lda; int n; int nt; int nf; int pad;
  float* d; float* e; float* tau;
  float* V; float* W;                     // n x NB (row r: NB floats)
  float* P; float* TS; float* RS; float* XH; float* SC;
  long long sP, sTS, sRS, sXH;            // slot strides (floats); 2 slots each
};

// debug: per-launch phase stamps of workgroup 0 of fin (s_memrealtime, 100 MHz)
__device__ unsigned long long* g_stamps = nullptr;
#define STAMP(k)                                                                            \
  do {                                                                                      \
    if (stamps && tid == 0) stamps[(long long)j * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__device__ inline void tri_index(int t, int mb, int& I, int& K) {
  int i = 0;
  while (t >= mb - i) { t -= mb - i; ++i; }
  I = i; K = i + t;
}

__device__ inline void hh_scalars(double alpha, double sig2, double& beta, double& tau,
                                  double& s) {
  if (sig2 == 0.0) {
    beta = alpha; tau = 0.0; s = 0.0;
  } else {
    beta = -copysign(sqrt(alpha * alpha + sig2), alpha);
    tau = (beta - alpha) / beta;
    s = 1.0 / (alpha - beta);
  }
}

// workgroup -> (matrix, local index) from the launch's host-built offsets:
// one compare per thread (offsets ascending), not a serial scan
__device__ inline void map_block(const int* __restrict__ offs, int nact, int* soff, int& mat,
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

// in-register transpose-reduce of 64 values per lane over the wave: lane L
// ends with the wave sum of value L (63 shuffles; pairwise, fixed order)
template <int M>
__device__ __forceinline__ void butterfly_stage(float (&v)[64], int lane) {
  const bool up = (lane & M) != 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const float send = up ? v[i] : v[i + M];
    const float keep = up ? v[i + M] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
}
__device__ __forceinline__ float butterfly64(float (&v)[64]) {
  const int lane = threadIdx.x & 63;
  butterfly_stage<32>(v, lane);
  butterfly_stage<16>(v, lane);
  butterfly_stage<8>(v, lane);
  butterfly_stage<4>(v, lane);
  butterfly_stage<2>(v, lane);
  butterfly_stage<1>(v, lane);
  return v[0];
}

// ------------------------------------------------------------------- fin
// partial-sum kinds of a fin block (RSW = 64: one per lane of the butterfly):
// |xh|^2, xh.a, W^T xh and V^T xh over the panel columns before the current
// one (at most NB - 1 of them)
constexpr int K_W = 2, K_V = 2 + (NB - 1);
static_assert(K_V + NB - 1 == RSW, "fin partial kinds must fill one wave");
constexpr int TSQ = (NTMAX * (NTMAX + 1) / 2 + 255) / 256;   // float4 tile-sum loads per lane
constexpr int NFP = (NFMAX + 3) / 4 * 4;                      // RS: blocks per kind (float4 rows)
// Every wave keeps its loads under the 63 a wave can have in flight
// (vmcnt is 6 bits): past that, each extra batch costs a full round trip.

struct FinWave {                  // one wave's private slice (no barrier needed)
  float s12[2 * NB];              // s1, s2
  float vw[4][NB];                // V[j], W[j], V[j+1], W[j+1] (current panel columns)
};

// Every wave of every fin workgroup derives column j-1's scalars and rows
// j / j+1 itself (redundantly, from the same partials, in the same order), so
// the waves never wait for each other until the block's partial sums at the
// end; the cross-lane sums are DPP / permlane (common.h wave_sum*).
__global__ __launch_bounds__(256) void sytrd_fin_kernel(const RMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int j) {
  __shared__ FinWave SW[4];
  __shared__ float wred[4][RSW];
  __shared__ int soff[MAXM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long* const stamps = blockIdx.x == 0 ? g_stamps : nullptr;
  STAMP(0);
  if (stamps && tid == 0) stamps[(long long)j * 16 + 8] = __builtin_amdgcn_s_memtime();
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const RMat M = mats[mi];
  const int n = M.n, nt = M.nt;
  const long long lda = M.lda;
  const int bf = j / FB + local;           // this workgroup's 256-row block
  const int r = bf * FB + tid;
  const bool lead = (local == 0 && wave == 0);
  const bool fin = (j == n - 1);
  const bool has1 = (j + 1 < n);
  const int c = j % NB;
  const int cp = (j >= 1) ? (c == 0 ? NB - 1 : c - 1) : 0;
  const bool pstart = (c == 0 && j > 0);
  const int cc = pstart ? NB : c;          // panel columns subtracted from A rows j, j+1
  const int cs = j & 1, ps = cs ^ 1;
  const int s0p = j / TB;                  // first tile block of symv(j-1)
  const int ntp = (nt + 3) & ~3;
  const int ntri = (nt - s0p) * (nt - s0p + 1) / 2;   // tiles of symv(j-1)
  const int f0p = (j - 1) / FB;            // first fin block of fin(j-1)
  const AS1 float* Pp = gptr(M.P) + ps * M.sP;
  const AS1 float* XHp = gptr(M.XH) + ps * M.sXH;
  const AS1 float* RSp = gptr(M.RS) + ps * M.sRS;
  const AS1 float* TSp = gptr(M.TS) + ps * M.sTS;
  AS1 float* const gA = gptr(M.A);
  AS1 float* const gV = gptr(M.V);
  AS1 float* const gW = gptr(M.W);
  AS1 float* const gSC = gptr(M.SC);
  STAMP(1);

  // ---- every load up front, branch-free (one memory round trip)
  const bool j1 = (j >= 1);
  // fin(j-1) block partials, kind-major [RSW][NFP]: lane = kind, float4s of
  // 4 blocks (blocks f0p .. nf-1 are valid)
  fx4 rq[NFP / 4];
#pragma unroll
  for (int u = 0; u < NFP / 4; ++u) rq[u] = *(const AS1 fx4*)(RSp + lane * NFP + 4 * u);
  fx4 tq[TSQ];                             // symv(j-1) tile sums, triangle order
#pragma unroll
  for (int u = 0; u < TSQ; ++u) tq[u] = *(const AS1 fx4*)(TSp + 4 * lane + 256 * u);
  const bool okp = j1 && lane >= s0p && lane < nt;
  const float pj = gld_if(Pp, j * ntp + lane, okp, 0.f);
  const float pj1 = gld_if(Pp, (j + 1) * ntp + lane, okp && has1, 0.f);
  const float xhj1 = gld_if(XHp, j + 1, j1 && has1, 0.f);
  const float alpha = gSC[ps * 4];
  const float dprev = gSC[ps * 4 + 1];
  float vj = gld_if(gV, j * NB + lane, lane < NB, 0.f);
  float wj = gld_if(gW, j * NB + lane, lane < NB, 0.f);
  float vj1 = gld_if(gV, (j + 1) * NB + lane, lane < NB && has1, 0.f);
  float wj1 = gld_if(gW, (j + 1) * NB + lane, lane < NB && has1, 0.f);
  const float ajj = gA[(long long)j * lda + j];
  const float ajj1 = gld_if(gA, (long long)j * lda + j + 1, has1, 0.f);
  // this thread's row (loads from a clamped row; unused lanes masked later)
  const bool rok = r < n && r >= j;
  const int rc = min(r, n - 1);
  float vr[NB], wr[NB];
  {
    const AS1 fx4* v4 = (const AS1 fx4*)(gV + rc * NB);
    const AS1 fx4* w4 = (const AS1 fx4*)(gW + rc * NB);
#pragma unroll
    for (int x = 0; x < NB / 4; ++x) {
      const fx4 a4 = v4[x], b4 = w4[x];
      vr[4 * x] = a4.x; vr[4 * x + 1] = a4.y; vr[4 * x + 2] = a4.z; vr[4 * x + 3] = a4.w;
      wr[4 * x] = b4.x; wr[4 * x + 1] = b4.y; wr[4 * x + 2] = b4.z; wr[4 * x + 3] = b4.w;
    }
  }
  const float arow = gA[(long long)j * lda + rc];                              // base row j
  const float brow = gld_if(gA, (long long)(j + 1) * lda + rc, has1 && r >= j + 1, 0.f);
  const float xhp = XHp[rc];
  fx4 pq[PQ4];
  {
    const AS1 fx4* pp = (const AS1 fx4*)(Pp + rc * ntp);
    const fx4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < PQ4; ++u) pq[u] = gld_if(pp, u, j1 && 4 * u + 3 >= s0p && 4 * u < nt, z4);
  }
  double pK = 0.0, pT = 0.0;               // this lane's kind over the blocks; tile sums
#pragma unroll
  for (int u = 0; u < NFP / 4; ++u) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int bb = 4 * u + e;
      pK += (j1 && bb >= f0p && bb < M.nf) ? (double)rq[u][e] : 0.0;
    }
  }
#pragma unroll
  for (int u = 0; u < TSQ; ++u) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = 4 * lane + 256 * u + e;
      pT += (j1 && f < ntri) ? (double)tq[u][e] : 0.0;
    }
  }
  // kinds to their consumers: |xh|^2 and xh.a broadcast, W_x / V_x to lane x
  const double pW = __shfl(pK, (K_W + lane) & 63, 64);
  const double pV = __shfl(pK, (K_V + lane) & 63, 64);
  const double sig2_b = __shfl(pK, 0, 64), xa_b = __shfl(pK, 1, 64);
  STAMP(2);

  // ---- step 1 (per wave): scalars of column j-1; step 2 for rows j, j+1
  double beta_p = 0.0, tau_p = 0.0, s_p = 0.0, alpha2 = 0.0;
  float s1f = 0.f, s2f = 0.f;
  if (j >= 1) {
    const double sig2 = sig2_b, xa = xa_b, xy = wave_sum_d(pT);
    hh_scalars((double)alpha, sig2, beta_p, tau_p, s_p);
    // s1 = W^T v, s2 = V^T v over rows >= j (v[j] = 1): row j of the panel
    double s1 = 0.0, s2 = 0.0;
    if (lane < cp) {
      s1 = (double)wj + s_p * pW;
      s2 = (double)vj + s_p * pV;
    }
    const double s1s2 = wave_sum_d(s1 * s2);
    const double vy = (double)ajj + 2.0 * s_p * xa + s_p * s_p * xy;
    alpha2 = -0.5 * tau_p * tau_p * (vy - 2.0 * s1s2);
    s1f = (float)s1;
    s2f = (float)s2;
    const float yv = wave_sum(pj), yv1 = wave_sum(pj1);
    const float cj = wave_sum(lane < cp ? vj * s1f + wj * s2f : 0.f);
    const float cj1 = wave_sum(lane < cp ? vj1 * s1f + wj1 * s2f : 0.f);
    const float ww = (float)(tau_p * ((double)ajj + s_p * (double)yv - (double)cj) + alpha2);
    const float vv1 = (float)(s_p * (double)xhj1);
    const float ww1 = (float)(tau_p * ((double)ajj1 + s_p * (double)yv1 - (double)cj1) +
                              alpha2 * (double)vv1);
    if (lane == cp) {
      vj = 1.f; wj = ww;
      vj1 = vv1; wj1 = ww1;
    }
    if (lead) {
      if (lane == cp) {
        gV[j * NB + cp] = 1.f;
        gW[j * NB + cp] = ww;
      }
      if (lane == 0) {
        M.d[j - 1] = dprev;
        M.e[j - 1] = (float)beta_p;
        M.tau[j - 1] = (float)tau_p;
        gA[(long long)(j - 1) * lda + j] = (float)beta_p;
      }
    }
  }
  {   // d_j = A(j, j) - 2 V[j] . W[j] over the panel columns
    const double dd = wave_sum_d(lane < cc ? (double)vj * (double)wj : 0.0);
    if (lead && lane == 0) {
      const float dj = (float)((double)ajj - 2.0 * dd);
      if (fin) {
        M.d[j] = dj;
        M.e[j] = 0.f;
        M.tau[j] = 0.f;
      } else {
        gSC[cs * 4 + 1] = dj;
      }
    }
  }
  FinWave& F = SW[wave];
  if (lane < NB) {
    F.s12[lane] = s1f;
    F.s12[NB + lane] = s2f;
    F.vw[0][lane] = vj; F.vw[1][lane] = wj;
    F.vw[2][lane] = vj1; F.vw[3][lane] = wj1;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  STAMP(3);

  // ---- step 2, this thread's row (r >= j+1)
  if (j >= 1 && rok && r >= j + 1) {
    float yh = 0.f;
#pragma unroll
    for (int u = 0; u < PQ4; ++u) {
      if (4 * u >= s0p) yh += pq[u].x;
      if (4 * u + 1 >= s0p) yh += pq[u].y;
      if (4 * u + 2 >= s0p) yh += pq[u].z;
      if (4 * u + 3 >= s0p) yh += pq[u].w;
    }
    float corr = 0.f;
#pragma unroll
    for (int x = 0; x < NB; ++x)
      if (x < cp) corr += vr[x] * F.s12[x] + wr[x] * F.s12[NB + x];
    const float vmy = (float)(s_p * (double)xhp);
    const float wmy =
        (float)(tau_p * ((double)arow + s_p * (double)yh - (double)corr) + alpha2 * (double)vmy);
#pragma unroll
    for (int x = 0; x < NB; ++x)
      if (x == cp) { vr[x] = vmy; wr[x] = wmy; }
    gV[r * NB + cp] = vmy;
    gW[r * NB + cp] = wmy;
    gA[(long long)(j - 1) * lda + r] = vmy;      // reflector j-1: v[2:] (r >= j+1)
  }
  if (fin) return;      // uniform: d/e/tau of the last two columns are written
  STAMP(4);

  // ---- step 3: x_j (rows >= j+1), a_j; alpha_j
  float xmy = 0.f, amy = 0.f;
  if (rok && r >= j + 1) {
    float corr = 0.f, corr1 = 0.f;
#pragma unroll
    for (int x = 0; x < NB; ++x) {
      if (x < cc) {
        corr += vr[x] * F.vw[1][x] + wr[x] * F.vw[0][x];
        corr1 += vr[x] * F.vw[3][x] + wr[x] * F.vw[2][x];
      }
    }
    xmy = arow - corr;
    amy = pstart ? brow - corr1 : brow;    // a_j = row j+1 of the NEW panel's base
  }
  const float xh = (rok && r >= j + 2) ? xmy : 0.f;
  if (r == j + 1 && r < n) gSC[cs * 4] = xmy;      // alpha_j
  if (r < n) gptr(M.XH)[cs * M.sXH + r] = xh;
  // ---- partial sums for fin(j+1): wave butterfly, then 4 waves in order
  {
    const int cn = pstart ? 0 : c;                // the current panel's columns (< NB)
    float pv[64];
    pv[0] = xh * xh;
    pv[1] = xh * amy;
#pragma unroll
    for (int x = 0; x < NB - 1; ++x) {
      pv[K_W + x] = (x < cn) ? wr[x] * xh : 0.f;
      pv[K_V + x] = (x < cn) ? vr[x] * xh : 0.f;
    }
    wred[wave][lane] = butterfly64(pv);
  }
  __syncthreads();
  STAMP(5);
  if (tid < RSW)
    gptr(M.RS)[cs * M.sRS + tid * NFP + bf] =
        (float)(((double)wred[0][tid] + (double)wred[1][tid]) +
                ((double)wred[2][tid] + (double)wred[3][tid]));
  STAMP(6);
  if (stamps && tid == 0) stamps[(long long)j * 16 + 9] = __builtin_amdgcn_s_memtime();
}

// ------------------------------------------------------------------- upd
// A[I][K] -= L_I R_K^T with L = [V | W], R = [W | V] (rows >= q+1, upper):
// the panel's rank-2NB update, exact-f32 MFMA, 4 waves of 64 x 64.
__global__ __launch_bounds__(256) void sytrd_upd_kernel(const RMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int q) {
  __shared__ float sL[TB][2 * NB + 1];
  __shared__ float sR[TB][2 * NB + 1];
  __shared__ int soff[MAXM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const RMat M = mats[mi];
  const int n = M.n, nt = M.nt;
  const int s0 = (q + 1) / TB;
  int I, K;
  tri_index(local, nt - s0, I, K);
  I += s0; K += s0;
  const AS1 float* gV = gptr(M.V);
  const AS1 float* gW = gptr(M.W);
#pragma unroll
  for (int e0 = 0; e0 < TB * NB; e0 += 256) {
    const int e = e0 + tid;
    const int rr = e / NB, x = e - rr * NB;
    const int ri = I * TB + rr, rk = K * TB + rr;
    const float vi = gld_if(gV, ri * NB + x, ri < n, 0.f);
    const float wi = gld_if(gW, ri * NB + x, ri < n, 0.f);
    const float vk = gld_if(gV, rk * NB + x, rk < n, 0.f);
    const float wk = gld_if(gW, rk * NB + x, rk < n, 0.f);
    sL[rr][x] = vi; sL[rr][NB + x] = wi;
    sR[rr][x] = wk; sR[rr][NB + x] = vk;
  }
  __syncthreads();
  const int wr = wave >> 1, wc = wave & 1;          // 2 x 2 waves of 64 x 64
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[a][b][x] = 0.f;
#pragma unroll 4
  for (int kk = 0; kk < NB; ++kk) {                 // k = 2 kk + lh over 2 NB
    const int k = 2 * kk + lh;
    float av[2], bv[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) av[a] = sL[wr * 64 + a * 32 + l31][k];
#pragma unroll
    for (int b = 0; b < 2; ++b) bv[b] = sR[wc * 64 + b * 32 + l31][k];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
  // C/D map of 32x32: row = (x&3) + 8 (x>>2) + 4 lh, col = lane & 31.  Per
  // 32 x 32 block: its 16 old values loaded (clamped, branch-free), then stored
  AS1 float* const A = gptr(M.A);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float old[16];
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh;
        const int gc = K * TB + wc * 64 + b * 32 + l31;
        const bool ok = gr >= q + 1 && gr < n && gc >= gr && gc < n;
        old[x] = gld_if(A, (long long)gr * M.lda + gc, ok, 0.f);
      }
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh;
        const int gc = K * TB + wc * 64 + b * 32 + l31;
        if (gr >= q + 1 && gr < n && gc >= gr && gc < n)
          A[(long long)gr * M.lda + gc] = old[x] - acc[a][b][x];
      }
    }
}

// ------------------------------------------------------------------- symv
__global__ __launch_bounds__(256) void sytrd_symv2_kernel(const RMat* __restrict__ mats,
                                                          const int* __restrict__ offs, int nact,
                                                          int j) {
  __shared__ float sv[2][TB];
  __shared__ float rowred[TB][33];
  __shared__ float colred[4][TB];
  __shared__ double tred[2];
  __shared__ int soff[MAXM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mi, local;
  map_block(offs, nact, soff, mi, local);
  const RMat M = mats[mi];
  const int n = M.n, nt = M.nt;
  const long long lda = M.lda;
  const int s0 = (j + 1) / TB;
  int I, K;
  tri_index(local, nt - s0, I, K);
  I += s0; K += s0;
  const bool diag = (I == K);
  const int cs = j & 1;
  const int ntp = (nt + 3) & ~3;
  // xh of the rows of blocks I and K (written by fin(j))
  {
    const int h = tid >> 7, lr = tid & (TB - 1);
    const int rr = (h ? K : I) * TB + lr;
    sv[h][lr] = gld_if(gptr(M.XH) + cs * M.sXH, rr, rr < n, 0.f);
  }
  const int hw = lane >> 5, cl = lane & 31;
  const int kk0 = cl * 4, k0 = K * TB + kk0;
  // branch-free tile loads: row clamped to n-1, column start clamped inside
  // the row (lda % 4 == 0, lda >= n); out-of-range entries zeroed after
  const int kc = min(k0, (int)lda - 4);
  const AS1 float* gA = gptr(M.A);
  float4 q[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int rr = I * TB + wave * 32 + it * 2 + hw;
    const fx4 t = *(const AS1 fx4*)(gA + (long long)min(rr, n - 1) * lda + kc);
    const bool ok = rr < n;
    q[it] = make_float4((ok && k0 < n) ? t.x : 0.f, (ok && k0 + 1 < n) ? t.y : 0.f,
                        (ok && k0 + 2 < n) ? t.z : 0.f, (ok && k0 + 3 < n) ? t.w : 0.f);
  }
  __syncthreads();
  float ca[4] = {0.f, 0.f, 0.f, 0.f};
  const float vk0 = sv[1][kk0], vk1 = sv[1][kk0 + 1], vk2 = sv[1][kk0 + 2], vk3 = sv[1][kk0 + 3];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int rr = wave * 32 + it * 2 + hw;
    float x0 = q[it].x, x1 = q[it].y, x2 = q[it].z, x3 = q[it].w;
    const float vrr = sv[0][rr];
    if (diag) {   // upper triangle only: row sums take k >= r, column sums k > r
      x0 = (kk0 >= rr) ? x0 : 0.f;
      x1 = (kk0 + 1 >= rr) ? x1 : 0.f;
      x2 = (kk0 + 2 >= rr) ? x2 : 0.f;
      x3 = (kk0 + 3 >= rr) ? x3 : 0.f;
      ca[0] += (kk0 > rr) ? x0 * vrr : 0.f;
      ca[1] += (kk0 + 1 > rr) ? x1 * vrr : 0.f;
      ca[2] += (kk0 + 2 > rr) ? x2 * vrr : 0.f;
      ca[3] += (kk0 + 3 > rr) ? x3 * vrr : 0.f;
    } else {
      ca[0] += x0 * vrr; ca[1] += x1 * vrr; ca[2] += x2 * vrr; ca[3] += x3 * vrr;
    }
    rowred[rr][cl] = x0 * vk0 + x1 * vk1 + x2 * vk2 + x3 * vk3;
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) ca[x] += __shfl_xor(ca[x], 32, 64);
  if (hw == 0) {
#pragma unroll
    for (int x = 0; x < 4; ++x) colred[wave][kk0 + x] = ca[x];
  }
  __syncthreads();
  AS1 float* const Pc = gptr(M.P) + cs * M.sP;
  double tp = 0.0;
  if (tid < TB) {
    float rs = 0.f;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) rs += rowred[tid][l];
    const float csum = colred[0][tid] + colred[1][tid] + colred[2][tid] + colred[3][tid];
    if (diag) {
      Pc[((long long)I * TB + tid) * ntp + K] = rs + csum;
      tp = (double)sv[0][tid] * (double)(rs + csum);
    } else {
      Pc[((long long)I * TB + tid) * ntp + K] = rs;
      Pc[((long long)K * TB + tid) * ntp + I] = csum;
      tp = (double)sv[0][tid] * (double)rs + (double)sv[1][tid] * (double)csum;
    }
  }
  tp = wave_sum_d(tp);
  if (lane == 0 && wave < 2) tred[wave] = tp;
  __syncthreads();
  if (tid == 0) gptr(M.TS)[cs * M.sTS + local] = (float)(tred[0] + tred[1]);   // triangle order
}

// ------------------------------------------------------------------ host
struct RPlan {
  RMat* d_mats = nullptr;
  int* d_offs = nullptr;        // [3][nmax][nm + 1]: fin, upd, symv workgroup offsets
  std::vector<int> n_sorted;    // descending
  std::vector<int> grid[3];     // [nmax] total workgroups per launch kind
  std::vector<int> nact[3];
  int nmax = 0;
  hipGraphExec_t exec = nullptr;
};

inline int h_tri(int m) { return m * (m + 1) / 2; }

// workgroups of matrix n at column j: fin, upd (panel start only), symv
void counts(int n, int j, int out[3]) {
  const int nt = (n + TB - 1) / TB, nf = (n + FB - 1) / FB;
  out[0] = (j <= n - 1) ? nf - j / FB : 0;
  out[1] = (j % NB == 0 && j > 0 && j <= n - 2) ? h_tri(nt - (j + 1) / TB) : 0;
  out[2] = (j <= n - 2) ? h_tri(nt - (j + 1) / TB) : 0;
}

int enqueue(const RPlan& P, hipStream_t stream) {
  const int nm = (int)P.n_sorted.size();
  const size_t kstride = (size_t)P.nmax * (nm + 1);
  for (int j = 0; j < P.nmax; ++j) {
    const int* of = P.d_offs + (size_t)j * (nm + 1);
    hipLaunchKernelGGL(sytrd_fin_kernel, dim3(P.grid[0][j]), dim3(256), 0, stream,
                       P.d_mats, of, P.nact[0][j], j);
    if (P.grid[1][j] > 0)
      hipLaunchKernelGGL(sytrd_upd_kernel, dim3(P.grid[1][j]), dim3(256), 0, stream, P.d_mats,
                         of + kstride, P.nact[1][j], j);
    if (P.grid[2][j] > 0)
      hipLaunchKernelGGL(sytrd_symv2_kernel, dim3(P.grid[2][j]), dim3(256), 0, stream,
                         P.d_mats, of + 2 * kstride, P.nact[2][j], j);
  }
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, RPlan> g_plans;

}  // namespace

// workspace floats per matrix (V, W and the 2-slot partial rings)
KFAC_API long long kfac_reduce_ws_floats(int n) {
  const long long nt = (n + TB - 1) / TB, nf = (n + FB - 1) / FB;
  auto a16 = [](long long x) { return (x + 15) / 16 * 16; };
  long long s = 2 * a16((long long)n * NB);               // V, W
  s += 2 * a16(nt * TB * ((nt + 3) / 4 * 4));             // P (row-major partials)
  s += 2 * std::max<long long>(a16(nt * nt), 256LL * TSQ);   // TS
  s += 2 * a16((long long)RSW * NFP);                     // RS (kind-major)
  s += 2 * a16(n);                                        // XH
  s += a16(8);                                            // SC
  return (s + 63) / 64 * 64;
}

struct KfacReduceRecord {
  float* A; long long lda; float* d; float* e; float* tau; float* ws; long long n;
};

namespace {

RPlan* plan_for(const KfacReduceRecord* recs, int count, bool capture, int* err) {
  std::vector<int> order(count);
  for (int i = 0; i < count; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return recs[a].n > recs[b].n; });
  std::vector<RMat> mats;
  for (int oi : order) {
    const KfacReduceRecord& r = recs[oi];
    if (r.n < 2 || r.lda < r.n || (r.lda & 3)) { *err = -2; return nullptr; }
    if (r.n > NTMAX * TB) { *err = -6; return nullptr; }
    RMat M;
    memset(&M, 0, sizeof(M));
    M.A = r.A; M.lda = r.lda; M.n = (int)r.n; M.nt = (int)((r.n + TB - 1) / TB);
    M.nf = (int)((r.n + FB - 1) / FB);
    M.d = r.d; M.e = r.e; M.tau = r.tau;
    const long long nt = M.nt, n = r.n;
    float* p = r.ws;
    auto take = [&](long long fl) { float* o = p; p += (fl + 15) / 16 * 16; return o; };
    M.V = take(n * NB); M.W = take(n * NB);
    M.sP = (nt * TB * ((nt + 3) / 4 * 4) + 15) / 16 * 16; M.P = take(2 * M.sP);
    M.sTS = std::max<long long>((nt * nt + 15) / 16 * 16, 256LL * TSQ);   // float4 reads
    M.TS = take(2 * M.sTS);
    M.sRS = RSW * NFP; M.RS = take(2 * M.sRS);
    M.sXH = (n + 15) / 16 * 16; M.XH = take(2 * M.sXH);
    M.SC = take(8);
    mats.push_back(M);
  }
  const std::string key((const char*)mats.data(), sizeof(RMat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    RPlan P;
    for (const RMat& M : mats) P.n_sorted.push_back(M.n);
    P.nmax = P.n_sorted[0];
    const int nm = (int)mats.size();
    if ((*err = (int)hipMalloc(&P.d_mats, sizeof(RMat) * mats.size())) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(RMat) * mats.size(),
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    std::vector<int> offs((size_t)3 * P.nmax * (nm + 1), 0);
    for (int k = 0; k < 3; ++k) {
      P.grid[k].assign(P.nmax, 0);
      P.nact[k].assign(P.nmax, 0);
    }
    for (int j = 0; j < P.nmax; ++j) {
      int acc[3] = {0, 0, 0};
      for (int i = 0; i < nm; ++i) {
        int cnt[3];
        counts(P.n_sorted[i], j, cnt);
        for (int k = 0; k < 3; ++k) {
          offs[((size_t)k * P.nmax + j) * (nm + 1) + i] = acc[k];
          if (cnt[k] > 0) P.nact[k][j] = i + 1;
          acc[k] += cnt[k];
        }
      }
      for (int k = 0; k < 3; ++k) {
        offs[((size_t)k * P.nmax + j) * (nm + 1) + nm] = acc[k];
        P.grid[k][j] = acc[k];
      }
    }
    if ((*err = (int)hipMalloc(&P.d_offs, sizeof(int) * offs.size())) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_offs, offs.data(), sizeof(int) * offs.size(),
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    it = g_plans.emplace(key, P).first;
  }
  RPlan* plan = &it->second;
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

// Tridiagonalise `count` symmetric matrices (any sizes <= 5120) with one
// launch sequence for all of them: A (n x lda, row-major, upper triangle read
// and overwritten by the reflectors), d, e, tau (n floats each), ws
// (kfac_reduce_ws_floats(n) floats, 256-byte aligned).
KFAC_API int kfac_reduce_batched(const KfacReduceRecord* recs, int count, int use_graph,
                                 hipStream_t stream) {
  if (count <= 0 || count > MAXM) return count <= 0 ? 0 : -5;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  int err = 0;
  RPlan* plan = plan_for(recs, count, graph, &err);
  if (!plan) return err ? err : -4;
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}

// debug: record phase stamps of the first fin workgroup of every column into
// `buf` (nmax x 16 uint64), or stop with nullptr
KFAC_API int kfac_reduce_stamps(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
}

KFAC_API int kfac_reduce_prepare(const KfacReduceRecord* recs, int count) {
  int err = 0;
  return plan_for(recs, count, true, &err) ? 0 : (err ? err : -4);
}
