// Fused Householder tridiagonalisation: ONE launch per column for a ragged
// batch of K-FAC factors (replaces the 3-launch-per-column
// csrc/eig_tridiag.hip path and rocSOLVER's sytrd).
//
// The reduction is a chain of n dependent columns; on MI355X each kernel
// boundary costs ~1.5-3 us, so the launch count per column sets the floor
// (profiles/r1_tridiag_kernel_stats_4608x3.csv: 3 launches = 20 us/column).
// Launch K(j) does, for EVERY matrix of the batch that still has column j:
//
//   step 1  the Householder scalars of column j-1 from the partial sums the
//           previous launch left (|xh|^2, W^T xh, V^T xh, xh.a, xh^T yh:
//           per-block / per-tile partials re-reduced in a fixed order, so the
//           result is deterministic -- no atomics)
//   step 2  w_{j-1} = tau (a + s yh - V s1 - W s2) + alpha2 v for the rows the
//           workgroup needs; the diagonal-tile workgroups store W/V columns,
//           the reflector row and the next vector
//   panel   at a panel start (every NB columns) the tile is updated in place,
//           A -= V W^T + W V^T, before it is used
//   step 3  x_j = base row j - V W[j]^T - W V[j]^T, kept UNNORMALISED (xh):
//           its Householder scale needs a global norm that only the next
//           launch knows -- y_j = a_j + s_j A22 xh_j is linear in the scale
//   step 4  yh = A22 xh over the upper 128 x 128 tiles (each off-diagonal
//           tile feeds both its row and its column block: half the traffic of
//           a full mat-vec), per-tile partials
//
// Base rows j, j+1 come from a snapshot the previous launch took, so a launch
// that rewrites tiles (panel start) never reads rows another workgroup of the
// same launch is writing.  The recurrence is modelled exactly (fp64, 1e-15)
// in scripts/models/sytrd_fused_model.py.  Storage as before: row-major,
// UPPER triangle maintained (== LAPACK lower, column-major); output d, e, tau
// and reflector j in row j (beta at j+1, v[2:] after) -- the layout the
// compact-WY back-transformation (csrc/eig_library.hip) reads.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int TB = 128;        // symv / update tile
constexpr int NB = 32;         // panel width
constexpr int RSW = 2 + 2 * NB + 2;   // row-block partials: |xh|^2, xh.a, W^T xh, V^T xh (+pad)
constexpr int MAXM = 255;      // matrices per batch (one launch-offset row each)
constexpr int NTMAX = 40;      // row blocks (n <= 5120): partial loads stay in registers
constexpr int PQ4 = NTMAX / 4; // float4 loads of a row's yh partials
constexpr int RSL = (NTMAX * RSW + 255) / 256;    // row-block partial loads per thread
constexpr int TSL = (NTMAX * NTMAX + 255) / 256;  // tile partial loads per thread

// debug: per-launch phase stamps of workgroup 0 (s_memrealtime, 100 MHz),
// enabled by kfac_reduce_stamps(buffer); null in normal runs
__device__ unsigned long long* g_stamps = nullptr;
#define STAMP(k)                                                                     \
  do {                                                                               \
    if (stamps && tid == 0) stamps[(long long)j * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

struct RMat {
  float* A; long long lda; int n; int nt;
  float* d; float* e; float* tau;
  float* V; float* W;                     // n x NB (row r: NB floats)
  float* P; float* TS; float* RS; float* XH; float* SN; float* SC;
  long long sP, sTS, sRS, sXH, sSN;       // slot strides (floats); 2 slots each
};

__device__ inline void tri_index(int t, int mb, int& I, int& K) {
  int i = 0;
  while (t >= mb - i) { t -= mb - i; ++i; }
  I = i; K = i + t;
}

__device__ inline int tri(int m) { return m * (m + 1) / 2; }

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

// copy base rows 0 and 1 into snapshot slot 1 (read by K(0))
__global__ __launch_bounds__(256) void reduce_prep_kernel(const RMat* __restrict__ mats) {
  const RMat M = mats[blockIdx.y];
  float* sn = M.SN + M.sSN;   // slot 1
  for (int r = blockIdx.x * 256 + threadIdx.x; r < M.n; r += gridDim.x * 256) {
    sn[r] = M.A[r];                                   // row 0 (upper: all columns)
    sn[M.n + r] = (r >= 1) ? M.A[M.lda + r] : 0.f;    // row 1, columns >= 1
  }
}

struct Shared {
  // step 1 / scalar rows
  double scal[8];                 // beta, tau, s, alpha2, prev d, alpha
  float s12[2 * NB];              // s1, s2
  float vwj[4][NB];               // V[j], W[j], V[j+1], W[j+1] (full panel columns)
  double red[4 * RSW];
  // symv
  float sv[2][TB];
  float rowred[TB][33];
  float colred[4][TB];
  int mat, tile;
};

__global__ __launch_bounds__(256) void sytrd_col_kernel(const RMat* __restrict__ mats,
                                                        const int* __restrict__ offs, int nact,
                                                        int j) {
  extern __shared__ __attribute__((aligned(16))) float upd[];   // panel start: V/W rows
  __shared__ Shared S;
  __shared__ int soff[MAXM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long* const stamps = blockIdx.x == 0 ? g_stamps : nullptr;
  STAMP(0);
  // ---- workgroup -> (matrix, tile): this launch's tile offsets (host-built,
  //      one parallel load) searched in LDS
  if (tid <= nact) soff[tid] = offs[tid];
  __syncthreads();
  if (tid == 0) {
    const int b = blockIdx.x;
    int mi = 0;
    while (mi + 1 < nact && soff[mi + 1] <= b) ++mi;
    S.mat = mi;
    S.tile = b - soff[mi];
  }
  __syncthreads();
  const RMat M = mats[S.mat];
  const int n = M.n, nt = M.nt;
  STAMP(1);
  const long long lda = M.lda;
  const bool fin = (j == n - 1);          // finisher: column n-2's tail, d[n-1]
  const int s0 = (j + 1) / TB;
  int I = 0, K = 0;
  if (!fin) {
    tri_index(S.tile, nt - s0, I, K);
    I += s0; K += s0;
  }
  const bool lead = (S.tile == 0);
  const bool diag = (I == K) && !fin;
  const int c = j % NB;                    // column j's panel position
  const int cp = (j >= 1) ? (c == 0 ? NB - 1 : c - 1) : 0;   // column j-1's position
  const bool pstart = (c == 0 && j > 0);
  const int cc = pstart ? NB : c;          // panel columns subtracted from base rows
  const int cs = j & 1, ps = cs ^ 1;
  const int s0p = j / TB;                  // first block of launch j-1
  const float* Pp = M.P + ps * M.sP;
  const float* SNp = M.SN + ps * M.sSN;
  const float* XHp = M.XH + ps * M.sXH;

  // ---- this thread's row: t < 128 -> block I, else block K
  const int h = tid >> 7, lr = tid & (TB - 1);
  const int r = (h ? K : I) * TB + lr;
  const bool rok = !fin && r < n;

  // ---- tile loads first (independent of everything below)
  const int hw = lane >> 5, cl = lane & 31;
  const int kk0 = cl * 4, k0 = K * TB + kk0;
  float4 q[16];
  if (!fin) {
    const bool full_cols = (k0 + 3 < n);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int rr = I * TB + wave * 32 + it * 2 + hw;
      q[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rr < n) {
        const float* row = M.A + (long long)rr * lda;
        if (full_cols) {
          q[it] = *(const float4*)(row + k0);
        } else {
          if (k0 < n) q[it].x = row[k0];
          if (k0 + 1 < n) q[it].y = row[k0 + 1];
          if (k0 + 2 < n) q[it].z = row[k0 + 2];
        }
      }
    }
  }
  // ---- every other load of the launch, issued before the first barrier
  //      (the chain is latency bound: one memory round trip, not one per loop)
  float vr[NB], wr[NB];
#pragma unroll
  for (int x = 0; x < NB; ++x) { vr[x] = 0.f; wr[x] = 0.f; }
  float xhp = 0.f, arow = 0.f, brow = 0.f;
  float4 pq[PQ4];                         // this row's yh partials (row-major in P)
#pragma unroll
  for (int u = 0; u < PQ4; ++u) pq[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int ntp = (nt + 3) & ~3;
  const bool prow = rok && r >= j;
  if (prow) {
    // only the panel columns this launch reads (cc: x_j / a_j corrections,
    // cp < cc: w_{j-1}, c <= cc: partial sums; all NB at a panel start)
#pragma unroll
    for (int x = 0; x < NB / 4; ++x) {
      if (4 * x < cc) {
        const float4 a4 = *(const float4*)(M.V + (long long)r * NB + 4 * x);
        const float4 b4 = *(const float4*)(M.W + (long long)r * NB + 4 * x);
        vr[4 * x] = a4.x; vr[4 * x + 1] = a4.y; vr[4 * x + 2] = a4.z; vr[4 * x + 3] = a4.w;
        wr[4 * x] = b4.x; wr[4 * x + 1] = b4.y; wr[4 * x + 2] = b4.z; wr[4 * x + 3] = b4.w;
      }
    }
    arow = SNp[r];            // base row j
    brow = SNp[n + r];        // base row j+1
    if (j >= 1) {
      xhp = XHp[r];
      const float4* pp = (const float4*)(Pp + (long long)r * ntp);
#pragma unroll
      for (int u = 0; u < PQ4; ++u)
        if (4 * u + 3 >= s0p && 4 * u < nt) pq[u] = pp[u];
    }
  }
  // waves 0 / 1: rows j / j+1 (every workgroup needs them for x_j and a_j)
  const int rw = j + wave;
  float vrow = 0.f, wrow = 0.f, pw = 0.f, xw = 0.f, aw = 0.f;
  if (wave < 2 && rw < n) {
    if (lane < NB) {
      vrow = M.V[(long long)rw * NB + lane];
      wrow = M.W[(long long)rw * NB + lane];
    }
    if (j >= 1) {
      if (lane >= s0p && lane < nt) pw = Pp[(long long)rw * ntp + lane];
      xw = XHp[rw];
    }
    aw = SNp[rw];
  }
  // step-1 partials: row-block sums (flat over blocks x kinds) and tile sums
  float rsv[RSL];
  double ts = 0.0;
  const int nbp = nt - s0p;
  if (j >= 1) {
    const float* RSp = M.RS + ps * M.sRS + (long long)s0p * RSW;
    const float* TSp = M.TS + ps * M.sTS;
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const int f = tid + 256 * u;
      rsv[u] = (f < nbp * RSW) ? RSp[f] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < TSL; ++u) {
      const int f = tid + 256 * u;
      if (f < nbp * nbp) {
        const int a = s0p + f / nbp, b = s0p + f % nbp;
        if (a <= b) ts += (double)TSp[(long long)a * nt + b];
      }
    }
  }

  STAMP(2);
  // ---- step 1: scalars of column j-1 (every workgroup, same fixed order)
  float* sRS = &S.rowred[0][0];           // staging: blocks x RSW
  if (wave < 2 && lane < NB) {
    S.vwj[2 * wave][lane] = vrow;
    S.vwj[2 * wave + 1][lane] = wrow;
  }
  if (j >= 1) {
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const int f = tid + 256 * u;
      if (f < nbp * RSW) sRS[f] = rsv[u];
    }
    ts = wave_reduce_sum_d(ts);
    if (lane == 0) S.red[3 * RSW + wave] = ts;
  }
  __syncthreads();
  if (j >= 1) {
    if (tid < RSW) {
      double acc = 0.0;
      if (tid < 2 + cp || (tid >= 2 + NB && tid < 2 + NB + cp))
        for (int bb = 0; bb < nbp; ++bb) acc += (double)sRS[bb * RSW + tid];
      S.red[tid] = acc;
    }
    __syncthreads();
    if (wave == 0) {
      const double sig2 = S.red[0], xa = S.red[1];
      const double xy = S.red[3 * RSW] + S.red[3 * RSW + 1] + S.red[3 * RSW + 2] +
                        S.red[3 * RSW + 3];
      const float* SCp = M.SC + ps * 4;
      const double alpha = SCp[0];
      double beta, tau, s;
      hh_scalars(alpha, sig2, beta, tau, s);
      // s1 = W^T v, s2 = V^T v over rows >= j (v[j] = 1): row j of the panel
      double s1 = 0.0, s2 = 0.0;
      if (lane < cp) {
        s1 = (double)S.vwj[1][lane] + s * S.red[2 + lane];
        s2 = (double)S.vwj[0][lane] + s * S.red[2 + NB + lane];
        S.s12[lane] = (float)s1;
        S.s12[NB + lane] = (float)s2;
      }
      const double s1s2 = wave_reduce_sum_d(s1 * s2);
      if (lane == 0) {
        const double vy = (double)SNp[j] + 2.0 * s * xa + s * s * xy;
        S.scal[0] = beta; S.scal[1] = tau; S.scal[2] = s; S.scal[4] = SCp[1];
        S.scal[3] = -0.5 * tau * tau * (vy - 2.0 * s1s2);
      }
    }
    __syncthreads();
  }
  const double beta_p = S.scal[0], tau_p = S.scal[1], s_p = S.scal[2], alpha2 = S.scal[3];
  STAMP(3);

  // ---- step 2 for rows j and j+1 (waves 0 / 1)
  if (wave < 2 && j >= 1 && rw < n) {
    const float yv = wave_reduce_sum(pw);
    float corr = (lane < cp) ? vrow * S.s12[lane] + wrow * S.s12[NB + lane] : 0.f;
    corr = wave_reduce_sum(corr);
    const float vv = (rw == j) ? 1.f : (float)(s_p * (double)xw);
    const float ww = (float)(tau_p * ((double)aw + s_p * (double)yv - (double)corr) +
                             alpha2 * (double)vv);
    if (lane == cp) {
      S.vwj[2 * wave][lane] = vv;
      S.vwj[2 * wave + 1][lane] = ww;
    }
    if (lead && rw == j && lane == 0) {
      M.V[(long long)rw * NB + cp] = vv;
      M.W[(long long)rw * NB + cp] = ww;
    }
  }
  __syncthreads();
  if (lead && tid == 0 && j >= 1) {
    M.d[j - 1] = (float)S.scal[4];
    M.e[j - 1] = (float)beta_p;
    M.tau[j - 1] = (float)tau_p;
    M.A[(long long)(j - 1) * lda + j] = (float)beta_p;
  }
  float yh = 0.f;
#pragma unroll
  for (int u = 0; u < PQ4; ++u) {
    if (4 * u >= s0p) yh += pq[u].x;
    if (4 * u + 1 >= s0p) yh += pq[u].y;
    if (4 * u + 2 >= s0p) yh += pq[u].z;
    if (4 * u + 3 >= s0p) yh += pq[u].w;
  }

  STAMP(4);
  // ---- step 2 for this thread's row (r >= j+1)
  float vmy = 0.f, wmy = 0.f;
  if (j >= 1 && rok && r >= j + 1) {
    float corr = 0.f;
#pragma unroll
    for (int x = 0; x < NB; ++x)
      if (x < cp) corr += vr[x] * S.s12[x] + wr[x] * S.s12[NB + x];
    vmy = (float)(s_p * (double)xhp);
    wmy = (float)(tau_p * ((double)arow + s_p * (double)yh - (double)corr) + alpha2 * (double)vmy);
#pragma unroll
    for (int x = 0; x < NB; ++x)
      if (x == cp) { vr[x] = vmy; wr[x] = wmy; }
    if (diag && h == 0) {
      M.V[(long long)r * NB + cp] = vmy;
      M.W[(long long)r * NB + cp] = wmy;
      M.A[(long long)(j - 1) * lda + r] = vmy;     // reflector j-1: v[2:] (r >= j+1)
    }
  }

  // ---- finisher: d[n-1] = base(n-1, n-1) - 2 V[n-1] . W[n-1] over cc columns
  if (fin) {
    if (tid == 0) {
      double dd = SNp[j];
      for (int x = 0; x < cc; ++x) dd -= 2.0 * (double)S.vwj[0][x] * (double)S.vwj[1][x];
      M.d[j] = (float)dd;
      M.e[j] = 0.f;
      M.tau[j] = 0.f;
    }
    return;
  }

  // ---- panel start: A_tile -= V W^T + W V^T (rows >= j, upper), in registers
  if (pstart) {
    float* sV = upd;                      // [256][NB+1]
    float* sW = upd + 256 * (NB + 1);
#pragma unroll
    for (int x = 0; x < NB; ++x) {
      sV[tid * (NB + 1) + x] = (rok && r >= j) ? vr[x] : 0.f;
      sW[tid * (NB + 1) + x] = (rok && r >= j) ? wr[x] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int rr = wave * 32 + it * 2 + hw;      // tile row (block I)
      const int gr = I * TB + rr;
      float u0 = 0.f, u1 = 0.f, u2 = 0.f, u3 = 0.f;
      const float* vi = sV + rr * (NB + 1);
      const float* wi = sW + rr * (NB + 1);
      const float* vk = sV + (128 + kk0) * (NB + 1);
      const float* wk = sW + (128 + kk0) * (NB + 1);
#pragma unroll 8
      for (int x = 0; x < NB; ++x) {
        const float a = vi[x], b = wi[x];
        u0 += a * wk[x] + b * vk[x];
        u1 += a * wk[(NB + 1) + x] + b * vk[(NB + 1) + x];
        u2 += a * wk[2 * (NB + 1) + x] + b * vk[2 * (NB + 1) + x];
        u3 += a * wk[3 * (NB + 1) + x] + b * vk[3 * (NB + 1) + x];
      }
      if (gr >= j + 1 && gr < n) {
        float* row = M.A + (long long)gr * lda + K * TB + kk0;
        const int gc = K * TB + kk0;
        if (gc >= gr && gc < n) { q[it].x -= u0; row[0] = q[it].x; }
        if (gc + 1 >= gr && gc + 1 < n) { q[it].y -= u1; row[1] = q[it].y; }
        if (gc + 2 >= gr && gc + 2 < n) { q[it].z -= u2; row[2] = q[it].z; }
        if (gc + 3 >= gr && gc + 3 < n) { q[it].w -= u3; row[3] = q[it].w; }
      }
    }
  }

  STAMP(5);
  // ---- step 3: x_j (rows >= j+1), a_j; d_j and alpha_j by the lead
  float* XHc = M.XH + cs * M.sXH;
  float xmy = 0.f, amy = 0.f;
  if (rok && r >= j + 1) {
    float corr = 0.f, corr1 = 0.f;
#pragma unroll
    for (int x = 0; x < NB; ++x) {
      if (x < cc) {
        corr += vr[x] * S.vwj[1][x] + wr[x] * S.vwj[0][x];
        corr1 += vr[x] * S.vwj[3][x] + wr[x] * S.vwj[2][x];
      }
    }
    xmy = arow - corr;
    amy = pstart ? brow - corr1 : brow;
  }
  const float xh = (rok && r >= j + 2) ? xmy : 0.f;
  if (lead && tid == 0) {
    double dd = SNp[j];
    for (int x = 0; x < cc; ++x) dd -= 2.0 * (double)S.vwj[0][x] * (double)S.vwj[1][x];
    float* SCc = M.SC + cs * 4;
    SCc[1] = (float)dd;
  }
  if (rok && r == j + 1 && diag && h == 0) M.SC[cs * 4] = xmy;   // alpha_j
  if (diag && h == 0 && rok) XHc[r] = xh;
  S.sv[h][lr] = xh;

  // ---- row-block partials (diagonal tiles): |xh|^2, xh.a_j, W^T xh, V^T xh
  //      (new panel columns), transposed through LDS and summed per kind
  if (diag) {
    const int cn = pstart ? 0 : c;     // columns of the current panel
    const int nk = 2 + 2 * NB;
    float* T = upd;                    // [TB][RSW]
    __syncthreads();                   // the panel-start staging in upd is consumed
    if (h == 0) {
      float* row = T + lr * RSW;
      row[0] = xh * xh;
      row[1] = xh * amy;
#pragma unroll
      for (int x = 0; x < NB; ++x) {
        row[2 + x] = (x < cn) ? wr[x] * xh : 0.f;
        row[2 + NB + x] = (x < cn) ? vr[x] * xh : 0.f;
      }
    }
    __syncthreads();
    if (tid < 3 * RSW) {
      const int k = tid % RSW, g = tid / RSW;
      double acc = 0.0;
      if (k < nk)
        for (int rr = g; rr < TB; rr += 3) acc += (double)T[rr * RSW + k];
      S.red[g * RSW + k] = acc;
    }
    __syncthreads();
    float* RSc = M.RS + cs * M.sRS + (long long)I * RSW;
    if (tid < RSW)
      RSc[tid] = (float)(S.red[tid] + S.red[RSW + tid] + S.red[2 * RSW + tid]);
  }
  __syncthreads();

  STAMP(6);
  // ---- snapshot rows j+1, j+2 of the (updated) base for K(j+1)
  float* SNc = M.SN + cs * M.sSN;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int gr = I * TB + wave * 32 + it * 2 + hw;
    const int gc = K * TB + kk0;
    if (gr == j + 1 || gr == j + 2) {
      float* o = SNc + (gr == j + 1 ? 0 : n);
      if (gc >= gr && gc < n) o[gc] = q[it].x;
      if (gc + 1 >= gr && gc + 1 < n) o[gc + 1] = q[it].y;
      if (gc + 2 >= gr && gc + 2 < n) o[gc + 2] = q[it].z;
      if (gc + 3 >= gr && gc + 3 < n) o[gc + 3] = q[it].w;
    }
  }

  STAMP(7);
  // ---- step 4: yh partials over the tile (upper triangle of diagonal tiles)
  float ca[4] = {0.f, 0.f, 0.f, 0.f};
  const float vk0 = S.sv[1][kk0], vk1 = S.sv[1][kk0 + 1], vk2 = S.sv[1][kk0 + 2],
              vk3 = S.sv[1][kk0 + 3];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int rr = wave * 32 + it * 2 + hw;
    float x0 = q[it].x, x1 = q[it].y, x2 = q[it].z, x3 = q[it].w;
    const float vrr = S.sv[0][rr];
    if (diag) {
      x0 = (kk0 >= rr) ? x0 : 0.f;
      x1 = (kk0 + 1 >= rr) ? x1 : 0.f;
      x2 = (kk0 + 2 >= rr) ? x2 : 0.f;
      x3 = (kk0 + 3 >= rr) ? x3 : 0.f;
      S.rowred[rr][cl] = x0 * vk0 + x1 * vk1 + x2 * vk2 + x3 * vk3;
      ca[0] += (kk0 > rr) ? x0 * vrr : 0.f;
      ca[1] += (kk0 + 1 > rr) ? x1 * vrr : 0.f;
      ca[2] += (kk0 + 2 > rr) ? x2 * vrr : 0.f;
      ca[3] += (kk0 + 3 > rr) ? x3 * vrr : 0.f;
    } else {
      S.rowred[rr][cl] = x0 * vk0 + x1 * vk1 + x2 * vk2 + x3 * vk3;
      ca[0] += x0 * vrr; ca[1] += x1 * vrr; ca[2] += x2 * vrr; ca[3] += x3 * vrr;
    }
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) ca[x] += __shfl_xor(ca[x], 32, 64);
  if (hw == 0) {
#pragma unroll
    for (int x = 0; x < 4; ++x) S.colred[wave][kk0 + x] = ca[x];
  }
  __syncthreads();
  float* Pc = M.P + cs * M.sP;
  double tp = 0.0;
  if (tid < TB) {
    float rs = 0.f;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) rs += S.rowred[tid][l];
    const float csum = S.colred[0][tid] + S.colred[1][tid] + S.colred[2][tid] + S.colred[3][tid];
    if (diag) {
      Pc[((long long)I * TB + tid) * ntp + K] = rs + csum;
      tp = (double)S.sv[0][tid] * (double)(rs + csum);
    } else {
      Pc[((long long)I * TB + tid) * ntp + K] = rs;
      Pc[((long long)K * TB + tid) * ntp + I] = csum;
      tp = (double)S.sv[0][tid] * (double)rs + (double)S.sv[1][tid] * (double)csum;
    }
  }
  STAMP(8);
  tp = wave_reduce_sum_d(tp);
  if (lane == 0 && wave < 2) S.red[4 * RSW - 2 + wave] = tp;
  __syncthreads();
  if (tid == 0)
    M.TS[cs * M.sTS + (long long)I * nt + K] = (float)(S.red[4 * RSW - 2] + S.red[4 * RSW - 1]);
  STAMP(9);
}

// ------------------------------------------------------------------ host
struct RPlan {
  RMat* d_mats = nullptr;
  int* d_offs = nullptr;       // per launch j: (nm + 1) cumulative tile offsets
  std::vector<int> n_sorted;   // descending
  int nmax = 0;
  hipGraphExec_t exec = nullptr;
};

inline int h_tri(int m) { return m * (m + 1) / 2; }

int enqueue(const RPlan& P, hipStream_t stream) {
  const int nm = (int)P.n_sorted.size();
  hipLaunchKernelGGL(reduce_prep_kernel, dim3(8, nm), dim3(256), 0, stream, P.d_mats);
  const size_t upd_lds = 2 * 256 * (NB + 1) * sizeof(float);
  const size_t part_lds = TB * RSW * sizeof(float);
  for (int j = 0; j < P.nmax; ++j) {
    int nact = 0, grid = 0;
    for (int i = 0; i < nm; ++i) {
      const int n = P.n_sorted[i];
      if (j > n - 1) break;
      ++nact;
      const int nt = (n + TB - 1) / TB;
      grid += (j <= n - 2) ? h_tri(nt - (j + 1) / TB) : 1;
    }
    const bool pstart = (j % NB == 0 && j > 0);
    hipLaunchKernelGGL(sytrd_col_kernel, dim3(grid), dim3(256), pstart ? upd_lds : part_lds, stream,
                       P.d_mats, P.d_offs + (long long)j * (nm + 1), nact, j);
  }
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, RPlan> g_plans;

}  // namespace

// workspace floats per matrix (V, W and the 2-slot partial rings)
KFAC_API long long kfac_reduce_ws_floats(int n) {
  const long long nt = (n + TB - 1) / TB;
  long long s = 2LL * n * NB;                 // V, W
  s += 2 * nt * TB * ((nt + 3) / 4 * 4) + 32; // P (row-major partials)
  s += 2 * nt * nt;                           // TS
  s += 2 * nt * RSW;                          // RS
  s += 2LL * n;                               // XH
  s += 4LL * n;                               // SN
  s += 8;                                     // SC
  return (s + 63) / 64 * 64 + 64 * 8;
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
    M.d = r.d; M.e = r.e; M.tau = r.tau;
    const long long nt = M.nt, n = r.n;
    float* p = r.ws;
    // 16-byte aligned carving
    auto take = [&](long long fl) { float* o = p; p += (fl + 15) / 16 * 16; return o; };
    M.V = take(n * NB); M.W = take(n * NB);
    M.sP = (nt * TB * ((nt + 3) / 4 * 4) + 15) / 16 * 16; M.P = take(2 * M.sP);
    M.sTS = (nt * nt + 15) / 16 * 16; M.TS = take(2 * M.sTS);
    M.sRS = (nt * RSW + 15) / 16 * 16; M.RS = take(2 * M.sRS);
    M.sXH = (n + 15) / 16 * 16; M.XH = take(2 * M.sXH);
    M.sSN = (2 * n + 15) / 16 * 16; M.SN = take(2 * M.sSN);
    M.SC = take(8);
    mats.push_back(M);
  }
  const std::string key((const char*)mats.data(), sizeof(RMat) * mats.size());
  std::lock_guard<std::mutex> lk(g_mu);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)sytrd_col_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * 256 * (NB + 1) * (int)sizeof(float));
    attr = true;
  }
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    RPlan P;
    for (const RMat& M : mats) P.n_sorted.push_back(M.n);
    P.nmax = P.n_sorted[0];
    if ((*err = (int)hipMalloc(&P.d_mats, sizeof(RMat) * mats.size())) != 0) return nullptr;
    if ((*err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(RMat) * mats.size(),
                               hipMemcpyHostToDevice)) != 0)
      return nullptr;
    const int nm = (int)mats.size();
    std::vector<int> offs((size_t)P.nmax * (nm + 1), 0);
    for (int j = 0; j < P.nmax; ++j) {
      int acc = 0;
      for (int i = 0; i < nm; ++i) {
        offs[(size_t)j * (nm + 1) + i] = acc;
        const int n = P.n_sorted[i];
        if (j <= n - 1) acc += (j <= n - 2) ? h_tri((n + TB - 1) / TB - (j + 1) / TB) : 1;
      }
      offs[(size_t)j * (nm + 1) + nm] = acc;
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

// Tridiagonalise `count` symmetric matrices (any sizes) with one launch per
// column for all of them: A (n x lda, row-major, upper triangle read and
// overwritten by the reflectors), d, e, tau (n floats each), ws
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

// debug: record phase stamps of workgroup 0 of every launch into `buf`
// (nmax x 16 uint64), or stop with nullptr
KFAC_API int kfac_reduce_stamps(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
}

KFAC_API int kfac_reduce_prepare(const KfacReduceRecord* recs, int count) {
  int err = 0;
  return plan_for(recs, count, true, &err) ? 0 : (err ? err : -4);
}
