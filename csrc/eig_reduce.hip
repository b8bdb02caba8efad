// Batched Householder tridiagonalisation for a ragged batch of K-FAC factors
// (reference semantics kfac/layers/utils.py:45-74 -- the
// reduction stage of a symmetric eigensolver, LAPACK sytrd lower ==
// row-major upper here).
//
// The reduction is a chain of n dependent columns, so the latency of one
// column sets the speed.  Every matrix of the inverse update (any sizes, up to
// 16384) advances through ONE launch sequence, two launches per column:
//
//   F(j)  row-parallel, one workgroup per 64 rows of every matrix with j < n:
//         1. the global sums of column j-1 (|xh|^2, xh.a, W^T xh, V^T xh from
//            the row-block partials of S(j-1), xh^T yh from its tile sums),
//            reduced once per workgroup: lane = partial kind, wave = quarter
//            of the blocks, one LDS exchange -- fixed order, deterministic
//         2. Householder scalars of column j-1; w_{j-1} = tau (a + s yh - V s1
//            - W s2) + alpha2 v for the workgroup's rows -> panel column c-1
//         3. x_j = A row j - V W[j]^T - W V[j]^T (UNNORMALISED: its scale needs
//            a global norm only the next F knows; y_j = a_j + s_j A22 xh_j is
//            linear in it), a_j = column j+1 of A22 -> XH, AV
//         No partial sums, no workgroup barrier after a global store.
//   U(j)  at a panel start (every NB = 32 columns): A22 -= V W^T + W V^T on
//         the upper 128 x 128 tiles, exact-f32 MFMA
//   S(j)  tile-parallel: yh = A22 xh over the upper tiles (an off-diagonal
//         tile feeds its row and its column block), per-row partials + one
//         xh.yh sum per tile; and, in extra workgroups of the same launch,
//         the per-128-row-block partial sums F(j+1) needs (|xh|^2, xh.a, the
//         panel's W^T xh and V^T xh)
//
// Round 2 computed those row-block sums at the end of F with a 63-shuffle
// butterfly and a workgroup barrier that drained F's global stores; F took
// ~9.5 us per column (profiles/r3_stamps_*.log).  Moving them into S, where
// they run beside the tiles, leaves F a load -> reduce -> scalar -> row chain.
//
// Once a matrix's trailing part is at most KFAC_REDUCE_TAIL rows (default
// 768), its columns run as ONE launch each (L below: F's row work done
// redundantly by the tile workgroups, the panel replaced by an in-register
// rank-2 update of the tile; model scripts/models/sytrd_tail_model.py), and
// in columns where blocked and tail matrices meet, S and L share a launch.
//
// The recurrence (unnormalised xh, scalars one launch late) is modelled
// exactly in scripts/models/sytrd_fused_model.py (fp64, 1e-15).  Storage:
// row-major, UPPER triangle maintained; output d, e, tau and reflector j in
// row j (beta at j+1, v[2:] after): the layout the compact-WY back-
// transformation (csrc/eig_backtransform.hip) reads.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int TB = 128;        // symv / update tile
constexpr int HT = 64;         // rows per symv workgroup (half a tile)
constexpr int FB = 64;         // rows per F workgroup
constexpr int NB = 32;         // panel width
constexpr int NK = 64;         // partial kinds per row block (one per lane)
constexpr int K_W = 2, K_V = 2 + (NB - 1);   // kinds: |xh|^2, xh.a, W^T xh, V^T xh
static_assert(K_V + NB - 1 == NK, "partial kinds must fill one wave");
constexpr int MAXM = 255;      // matrices per batch
constexpr int NMAX = 16384;    // largest factor (F's unrolled loads: RB <= 128 blocks)

struct RMat {
  float* A; long long lda; int n; int nt; int nf; int ld;   // ld = nt * TB
  float* d; float* e; float* tau;
  float* V; float* W;                     // NB columns of ld floats (column-major)
  float* P; float* TS; float* DS; float* XH; float* AV; float* SC;   // P: nt columns of ld
  long long sP, sTS, sDS, sX;             // slot strides (floats); 2 slots each
};

__host__ __device__ inline long long kfac_a16(long long x) { return (x + 15) / 16 * 16; }

// Workspace layout of one matrix (floats): V, W and the 2-slot partial rings
struct WsLayout {
  long long V, W, P, TS, DS, XH, AV, SC, total, sP, sTS, sDS, sX;
  int nt, ld;
};

__host__ __device__ inline WsLayout ws_layout(long long n) {
  WsLayout L;
  L.nt = (int)((n + TB - 1) / TB);
  L.ld = L.nt * TB;
  const long long nt = L.nt;
  L.sP = kfac_a16(2 * nt * L.ld);
  L.sTS = kfac_a16(nt * (nt + 1) > 4 ? nt * (nt + 1) : 4);
  L.sDS = kfac_a16(nt * NK);
  L.sX = kfac_a16(L.ld);
  long long o = 0;
  L.V = o; o += kfac_a16((long long)NB * L.ld);
  L.W = o; o += kfac_a16((long long)NB * L.ld);
  L.P = o; o += 2 * L.sP;
  L.TS = o; o += 2 * L.sTS + 1024;         // float4 loads past the triangle stay inside
  L.DS = o; o += 2 * L.sDS;
  L.XH = o; o += 2 * L.sX;
  L.AV = o; o += 2 * L.sX;
  L.SC = o; o += kfac_a16(8);
  L.total = (o + 63) / 64 * 64;
  return L;
}


// debug: per-column stamps (s_memrealtime, 100 MHz) of the first F and S
// workgroups into a caller buffer (kfac_reduce_stamps)
__device__ unsigned long long* g_stamps = nullptr;
#define STAMP(k)                                                                            \
  do {                                                                                      \
    if (stamps && threadIdx.x == 0) stamps[(long long)j * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
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

// workgroup -> (matrix, first workgroup of that matrix) from the launch's
// ascending offsets: lane i tests offset i (one load + ballot, no LDS); a
// launch whose active matrices all have the same workgroup count passes
// -count instead (one dependent table read less per launch: the batch of
// equal-size largest factors is the inverse update's critical chain)
__device__ __forceinline__ void find_mat_b(const int* __restrict__ offs, int nact, int b,
                                           int& mi, int& base) {
  const int lane = threadIdx.x & 63;
  if (nact < 0) {      // uniform launch: every active matrix has -nact workgroups (no table read)
    mi = b / -nact;
    base = mi * -nact;
    return;
  }
  if (nact <= 64) {     // one load; the base offset comes from lane mi (no second round trip)
    const int o = gld_if(gptr(offs), lane, lane < nact, 0x7fffffff);
    mi = __builtin_amdgcn_readfirstlane(__popcll(__ballot(o <= b)) - 1);
    base = __builtin_amdgcn_readlane(o, mi);
    return;
  }
  int cnt = 0;
  for (int c0 = 0; c0 < nact; c0 += 64) {
    const int i = c0 + lane;
    const int o = gld_if(gptr(offs), i, i < nact, 0x7fffffff);
    cnt += __popcll(__ballot(o <= b));
  }
  mi = cnt - 1;
  base = offs[mi];
}
__device__ __forceinline__ void find_mat(const int* __restrict__ offs, int nact, int& mi,
                                         int& base) {
  find_mat_b(offs, nact, blockIdx.x, mi, base);
}

// ------------------------------------------------------------------- F
// One workgroup per FB = 64 rows: lane = row, wave q = a quarter of the
// per-row work (panel columns 8q .. 8q+7, yh partial columns s0p+q+4i), so a
// workgroup moves ~25 KB instead of ~100 KB (the round-2 kernel's 256 rows x
// (32+32 panel floats + one partial per tile) came in at ~25 GB/s per
// workgroup: profiles/r3_r2kernel_stamps_*.log).  RB >= the active 128-row
// blocks of S(j-1) (nt - j / TB) of every matrix of the launch: fixes the
// number of partial loads per thread, all issued up front.
template <int RB>
__device__ __forceinline__ void fin_body(const RMat& M, int base, int j) {
  constexpr int DQ = RB / 4;                            // DS loads per thread
  constexpr int TQ = (RB * (RB + 1) + 1023) / 1024;     // float4 TS loads per thread
  constexpr int PK = RB / 4;                            // P partial pairs per thread
  constexpr int XQ = NB / 4;                            // panel columns per quarter
  __shared__ double sdk[4][NK];
  __shared__ double stt[4];
  __shared__ float sq[4][4][FB];                        // per quarter: yh, c3, c3', c2 of each row
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  unsigned long long* const stamps = blockIdx.x == 0 ? g_stamps : nullptr;
  const int n = M.n, nt = M.nt;
  const long long lda = M.lda, ld = M.ld;
  // first row block: the first row S(j) reads (its tiles start at a 128-row
  // boundary <= j+1; rows below j+1 get xh = a = 0), or row j's block
  const int fb0 = min(((j + 1) / TB) * (TB / FB), j / FB);
  const int r = (fb0 + (blockIdx.x - base)) * FB + lane;   // this thread's row
  const bool lead = (blockIdx.x == base && q == 0);
  const bool last = (j == n - 1);
  const bool j1 = (j >= 1), has1 = (j + 1 < n);
  const int c = j % NB;
  const int cp = j1 ? (c == 0 ? NB - 1 : c - 1) : 0;    // panel column of j-1 (cc = cp + 1)
  const bool pstart = (c == 0 && j > 0);
  const int cs = j & 1, ps = cs ^ 1;
  const int s0p = j / TB;                               // first block of S(j-1)
  const int ntri = (nt - s0p) * (nt - s0p + 1);         // tile halves of S(j-1)
  const AS1 float* DSp = gptr(M.DS) + ps * M.sDS;
  const AS1 float* TSp = gptr(M.TS) + ps * M.sTS;
  const AS1 float* Pp = gptr(M.P) + ps * M.sP;
  const AS1 float* XHp = gptr(M.XH) + ps * M.sX;
  AS1 float* const gA = gptr(M.A);
  AS1 float* const gV = gptr(M.V);
  AS1 float* const gW = gptr(M.W);
  AS1 float* const gSC = gptr(M.SC);
  STAMP(1);

  // ---- every load up front (one memory round trip).  Indices are clamped
  // into the buffers and out-of-range terms dropped at use: per-load
  // predicates would cost one SGPR mask each.  At j = 0 the partial sums
  // read stale slot data; they feed only the j >= 1 branch (no j1 test in
  // the loads: a uniform test there became a branch, and a branch in the
  // load section makes the compiler wait for every load before it).
  // 32-bit element offsets from uniform bases (one offset VGPR per load, not
  // a 64-bit address pair: at ~60 loads that sets the register budget)
  const unsigned uld = (unsigned)ld, ulda = (unsigned)lda;
  float dk[DQ];                                         // kind `lane`, blocks s0p + q + 4 i
#pragma unroll
  for (int i = 0; i < DQ; ++i) dk[i] = DSp[(unsigned)min(s0p + q + 4 * i, nt - 1) * NK + lane];
  fx4 tq[TQ];
  const fx4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < TQ; ++u)
    tq[u] = gld_if32((const AS1 fx4*)TSp, (unsigned)(tid + 256 * u), 4 * (tid + 256 * u) < ntri, z4);
  // rows j, j+1: yh partials, lane = P column 2T + h - 2 s0p (several per lane);
  // column 2T+1 of a row of block B exists only for T <= B (see S)
  const int bj = j / TB, bj1 = (j + 1) / TB;
  // (bitwise & / |: a short-circuit && would branch, and a branch in the load
  // section makes the compiler wait for every load issued before it)
  auto pcol_ok = [&](int col, int B) -> bool {
    return (col >= 2 * s0p) & (col < 2 * nt) & (((col & 1) == 0) | ((col >> 1) <= B));
  };
  float pj = 0.f, pj1 = 0.f;
#pragma unroll
  for (int h = 0; h < (2 * RB + 63) / 64; ++h) {
    const int col = 2 * s0p + lane + 64 * h;           // the 2 (nt - s0p) <= 2 RB live columns
    pj += gld_if32(Pp, (unsigned)col * uld + j, pcol_ok(col, bj), 0.f);
    pj1 += gld_if32(Pp, (unsigned)col * uld + j + 1, has1 & pcol_ok(col, bj1), 0.f);
  }
  const float xhj1 = gld_if32(XHp, j + 1, has1, 0.f);
  const float alpha = gSC[ps * 4];
  const float dprev = gSC[ps * 4 + 1];
  float vj = gld_if32(gV, (unsigned)lane * uld + j, lane < NB, 0.f);   // panel row j (lane = column)
  float wj = gld_if32(gW, (unsigned)lane * uld + j, lane < NB, 0.f);
  float vj1 = gld_if32(gV, (unsigned)lane * uld + j + 1, (lane < NB) & has1, 0.f);
  float wj1 = gld_if32(gW, (unsigned)lane * uld + j + 1, (lane < NB) & has1, 0.f);
  const float ajj = gA[(unsigned)j * ulda + j];
  const float ajj1 = gld_if32(gA, (unsigned)j * ulda + j + 1, has1, 0.f);
  const bool rok = (r < n) & (r >= j + 1);              // rows that get w_{j-1} and x_j
  const int rc = min(r, n - 1);
  float vr[XQ], wr[XQ];                                 // this quarter's panel columns of row r
#pragma unroll
  for (int i = 0; i < XQ; ++i) {
    vr[i] = gV[(unsigned)(q * XQ + i) * uld + rc];
    wr[i] = gW[(unsigned)(q * XQ + i) * uld + rc];
  }
  const float arow = gA[(unsigned)j * ulda + rc];                     // base row j
  const float brow = gld_if32(gA, (unsigned)(j + 1) * ulda + rc, has1 & rok, 0.f);
  const float xhp = XHp[(unsigned)rc];
  float pk[2 * PK];                                      // yh partials, P columns 2T, 2T+1, T = s0p + q + 4 i
#pragma unroll
  for (int i = 0; i < PK; ++i) {
    const unsigned t2 = 2 * min(s0p + q + 4 * i, nt - 1);
    pk[2 * i] = Pp[t2 * uld + rc];
    pk[2 * i + 1] = Pp[(t2 + 1) * uld + rc];
  }
  // every load above is issued before anything consumes one (the scheduler
  // otherwise interleaves early sums and waits on a half-issued batch)
  __builtin_amdgcn_sched_barrier(0);

  // ---- global sums of column j-1 (wave = quarter of the blocks, lane = kind)
  //      and this quarter's share of each row's yh and old-panel corrections
  {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < DQ; ++i) acc += (s0p + q + 4 * i < nt) ? (double)dk[i] : 0.0;
    sdk[q][lane] = acc;
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < TQ; ++u) {
      const int f = 4 * (tid + 256 * u);
      t += (f < ntri) ? (double)tq[u].x : 0.0;
      t += (f + 1 < ntri) ? (double)tq[u].y : 0.0;
      t += (f + 2 < ntri) ? (double)tq[u].z : 0.0;
      t += (f + 3 < ntri) ? (double)tq[u].w : 0.0;
    }
    t = wave_sum_d(t);
    if (lane == 0) stt[q] = t;
    float yq = 0.f;
    const int br = rc / TB;
#pragma unroll
    for (int i = 0; i < PK; ++i) {
      const int T = s0p + q + 4 * i;
      yq += (T < nt) ? pk[2 * i] : 0.f;
      yq += ((T < nt) & (T <= br)) ? pk[2 * i + 1] : 0.f;
    }
    float c3 = 0.f, c3p = 0.f;                           // old columns x < cp
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int x = q * XQ + i;
      const float Wj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj), x));
      const float Vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vj), x));
      const float Wj1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj1), x));
      const float Vj1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vj1), x));
      if (x < cp) {
        c3 += vr[i] * Wj + wr[i] * Vj;
        c3p += vr[i] * Wj1 + wr[i] * Vj1;
      }
    }
    sq[q][0][lane] = yq;
    sq[q][1][lane] = c3;
    sq[q][2][lane] = c3p;
  }
  kfac_lds_barrier();
  STAMP(2);
  const double sig2 = ((sdk[0][0] + sdk[1][0]) + (sdk[2][0] + sdk[3][0]));
  const double xa = ((sdk[0][1] + sdk[1][1]) + (sdk[2][1] + sdk[3][1]));
  const int kw = K_W + min(lane, NB - 2), kv = K_V + min(lane, NB - 2);
  const double pW = ((sdk[0][kw] + sdk[1][kw]) + (sdk[2][kw] + sdk[3][kw]));
  const double pV = ((sdk[0][kv] + sdk[1][kv]) + (sdk[2][kv] + sdk[3][kv]));
  const double xy = ((stt[0] + stt[1]) + (stt[2] + stt[3]));

  // ---- step 1 (every wave, identically): scalars of column j-1; rows j, j+1
  double tau_p = 0.0, s_p = 0.0, alpha2 = 0.0;
  float s1f = 0.f, s2f = 0.f;
  if (j1) {
    double beta_p;
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
        gV[cp * ld + j] = 1.f;
        gW[cp * ld + j] = ww;
      }
      if (lane == 0) {
        M.d[j - 1] = dprev;
        M.e[j - 1] = (float)beta_p;
        M.tau[j - 1] = (float)tau_p;
        gA[(long long)(j - 1) * lda + j] = (float)beta_p;
      }
    }
  }
  {   // d_j = A(j, j) - 2 V[j] . W[j] over the panel columns 0 .. cp
    const double dd = wave_sum_d(j1 && lane <= cp ? (double)vj * (double)wj : 0.0);
    if (lead && lane == 0) {
      const float dj = (float)((double)ajj - 2.0 * dd);
      if (last) {
        M.d[j] = dj;
        M.e[j] = 0.f;
        M.tau[j] = 0.f;
      } else {
        gSC[cs * 4 + 1] = dj;
      }
    }
  }
  // this quarter's share of the step-2 correction V s1 + W s2 (columns < cp)
  {
    float c2 = 0.f;
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int x = q * XQ + i;
      const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s1f), x));
      const float a2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s2f), x));
      if (x < cp) c2 += vr[i] * a1 + wr[i] * a2;
    }
    sq[q][3][lane] = c2;
  }
  kfac_lds_barrier();
  STAMP(3);
  if (q != 0) return;

  // ---- wave 0, this thread's row: step 2 (w_{j-1}, v_{j-1}), step 3 (x_j, a_j)
  const float yh = (sq[0][0][lane] + sq[1][0][lane]) + (sq[2][0][lane] + sq[3][0][lane]);
  const float c2 = (sq[0][3][lane] + sq[1][3][lane]) + (sq[2][3][lane] + sq[3][3][lane]);
  const float c3 = (sq[0][1][lane] + sq[1][1][lane]) + (sq[2][1][lane] + sq[3][1][lane]);
  const float c3p = (sq[0][2][lane] + sq[1][2][lane]) + (sq[2][2][lane] + sq[3][2][lane]);
  float vmy = 0.f, wmy = 0.f;
  if (j1 && rok) {
    vmy = (float)(s_p * (double)xhp);
    wmy = (float)(tau_p * ((double)arow + s_p * (double)yh - (double)c2) + alpha2 * (double)vmy);
    gV[cp * ld + r] = vmy;
    gW[cp * ld + r] = wmy;
    gA[(long long)(j - 1) * lda + r] = vmy;      // reflector j-1: v[2:] (r >= j+1)
  }
  if (last) return;     // uniform: d/e/tau of the last two columns are written
  float xmy = 0.f, amy = 0.f;
  if (rok) {
    // column cp (new): V[j][cp] = 1, W[j][cp] = ww; row j+1: vv1, ww1
    const float Wj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj), cp));
    const float Vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vj), cp));
    const float Wj1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj1), cp));
    const float Vj1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vj1), cp));
    const float t3 = j1 ? vmy * Wj + wmy * Vj : 0.f;
    const float t3p = j1 ? vmy * Wj1 + wmy * Vj1 : 0.f;
    xmy = arow - (c3 + t3);
    amy = pstart ? brow - (c3p + t3p) : brow;   // a_j = row j+1 of the NEW panel's base
  }
  if (r == j + 1 && r < n) gSC[cs * 4] = xmy;      // alpha_j
  if (r < n) {
    gptr(M.XH)[cs * M.sX + r] = (rok && r >= j + 2) ? xmy : 0.f;
    gptr(M.AV)[cs * M.sX + r] = amy;
  }
  STAMP(4);
}

template <int RB>
__global__ __launch_bounds__(256) void red_fin_kernel(const RMat* __restrict__ mats,
                                                      const int* __restrict__ offs, int nact,
                                                      int j) {
  unsigned long long* const stamps = blockIdx.x == 0 ? g_stamps : nullptr;
  STAMP(0);
  int mi, base;
  find_mat(offs, nact, mi, base);
  const RMat M = mats[mi];
  fin_body<RB>(M, base, j);
}

// ------------------------------------------------------------------- U
// A[I][K] -= L_I R_K^T with L = [V | W], R = [W | V] (rows >= q+1, upper):
// the panel's rank-2NB update, 4 waves of 64 x 64.  X6 (default): the fp32
// operands split into bf16 hi / mid / lo planes as the fragments are read from
// LDS, six v_mfma_f32_32x32x16_bf16 products per term (every term above 2^-24
// relative, the precision scheme of csrc/precond_gemm.hip's bf16x6): fp32-level
// error at 2.7x fewer MFMA cycles than the exact-f32 32x32x2 MFMA path
// (KFAC_REDUCE_UPD=f32), which held each update workgroup ~4 us.
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f32_to_bf16_bits(x);
  const float r = x - bf16_bits_to_f32(h);
  m = f32_to_bf16_bits(r);
  l = f32_to_bf16_bits(r - bf16_bits_to_f32(m));
}
// 8 consecutive fp32 of an LDS row -> the three bf16x8 planes of one fragment
__device__ __forceinline__ void frag3(const float* src, bf16x8_t& h8, bf16x8_t& m8, bf16x8_t& l8) {
  typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
  u16x8 h, m, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    uint16_t a, b, c;
    split3(src[e], a, b, c);
    h[e] = a; m[e] = b; l[e] = c;
  }
  h8 = __builtin_bit_cast(bf16x8_t, h);
  m8 = __builtin_bit_cast(bf16x8_t, m);
  l8 = __builtin_bit_cast(bf16x8_t, l);
}

template <bool X6>
__device__ __forceinline__ void upd_body(const RMat& M, int base, int q) {
  __shared__ float sL[TB][2 * NB + 1];
  __shared__ float sR[TB][2 * NB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = M.n, nt = M.nt;
  const int s0 = (q + 1) / TB;
  int I, K;
  tri_index(blockIdx.x - base, nt - s0, I, K);
  I += s0; K += s0;
  const AS1 float* gV = gptr(M.V);
  const AS1 float* gW = gptr(M.W);
  AS1 float* const A = gptr(M.A);
  const unsigned uld = (unsigned)M.ld, ulda = (unsigned)M.lda;
  const int wr = wave >> 1, wc = wave & 1;          // 2 x 2 waves of 64 x 64
  const int l31 = lane & 31, lh = lane >> 5;
  // the panel rows of blocks I and K in one memory round trip (32-bit
  // offsets, clamped, branch-free), then staged in LDS (loading each chunk
  // right before its LDS store made the compiler wait 16 times)
  float pv[4][TB * NB / 256];
#pragma unroll
  for (int u = 0; u < TB * NB / 256; ++u) {
    const int e = u * 256 + tid;
    const int x = e / TB, rr = e - x * TB;            // rows fastest: coalesced columns
    const int ri = min(I * TB + rr, n - 1), rk = min(K * TB + rr, n - 1);
    pv[0][u] = gV[(unsigned)x * uld + ri];
    pv[1][u] = gW[(unsigned)x * uld + ri];
    pv[2][u] = gV[(unsigned)x * uld + rk];
    pv[3][u] = gW[(unsigned)x * uld + rk];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < TB * NB / 256; ++u) {
    const int e = u * 256 + tid;
    const int x = e / TB, rr = e - x * TB;
    const bool oi = I * TB + rr < n, ok = K * TB + rr < n;
    sL[rr][x] = oi ? pv[0][u] : 0.f; sL[rr][NB + x] = oi ? pv[1][u] : 0.f;
    sR[rr][x] = ok ? pv[3][u] : 0.f; sR[rr][NB + x] = ok ? pv[2][u] : 0.f;
  }
  __syncthreads();
  // the old tile values, issued now: they land under the MFMA loop
  float old[2][2][16];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = min(I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh, n - 1);
        const int gc = min(K * TB + wc * 64 + b * 32 + l31, n - 1);
        old[a][b][x] = A[(unsigned)gr * ulda + gc];
      }
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[a][b][x] = 0.f;
  if constexpr (X6) {
#pragma unroll
    for (int kc = 0; kc < 2 * NB / 16; ++kc) {      // k = 16 kc + 8 lh + (0..7)
      const int k0 = 16 * kc + 8 * lh;
      bf16x8_t ap[3][2], bp[3][2];
#pragma unroll
      for (int a = 0; a < 2; ++a) frag3(&sL[wr * 64 + a * 32 + l31][k0], ap[0][a], ap[1][a], ap[2][a]);
#pragma unroll
      for (int b = 0; b < 2; ++b) frag3(&sR[wc * 64 + b * 32 + l31][k0], bp[0][b], bp[1][b], bp[2][b]);
      // smallest terms first: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
      constexpr int TA[6] = {2, 0, 1, 1, 0, 0}, TB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[TA[t]][a], bp[TB[t]][b],
                                                                acc[a][b], 0, 0, 0);
    }
  } else {
#pragma unroll 4
    for (int kk = 0; kk < NB; ++kk) {               // k = 2 kk + lh over 2 NB
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
  }
  // C/D map of 32x32: row = (x&3) + 8 (x>>2) + 4 lh, col = lane & 31
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const int gr = I * TB + wr * 64 + a * 32 + (x & 3) + 8 * (x >> 2) + 4 * lh;
        const int gc = K * TB + wc * 64 + b * 32 + l31;
        if ((gr >= q + 1) & (gr < n) & (gc >= gr) & (gc < n))
          A[(unsigned)gr * ulda + gc] = old[a][b][x] - acc[a][b][x];
      }
}

template <bool X6>
__global__ __launch_bounds__(256) void red_upd_kernel(const RMat* __restrict__ mats,
                                                      const int* __restrict__ offs, int nact,
                                                      int q) {
  int mi, base;
  find_mat(offs, nact, mi, base);
  const RMat M = mats[mi];
  upd_body<X6>(M, base, q);
}

// ------------------------------------------------------------------- S
// One half tile (I, K, hr): rows rb .. rb+63 (rb = I TB + 64 hr) x columns
// K TB .. K TB + 127 of A22, times xh.  Thread (wave w, lane = 16 rg + cg)
// owns rows 4 R .. 4 R + 3 (R = 4 w + rg) x columns 8 cg .. 8 cg + 7: eight
// 16-byte loads, 32 FMAs for its 4 row partials and 32 for its 8 column
// partials; rows are summed over the 16 lanes of a DPP row, columns over the
// 4 row groups of a wave (permlane swaps) and the 4 waves (one LDS pass).
// A and xh are zero past n up to nt TB (the buffers are padded), so no load
// is masked.  P columns: 2T + h, T = the other tile index (see F):
// off-diagonal: row sums -> 2K, column sums of half hr -> 2I + hr; diagonal:
// half hr -> 2I + hr for all 128 rows of block I (column sums, plus the row
// sums of its own 64 rows).  The tile's xh.yh -> TS (triangle order).
// half tiles per S workgroup (1 or 2).  2 (64 KB per workgroup) measured
// slower: the first workgroup's loads took 1.6 vs 0.74 us at the tail (a
// workgroup pulls ~40 GB/s), 4608 x 3 75.9 vs 74.7 ms
// (profiles/r3_symv_snh2_stamps_4608x3.log)
constexpr int SNH = 1;
struct SymvShared {
  float cred[SNH][4][TB];   // column partials per half and wave
  float rsum[SNH][HT];      // row sums (diagonal tiles)
  double tred[SNH][4];
};

__device__ __forceinline__ float row16_sum(float v) {   // over the 16 lanes of a DPP row
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}

// NH = SNH consecutive half tiles hr0 .. hr0 + NH - 1 of tile (I, K); `half0`
// = the first one's index in triangle order (its TS slot)
template <bool DIAG, int NH>
__device__ __forceinline__ void symv_halves(const RMat& M, int I, int K, int hr0, int cs,
                                            int half0, SymvShared& sh, int j,
                                            unsigned long long* stamps) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rg = lane >> 4, cg = lane & 15;
  const int R = wave * 4 + rg;                          // row group of 4 rows
  const unsigned ulda = (unsigned)M.lda;
  const AS1 float* gA = gptr(M.A);
  const AS1 float* XH = gptr(M.XH) + cs * M.sX;
  // ---- loads, one round trip
  fx4 a[NH][4][2], xr[NH];
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const int rb = I * TB + (hr0 + u) * HT;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        a[u][rr][h] =
            *(const AS1 fx4*)(gA + (unsigned)(rb + 4 * R + rr) * ulda + K * TB + 8 * cg + 4 * h);
    xr[u] = *(const AS1 fx4*)(XH + (unsigned)(rb + 4 * R));
  }
  const fx4 xc0 = *(const AS1 fx4*)(XH + (unsigned)(K * TB + 8 * cg));
  const fx4 xc1 = *(const AS1 fx4*)(XH + (unsigned)(K * TB + 8 * cg + 4));
  const float xcol = XH[(unsigned)(K * TB + (tid & (TB - 1)))];   // column `tid`
  if (stamps && blockIdx.x == 0 && tid == 0)
    stamps[(long long)j * 16 + 14] = __builtin_amdgcn_s_memrealtime();
  const float xcv[8] = {xc0.x, xc0.y, xc0.z, xc0.w, xc1.x, xc1.y, xc1.z, xc1.w};
  AS1 float* const Pc = gptr(M.P) + cs * M.sP;
  const unsigned uld = (unsigned)M.ld;
  double tp[NH];
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const int hr = hr0 + u;
    const float xrv[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
    float rp[4], cp[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) cp[c] = 0.f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const float av[8] = {a[u][rr][0].x, a[u][rr][0].y, a[u][rr][0].z, a[u][rr][0].w,
                           a[u][rr][1].x, a[u][rr][1].y, a[u][rr][1].z, a[u][rr][1].w};
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (DIAG) {      // upper triangle: row sums take col >= row, column sums col > row
          const int lr = hr * HT + 4 * R + rr, lc = 8 * cg + c;
          acc += (lc >= lr) ? av[c] * xcv[c] : 0.f;
          cp[c] += (lc > lr) ? av[c] * xrv[rr] : 0.f;
        } else {
          acc += av[c] * xcv[c];
          cp[c] += av[c] * xrv[rr];
        }
      }
      rp[rr] = row16_sum(acc);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) cp[c] = swap_sum32(swap_sum16(cp[c]));
    if (rg == 0) {
#pragma unroll
      for (int c = 0; c < 8; ++c) sh.cred[u][wave][8 * cg + c] = cp[c];
    }
    // this lane's row (cg < 4): row 4 R + cg of the half
    const float myrow = cg == 0 ? rp[0] : (cg == 1 ? rp[1] : (cg == 2 ? rp[2] : rp[3]));
    const float myx = cg == 0 ? xrv[0] : (cg == 1 ? xrv[1] : (cg == 2 ? xrv[2] : xrv[3]));
    tp[u] = 0.0;
    if (DIAG) {
      if (cg < 4) sh.rsum[u][4 * R + cg] = myrow;
    } else if (cg < 4) {
      Pc[(unsigned)(2 * K) * uld + I * TB + hr * HT + 4 * R + cg] = myrow;
      tp[u] = (double)myx * (double)myrow;
    }
  }
  if (stamps && blockIdx.x == 0 && tid == 0)
    stamps[(long long)j * 16 + 15] = __builtin_amdgcn_s_memrealtime();
  kfac_lds_barrier();
  if (tid < TB) {
#pragma unroll
    for (int u = 0; u < NH; ++u) {
      const int hr = hr0 + u;
      float v = (sh.cred[u][0][tid] + sh.cred[u][1][tid]) + (sh.cred[u][2][tid] + sh.cred[u][3][tid]);
      if (DIAG) {
        const int rl = tid - hr * HT;
        if (rl >= 0 && rl < HT) v += sh.rsum[u][rl];
      }
      Pc[(unsigned)(2 * I + hr) * uld + K * TB + tid] = v;
      tp[u] += (double)xcol * (double)v;
    }
  }
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const double t = wave_sum_d(tp[u]);
    if (lane == 0) sh.tred[u][wave] = t;
  }
  kfac_lds_barrier();
  if (tid < NH)
    gptr(M.TS)[cs * M.sTS + half0 + tid] =
        (float)((sh.tred[tid][0] + sh.tred[tid][1]) + (sh.tred[tid][2] + sh.tred[tid][3]));
  if (stamps && blockIdx.x == 0 && tid == 0)
    stamps[(long long)j * 16 + 11] = __builtin_amdgcn_s_memrealtime();
}

// Workgroups 0 .. nh / SNH - 1 of a matrix (nh half tiles): SNH half tiles
// each (symv_halves).  Workgroups nh / SNH .. + nb - 1: row block b = s0 +
// (local - nh / SNH), the NK
// partial kinds of its 128 rows into DS (wave = 16 kinds, lane = row, fixed
// order).
__device__ __forceinline__ void symv_body(const RMat& M, int base, int j) {
  __shared__ SymvShared sred;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long* const stamps = g_stamps;
  const int n = M.n, nt = M.nt;
  const long long ld = M.ld;
  const int s0 = (j + 1) / TB;
  const int ntri = (nt - s0) * (nt - s0 + 1) / SNH;    // tile workgroups
  const int local = blockIdx.x - base;
  const int cs = j & 1;
  if (local >= ntri) {
    // ---- row-block partial kinds: 0 |xh|^2, 1 xh.a, K_W+x W[:,x].xh, K_V+x V[:,x].xh
    if (stamps && blockIdx.x == base + ntri && tid == 0)
      stamps[(long long)j * 16 + 12] = __builtin_amdgcn_s_memrealtime();
    const int b = s0 + (local - ntri);
    const int cn = j % NB;                      // finished columns of the current panel
    const AS1 float* XH = gptr(M.XH) + cs * M.sX;
    const AS1 float* AV = gptr(M.AV) + cs * M.sX;
    // wave w: kinds 16 w .. 16 w + 15; lane = row, two passes of 64 rows
    float x2[2], a2[2], m[2][16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = b * TB + 64 * h + lane;
      const bool ok = rr < n;
      x2[h] = gld_if(XH, rr, ok, 0.f);
      a2[h] = gld_if(AV, rr, ok, 0.f);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = 16 * wave + i;
        const bool isw = k >= K_W && k < K_W + cn, isv = k >= K_V && k < K_V + cn;
        const AS1 float* src = isw ? gptr(M.W) : gptr(M.V);
        const int col = isw ? k - K_W : (isv ? k - K_V : 0);
        m[h][i] = gld_if(src, col * ld + rr, ok && (isw || isv), 0.f);
      }
    }
    float val[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = 16 * wave + i;
      float acc = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float v = k == 0 ? x2[h] : (k == 1 ? a2[h] : m[h][i]);
        acc += v * x2[h];
      }
      val[i] = acc;
    }
    const float tot = kfac_butterfly16(val);      // lanes (lane & 15) == i: kind 16 wave + i
    if (lane < 16) gptr(M.DS)[cs * M.sDS + (long long)b * NK + 16 * wave + lane] = tot;
    if (stamps && blockIdx.x == base + ntri && tid == 0)
      stamps[(long long)j * 16 + 13] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  if (stamps && blockIdx.x == 0 && tid == 0)
    stamps[(long long)j * 16 + 10] = __builtin_amdgcn_s_memrealtime();
  const int half0 = local * SNH;
  int I, K;
  tri_index(half0 >> 1, nt - s0, I, K);
  I += s0; K += s0;
  if (I == K)
    symv_halves<true, SNH>(M, I, K, half0 & 1, cs, half0, sred, j, stamps);
  else
    symv_halves<false, SNH>(M, I, K, half0 & 1, cs, half0, sred, j, stamps);
}

__global__ __launch_bounds__(256) void red_symv_kernel(const RMat* __restrict__ mats,
                                                       const int* __restrict__ offs, int nact,
                                                       int j) {
  int mi, base;
  find_mat(offs, nact, mi, base);
  const RMat M = mats[mi];
  symv_body(M, base, j);
}

// ------------------------------------------------------------------- L
// The single-launch tail (model: scripts/models/sytrd_tail_model.py).  Once a
// matrix's trailing part is small (n - j0 <= the tail size, j0 a panel start
// whose U flushed the panel), column k > j0 is ONE launch: F's row work moves
// into the tile workgroups (each finishes column k-1 redundantly for the 192
// rows its half tile touches) and the panel goes away -- the launch applies
// column k-1's rank-2 update to its tile in registers, stores it (rows >= k+2:
// row k+1 is read by every workgroup of the launch, its update lives in AV),
// then runs the symv of column k on the updated tile.  Per column that is one
// dependent launch instead of two and no V / W panel; the price is a
// read-modify-write of the trailing upper triangle, which is L2 / MALL
// resident at these sizes.
//
// Entering L(k) (slot ps = what S(k-1) / L(k-1) left): storage rows >= k+1 =
// A^(k-1); AV = row k of A^(k-1); XH = xh_{k-1}; P / TS / DS its partial sums;
// SC = alpha_{k-1}, d_{k-1}.  Row slots: 0..127 the K block's rows (the
// tile's columns), 128..191 the I half's rows (off-diagonal tiles only).
// The diagonal half 0 of block b owns block b's outputs (XH, AV, DS, the
// reflector); workgroup 0 the scalars.  k == n-1: one workgroup, scalars only.
constexpr int TSLOT = 192;

__device__ __forceinline__ void tail_vw(double tau, double s, double alpha2, bool pivot, float xh,
                                        float a, float yh, float& v, float& w) {
  v = pivot ? 1.f : (float)(s * (double)xh);
  w = (float)(tau * ((double)a + s * (double)yh) + alpha2 * (double)v);
}

// the half tile (I, K, hr) of L: column k-1's rank-2 update applied to the
// loaded values (row k+1 taken from a_k), rows >= k+2 stored, then the symv
// of column k on the updated values (as symv_halves).  Thread: rows
// 4 R .. 4 R + 3 of the half x columns 8 cg .. 8 cg + 7.  Every operand comes
// from LDS as 16-byte reads issued together; the diagonal masks are selects.
template <bool DIAG>
__device__ __forceinline__ void tail_tile(const fx4 (&at)[4][2], const float* sv, const float* sw,
                                          const float* sx, const float* sa, float (*cred)[TB],
                                          float* rsum, AS1 float* gA, const RMat& M, int cs, int k,
                                          int I, int K, int hr, double& tp) {
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  const int rg = lane >> 4, cg = lane & 15, R = q * 4 + rg;
  const int n = M.n, ib = I * TB + hr * HT;
  const unsigned uld = (unsigned)M.ld, ulda = (unsigned)M.lda;
  const int rs = (DIAG ? hr * HT : TB) + 4 * R;          // slot of this thread's first row
  const fx4 vr4 = *(const fx4*)(sv + rs), wr4 = *(const fx4*)(sw + rs), xr4 = *(const fx4*)(sx + rs);
  const fx4 vc0 = *(const fx4*)(sv + 8 * cg), vc1 = *(const fx4*)(sv + 8 * cg + 4);
  const fx4 wc0 = *(const fx4*)(sw + 8 * cg), wc1 = *(const fx4*)(sw + 8 * cg + 4);
  const fx4 xc0 = *(const fx4*)(sx + 8 * cg), xc1 = *(const fx4*)(sx + 8 * cg + 4);
  const fx4 ac0 = *(const fx4*)(sa + 8 * cg), ac1 = *(const fx4*)(sa + 8 * cg + 4);
  const float vr[4] = {vr4.x, vr4.y, vr4.z, vr4.w}, wr[4] = {wr4.x, wr4.y, wr4.z, wr4.w};
  const float xrv[4] = {xr4.x, xr4.y, xr4.z, xr4.w};
  const float vc[8] = {vc0.x, vc0.y, vc0.z, vc0.w, vc1.x, vc1.y, vc1.z, vc1.w};
  const float wc[8] = {wc0.x, wc0.y, wc0.z, wc0.w, wc1.x, wc1.y, wc1.z, wc1.w};
  const float xcv[8] = {xc0.x, xc0.y, xc0.z, xc0.w, xc1.x, xc1.y, xc1.z, xc1.w};
  const float acv[8] = {ac0.x, ac0.y, ac0.z, ac0.w, ac1.x, ac1.y, ac1.z, ac1.w};
  float av[4][8];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const bool piv = (ib + 4 * R + rr == k + 1);
    const float t[8] = {at[rr][0].x, at[rr][0].y, at[rr][0].z, at[rr][0].w,
                        at[rr][1].x, at[rr][1].y, at[rr][1].z, at[rr][1].w};
#pragma unroll
    for (int c = 0; c < 8; ++c) av[rr][c] = piv ? acv[c] : t[c] - (vr[rr] * wc[c] + wr[rr] * vc[c]);
  }
  // store rows >= k+2 (row k+1 stays A^(k-1): every workgroup reads it), upper, inside n.
  // Plain stores: the line stays in this XCD's L2, and within a 128-column
  // window the same workgroup index (same XCD) reads the tile next column;
  // write-through (sc1) stores measured slower (profiles/r6_wt_*.log)
  const int gc0 = K * TB + 8 * cg;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int gr = ib + 4 * R + rr;
    AS1 float* dst = gA + (unsigned)gr * ulda + gc0;
    const bool rok = (gr >= k + 2) & (gr < n);
    if (rok & (gc0 + 8 <= n) & (!DIAG || gc0 >= gr)) {
      const fx4 o0 = {av[rr][0], av[rr][1], av[rr][2], av[rr][3]};
      const fx4 o1 = {av[rr][4], av[rr][5], av[rr][6], av[rr][7]};
      *(AS1 fx4*)dst = o0;
      *(AS1 fx4*)(dst + 4) = o1;
    } else if (rok) {
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if ((gc0 + c < n) & (!DIAG || gc0 + c >= gr)) dst[c] = av[rr][c];
    }
  }
  float rp[4], cp[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) cp[c] = 0.f;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (DIAG) {   // upper triangle: row sums take col >= row, column sums col > row
        const int lr = hr * HT + 4 * R + rr, lc = 8 * cg + c;
        acc += (lc >= lr) ? av[rr][c] * xcv[c] : 0.f;
        cp[c] += (lc > lr) ? av[rr][c] * xrv[rr] : 0.f;
      } else {
        acc += av[rr][c] * xcv[c];
        cp[c] += av[rr][c] * xrv[rr];
      }
    }
    rp[rr] = row16_sum(acc);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) cp[c] = swap_sum32(swap_sum16(cp[c]));
  if (rg == 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) cred[q][8 * cg + c] = cp[c];
  }
  const float myrow = cg == 0 ? rp[0] : (cg == 1 ? rp[1] : (cg == 2 ? rp[2] : rp[3]));
  const float myx = cg == 0 ? xrv[0] : (cg == 1 ? xrv[1] : (cg == 2 ? xrv[2] : xrv[3]));
  if (DIAG) {
    if (cg < 4) rsum[4 * R + cg] = myrow;
  } else if (cg < 4) {
    gptr(M.P)[cs * M.sP + (unsigned)(2 * K) * uld + ib + 4 * R + cg] = myrow;
    tp = (double)myx * (double)myrow;
  }
}

template <int RB>
__device__ __forceinline__ void tail_body(const RMat& M, int local, int k, bool first) {
  constexpr int PK = RB / 4;
  constexpr int TQ = (RB * (RB + 1) + 1023) / 1024;
  static_assert(RB <= 64, "DS partials: one lane per row block");
  __shared__ float sq[4][TSLOT];        // per quarter of the P columns: yh partial of each slot row
  __shared__ __attribute__((aligned(16))) float sv[TSLOT], sw[TSLOT], sx[TSLOT], sa[TB];
  __shared__ float cred[4][TB];
  __shared__ float rsum[HT];
  __shared__ double sdk[2], stt[4], sds[2][2], tred[4];
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  const int n = M.n, nt = M.nt;
  const unsigned uld = (unsigned)M.ld, ulda = (unsigned)M.lda;
  const int cs = k & 1, ps = cs ^ 1;
  const int s0p = k / TB, s0 = (k + 1) / TB;
  const bool last = (k == n - 1), has1 = !last;
  int I = 0, K = 0;
  const int hr = local & 1;
  if (!last) {
    tri_index(local >> 1, nt - s0, I, K);
    I += s0; K += s0;
  }
  const bool diag = (I == K);
  const bool owner = !last && diag && hr == 0;
  const int nslot = last ? 0 : (diag ? TB : TSLOT);
  const int ib = I * TB + hr * HT;                       // first row of the half tile
  auto slot_row = [&](int sl) -> int { return sl < TB ? K * TB + sl : ib + (sl - TB); };
  const AS1 float* DSp = gptr(M.DS) + ps * M.sDS;
  const AS1 float* TSp = gptr(M.TS) + ps * M.sTS;
  const AS1 float* Pp = gptr(M.P) + ps * M.sP;
  const AS1 float* XHp = gptr(M.XH) + ps * M.sX;
  const AS1 float* AVp = gptr(M.AV) + ps * M.sX;
  AS1 float* const gA = gptr(M.A);
  AS1 float* const gSC = gptr(M.SC);
  const int ntri = (nt - s0p) * (nt - s0p + 1);          // half tiles of the previous launch
  unsigned long long* const stamps = first ? g_stamps : nullptr;
  const int j = k;
  STAMP(1);

  // ---- every load up front (clamped indices, out-of-range terms dropped at use)
  const float dk = gld_if32(DSp, (unsigned)min(s0p + lane, nt - 1) * NK + (q & 1),
                            (q < 2) & (s0p + lane < nt), 0.f);
  fx4 tq[TQ];
  const fx4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < TQ; ++u)
    tq[u] = gld_if32((const AS1 fx4*)TSp, (unsigned)(tid + 256 * u), 4 * (tid + 256 * u) < ntri, z4);
  auto pcol_ok = [&](int col, int B) -> bool {
    return (col >= 2 * s0p) & (col < 2 * nt) & (((col & 1) == 0) | ((col >> 1) <= B));
  };
  const int bk = k / TB, bk1 = (k + 1) / TB;
  float pj = 0.f, pj1 = 0.f;                             // pivot rows k, k+1: lane = P column
#pragma unroll
  for (int h = 0; h < (2 * RB + 63) / 64; ++h) {
    const int col = 2 * s0p + lane + 64 * h;
    pj += gld_if32(Pp, (unsigned)col * uld + k, pcol_ok(col, bk), 0.f);
    pj1 += gld_if32(Pp, (unsigned)col * uld + k + 1, has1 & pcol_ok(col, bk1), 0.f);
  }
  const float alpha = gSC[ps * 4];
  const float dprev = gSC[ps * 4 + 1];
  const float ak = AVp[k];
  const float ak1 = gld_if32(AVp, k + 1, has1, 0.f);
  const float xhk1 = gld_if32(XHp, k + 1, has1, 0.f);
  // this wave's quarter of the P columns of slot rows lane + 64 g
  float pk[3][2 * PK];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    const int rc = min(slot_row(lane + 64 * g), n - 1);
#pragma unroll
    for (int i = 0; i < PK; ++i) {
      const unsigned t2 = 2 * min(s0p + q + 4 * i, nt - 1);
      pk[g][2 * i] = Pp[t2 * uld + rc];
      pk[g][2 * i + 1] = Pp[(t2 + 1) * uld + rc];
    }
  }
  // the slot row of this thread (tid < nslot): xh_{k-1}, a_{k-1}, storage row k+1
  const int rme = slot_row(min(tid, TSLOT - 1));
  const int rmc = min(rme, n - 1);
  const float xhr = XHp[(unsigned)rmc];
  const float avr = AVp[(unsigned)rmc];
  const float arow = gld_if32(gA, (unsigned)(k + 1) * ulda + max(rmc, k + 1), has1, 0.f);
  // the half tile: rows ib + 4 R + rr, columns K TB + 8 cg + 0..7
  const int rg = lane >> 4, cg = lane & 15, R = q * 4 + rg;
  fx4 at[4][2];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      at[rr][h] = *(const AS1 fx4*)(gA + (unsigned)min(ib + 4 * R + rr, nt * TB - 1) * ulda +
                                    K * TB + 8 * cg + 4 * h);
  __builtin_amdgcn_sched_barrier(0);

  // ---- global sums of column k-1, the slot rows' yh partials
  {
    const double dsum = wave_sum_d((double)dk);
    if (q < 2 && lane == 0) sdk[q] = dsum;
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < TQ; ++u) {
      const int f = 4 * (tid + 256 * u);
      t += (f < ntri) ? (double)tq[u].x : 0.0;
      t += (f + 1 < ntri) ? (double)tq[u].y : 0.0;
      t += (f + 2 < ntri) ? (double)tq[u].z : 0.0;
      t += (f + 3 < ntri) ? (double)tq[u].w : 0.0;
    }
    t = wave_sum_d(t);
    if (lane == 0) stt[q] = t;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      const int B = slot_row(lane + 64 * g) / TB;
      float yq = 0.f;
#pragma unroll
      for (int i = 0; i < PK; ++i) {
        const int T = s0p + q + 4 * i;
        yq += (T < nt) ? pk[g][2 * i] : 0.f;
        yq += ((T < nt) & (T <= B)) ? pk[g][2 * i + 1] : 0.f;
      }
      sq[q][lane + 64 * g] = yq;
    }
  }
  const float yk = wave_sum(pj), yk1 = wave_sum(pj1);
  kfac_lds_barrier();
  STAMP(2);

  // ---- scalars of column k-1 (every thread, identically), pivot rows k, k+1
  const double sig2 = sdk[0], xa = sdk[1];
  const double xy = ((stt[0] + stt[1]) + (stt[2] + stt[3]));
  double beta, tau, s;
  hh_scalars((double)alpha, sig2, beta, tau, s);
  const double vy = (double)ak + 2.0 * s * xa + s * s * xy;
  const double alpha2 = -0.5 * tau * tau * vy;
  float vk, wk, vk1 = 0.f, wk1 = 0.f;
  tail_vw(tau, s, alpha2, true, 0.f, ak, yk, vk, wk);
  if (has1) tail_vw(tau, s, alpha2, false, xhk1, ak1, yk1, vk1, wk1);
  if (local == 0 && tid == 0) {
    M.d[k - 1] = dprev;
    M.e[k - 1] = (float)beta;
    M.tau[k - 1] = (float)tau;
    gA[(unsigned)(k - 1) * ulda + k] = (float)beta;
    const float dkk = (float)((double)ak - 2.0 * (double)wk);
    if (last) {
      M.d[k] = dkk;
      M.e[k] = 0.f;
      M.tau[k] = 0.f;
    } else {
      gSC[cs * 4 + 1] = dkk;
    }
  }
  if (last) return;
  STAMP(3);

  // ---- the slot rows: v, w of column k-1; x_k (-> xh_k), a_k = row k+1 of A^(k)
  {
    float v = 0.f, w = 0.f, xn = 0.f, an = 0.f;
    if (tid < nslot) {
      const int r = rme;
      float yh = (sq[0][tid] + sq[1][tid]) + (sq[2][tid] + sq[3][tid]);
      if (r >= k && r < n) {
        if (r == k) {
          v = vk; w = wk;
        } else if (r == k + 1) {
          v = vk1; w = wk1;
        } else {
          tail_vw(tau, s, alpha2, false, xhr, avr, yh, v, w);
        }
      }
      const float x = avr - w - wk * v;
      xn = (r >= k + 2 && r < n) ? x : 0.f;
      an = (r >= k + 1 && r < n) ? arow - vk1 * w - wk1 * v : 0.f;
      sv[tid] = v; sw[tid] = w; sx[tid] = xn;
      if (tid < TB) sa[tid] = an;
      if (owner && r < n) {
        gptr(M.XH)[cs * M.sX + r] = xn;
        gptr(M.AV)[cs * M.sX + r] = an;
        if (r >= k + 1) gA[(unsigned)(k - 1) * ulda + r] = v;   // reflector k-1: v[k+1:]
        if (r == k + 1) gSC[cs * 4] = x;                       // alpha_k
      }
    }
    if (owner && q < 2) {        // block sums |xh_k|^2, xh_k . a_k (rows 0..127 = waves 0, 1)
      const double s0v = wave_sum_d((double)xn * (double)xn);
      const double s1v = wave_sum_d((double)xn * (double)an);
      if (lane == 0) { sds[q][0] = s0v; sds[q][1] = s1v; }
    }
  }
  kfac_lds_barrier();
  STAMP(4);
  if (owner && tid < 2)
    gptr(M.DS)[cs * M.sDS + (long long)K * NK + tid] = (float)(sds[0][tid] + sds[1][tid]);

  // ---- the tile: column k-1's rank-2 update, store, then the symv of column k
  double tp = 0.0;
  if (diag)
    tail_tile<true>(at, sv, sw, sx, sa, cred, rsum, gA, M, cs, k, I, K, hr, tp);
  else
    tail_tile<false>(at, sv, sw, sx, sa, cred, rsum, gA, M, cs, k, I, K, hr, tp);
  AS1 float* const Pc = gptr(M.P) + cs * M.sP;
  STAMP(5);
  kfac_lds_barrier();
  if (tid < TB) {
    float v = (cred[0][tid] + cred[1][tid]) + (cred[2][tid] + cred[3][tid]);
    if (diag) {
      const int rl = tid - hr * HT;
      if (rl >= 0 && rl < HT) v += rsum[rl];
    }
    Pc[(unsigned)(2 * I + hr) * uld + K * TB + tid] = v;
    tp += (double)sx[tid] * (double)v;
  }
  {
    const double t = wave_sum_d(tp);
    if (lane == 0) tred[q] = t;
  }
  kfac_lds_barrier();
  if (tid == 0)
    gptr(M.TS)[cs * M.sTS + local] = (float)((tred[0] + tred[1]) + (tred[2] + tred[3]));
  STAMP(6);
}

template <int RB>
__global__ __launch_bounds__(256) void red_tail_kernel(const RMat* __restrict__ mats,
                                                       const int* __restrict__ offs, int nact,
                                                       int k) {
  unsigned long long* const stamps = blockIdx.x == 0 ? g_stamps : nullptr;
  const int j = k;
  STAMP(0);
  int mi, base;
  find_mat(offs, nact, mi, base);
  const RMat M = mats[mi];
  tail_body<RB>(M, blockIdx.x - base, k, blockIdx.x == 0);
}

// a column where blocked and tail matrices are both active: S(j) of the
// blocked ones (workgroups 0 .. grid_s - 1) and L(j) of the tail ones in ONE
// launch, so a mixed batch does not pay a third dependent launch per column
template <int RB>
__global__ __launch_bounds__(256) void red_symv_tail_kernel(const RMat* __restrict__ mats,
                                                            const int* __restrict__ offs_s,
                                                            int nact_s, int grid_s,
                                                            const int* __restrict__ offs_l,
                                                            int nact_l, int j) {
  int mi, base;
  if ((int)blockIdx.x < grid_s) {
    find_mat_b(offs_s, nact_s, blockIdx.x, mi, base);
    const RMat M = mats[mi];
    symv_body(M, base, j);
  } else {
    const int b = blockIdx.x - grid_s;
    find_mat_b(offs_l, nact_l, b, mi, base);
    const RMat M = mats[mi];
    tail_body<RB>(M, b - base, j, false);
  }
}

// ------------------------------------------------------------------ host
constexpr int NKIND = 4;        // F, U, S, L
struct RPlan {
  RMat* d_mats = nullptr;
  int* d_offs = nullptr;        // [NKIND][nmax][nm + 1]: F, U, S, L workgroup offsets
  std::vector<int> n_sorted;    // descending
  std::vector<int> grid[NKIND]; // [nmax] total workgroups per launch kind
  std::vector<int> nact[NKIND];
  std::vector<int> rb;          // [nmax] F unroll class
  std::vector<int> rbt;         // [nmax] L unroll class
  int nmax = 0;
  hipGraphExec_t exec = nullptr;
};

inline int h_tri(int m) { return m * (m + 1) / 2; }

// trailing size (rows) from which a matrix's columns run as single tail
// launches (KFAC_REDUCE_TAIL, 0 = never); capped so the tail's P partials fit
// its unroll classes (<= 40 row blocks)
constexpr int TAIL_MAX = 38 * TB;
int g_tail_override = -1;    // kfac_reduce_set_tail: the next plans' threshold
int tail_rows() {
  static const int t = [] {
    const char* e = getenv("KFAC_REDUCE_TAIL");
    const int v = e ? atoi(e) : 768;
    return std::max(0, std::min(v, TAIL_MAX));
  }();
  return g_tail_override >= 0 ? std::min(g_tail_override, TAIL_MAX) : t;
}

// the panel start j0 after which matrix n runs tail launches (n: no tail)
int tail_start(int n) {
  const int T = tail_rows();
  if (T <= 0) return n;
  const int j0 = n <= T ? 0 : (n - T + NB - 1) / NB * NB;
  return j0 >= n - 1 ? n : j0;
}

// workgroups of matrix n at column j: F, U (panel start only), S -- blocked
// columns j <= j0 -- and L, the tail columns j > j0
void counts(int n, int j, int out[NKIND]) {
  const int nt = (n + TB - 1) / TB, nf = (n + FB - 1) / FB;
  const int ntr = nt - (j + 1) / TB;
  const int j0 = tail_start(n);
  const bool blk = j <= j0;
  out[0] = (blk && j <= n - 1) ? nf - std::min(((j + 1) / TB) * (TB / FB), j / FB) : 0;
  out[1] = (blk && j % NB == 0 && j > 0 && j <= n - 2) ? h_tri(ntr) : 0;
  out[2] = (blk && j <= n - 2) ? 2 * h_tri(ntr) / SNH + ntr : 0;
  out[3] = blk ? 0 : (j <= n - 2 ? 2 * h_tri(ntr) : (j == n - 1 ? 1 : 0));
}

int rb_class(int blocks) {
  static const int cls[] = {8, 16, 24, 40, 64, 96, 128};
  for (int c : cls)
    if (blocks <= c) return c;
  return -1;
}

template <int RB>
void launch_fin(const RPlan& P, const int* of, int j, hipStream_t s) {
  hipLaunchKernelGGL(red_fin_kernel<RB>, dim3(P.grid[0][j]), dim3(256), 0, s, P.d_mats, of,
                     P.nact[0][j], j);
}

// panel-update MFMA precision: bf16x6 (default) or exact f32 (KFAC_REDUCE_UPD=f32)
const bool g_upd_x6 = [] {
  const char* e = getenv("KFAC_REDUCE_UPD");
  return !(e && !strcmp(e, "f32"));
}();

template <int RB>
void launch_tail(const RPlan& P, const int* of, int j, hipStream_t s) {
  hipLaunchKernelGGL(red_tail_kernel<RB>, dim3(P.grid[3][j]), dim3(256), 0, s, P.d_mats, of,
                     P.nact[3][j], j);
}

int enqueue(const RPlan& P, hipStream_t stream) {
  const int nm = (int)P.n_sorted.size();
  const size_t kstride = (size_t)P.nmax * (nm + 1);
  for (int j = 0; j < P.nmax; ++j) {
    const int* of = P.d_offs + (size_t)j * (nm + 1);
    if (P.grid[0][j] > 0) {
      switch (P.rb[j]) {
        case 8: launch_fin<8>(P, of, j, stream); break;
        case 16: launch_fin<16>(P, of, j, stream); break;
        case 24: launch_fin<24>(P, of, j, stream); break;
        case 40: launch_fin<40>(P, of, j, stream); break;
        case 64: launch_fin<64>(P, of, j, stream); break;
        case 96: launch_fin<96>(P, of, j, stream); break;
        default: launch_fin<128>(P, of, j, stream); break;
      }
    }
    if (P.grid[1][j] > 0) {
      const dim3 g(P.grid[1][j]);
      const int* ou = of + kstride;
      if (g_upd_x6)
        hipLaunchKernelGGL(red_upd_kernel<true>, g, dim3(256), 0, stream, P.d_mats, ou,
                           P.nact[1][j], j);
      else
        hipLaunchKernelGGL(red_upd_kernel<false>, g, dim3(256), 0, stream, P.d_mats, ou,
                           P.nact[1][j], j);
    }
    if (P.grid[2][j] > 0 && P.grid[3][j] > 0) {
      const int* os = of + 2 * kstride;
      const int* ot = of + 3 * kstride;
      const dim3 g(P.grid[2][j] + P.grid[3][j]);
#define KFAC_ST(RB_)                                                                          \
  hipLaunchKernelGGL(red_symv_tail_kernel<RB_>, g, dim3(256), 0, stream, P.d_mats, os,        \
                     P.nact[2][j], P.grid[2][j], ot, P.nact[3][j], j)
      switch (P.rbt[j]) {
        case 8: KFAC_ST(8); break;
        case 16: KFAC_ST(16); break;
        case 24: KFAC_ST(24); break;
        default: KFAC_ST(40); break;
      }
#undef KFAC_ST
      continue;
    }
    if (P.grid[2][j] > 0)
      hipLaunchKernelGGL(red_symv_kernel, dim3(P.grid[2][j]), dim3(256), 0, stream, P.d_mats,
                         of + 2 * kstride, P.nact[2][j], j);
    if (P.grid[3][j] > 0) {
      const int* ot = of + 3 * kstride;
      switch (P.rbt[j]) {
        case 8: launch_tail<8>(P, ot, j, stream); break;
        case 16: launch_tail<16>(P, ot, j, stream); break;
        case 24: launch_tail<24>(P, ot, j, stream); break;
        default: launch_tail<40>(P, ot, j, stream); break;
      }
    }
  }
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, RPlan> g_plans;

}  // namespace

// workspace floats per matrix (V, W and the 2-slot partial rings), zeroed by
// the caller once (rows past n of XH / AV / P must read 0)
// Tail threshold for plans built from now on (-1: KFAC_REDUCE_TAIL / 768); a
// plan keeps the threshold it was built with.  Returns the previous override.
KFAC_API int kfac_reduce_set_tail(int rows) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int prev = g_tail_override;
  g_tail_override = rows;
  return prev;
}

KFAC_API long long kfac_reduce_ws_floats(int n) { return ws_layout(n).total; }

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
    if (r.n < 2) { *err = -2; return nullptr; }
    if (r.n > NMAX) { *err = -6; return nullptr; }
    const WsLayout L = ws_layout(r.n);
    if (r.lda < (long long)L.nt * TB || (r.lda % TB)) { *err = -2; return nullptr; }
    RMat M;
    memset(&M, 0, sizeof(M));
    M.A = r.A; M.lda = r.lda; M.n = (int)r.n; M.nt = L.nt; M.ld = L.ld;
    M.nf = (int)((r.n + FB - 1) / FB);
    M.d = r.d; M.e = r.e; M.tau = r.tau;
    M.V = r.ws + L.V; M.W = r.ws + L.W; M.P = r.ws + L.P; M.TS = r.ws + L.TS;
    M.DS = r.ws + L.DS; M.XH = r.ws + L.XH; M.AV = r.ws + L.AV; M.SC = r.ws + L.SC;
    M.sP = L.sP; M.sTS = L.sTS; M.sDS = L.sDS; M.sX = L.sX;
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
    std::vector<int> offs((size_t)NKIND * P.nmax * (nm + 1), 0);
    for (int k = 0; k < NKIND; ++k) {
      P.grid[k].assign(P.nmax, 0);
      P.nact[k].assign(P.nmax, 0);
    }
    P.rb.assign(P.nmax, 0);
    P.rbt.assign(P.nmax, 0);
    for (int j = 0; j < P.nmax; ++j) {
      int acc[NKIND] = {0, 0, 0, 0};
      int rbf = 1, rbl = 1;     // row blocks of the previous launch's partials (F / L readers)
      for (int i = 0; i < nm; ++i) {
        int cnt[NKIND];
        counts(P.n_sorted[i], j, cnt);
        const int blocks = (P.n_sorted[i] + TB - 1) / TB - j / TB;
        if (cnt[0] > 0) rbf = std::max(rbf, blocks);
        if (cnt[3] > 0) rbl = std::max(rbl, blocks);
        for (int k = 0; k < NKIND; ++k) {
          offs[((size_t)k * P.nmax + j) * (nm + 1) + i] = acc[k];
          if (cnt[k] > 0) P.nact[k][j] = i + 1;
          acc[k] += cnt[k];
        }
      }
      for (int k = 0; k < NKIND; ++k) {
        offs[((size_t)k * P.nmax + j) * (nm + 1) + nm] = acc[k];
        P.grid[k][j] = acc[k];
        // uniform launch: the active matrices (a prefix: sizes descend) share one count
        const int na = P.nact[k][j];
        if (na > 0 && acc[k] % na == 0) {
          int c0[NKIND];
          counts(P.n_sorted[0], j, c0);
          bool uni = true;
          for (int i = 1; i < na && uni; ++i) {
            int ci[NKIND];
            counts(P.n_sorted[i], j, ci);
            uni = ci[k] == c0[k];
          }
          if (uni && c0[k] > 0 && c0[k] * na == acc[k]) P.nact[k][j] = -c0[k];
        }
      }
      // F / L read the partials of the previous launch: nt - j / TB blocks
      static const int rb_min = getenv("KFAC_REDUCE_RB_MIN") ? atoi(getenv("KFAC_REDUCE_RB_MIN")) : 1;
      P.rb[j] = rb_class(std::max(rb_min, rbf));
      if (P.rb[j] < 0) { *err = -6; return nullptr; }
      P.rbt[j] = rbl <= 8 ? 8 : (rbl <= 16 ? 16 : (rbl <= 24 ? 24 : 40));
      if (rbl > 40) { *err = -6; return nullptr; }
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

// Tridiagonalise `count` symmetric matrices (any sizes 2 .. 16384) with one
// launch sequence for all of them: A (lda x lda, row-major, lda = n rounded up
// to a multiple of 128, zero outside the leading n x n block; its upper
// triangle is read and overwritten by the reflectors), d, e, tau (n floats each), ws
// (kfac_reduce_ws_floats(n) floats, 256-byte aligned, zeroed once).
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

// debug: record per-column stamps of the first F / S workgroups into `buf`
// (nmax x 16 uint64: F 0-4, S tile 10-11, S row-block partials 12-13), or
// stop with nullptr
KFAC_API int kfac_reduce_stamps(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
}

KFAC_API int kfac_reduce_prepare(const KfacReduceRecord* recs, int count) {
  int err = 0;
  return plan_for(recs, count, true, &err) ? 0 : (err ? err : -4);
}

KFAC_API int kfac_reduce_max_n() { return NMAX; }
