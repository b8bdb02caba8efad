// Batched symmetric tridiagonal divide-and-conquer eigensolver for gfx950
// (stage 2 of the hand-written eigensolver, between the
// tridiagonal reduction of csrc/eig_reduce.hip and the back-transformation of
// csrc/eig_backtransform.hip).
//
// Every matrix of an inverse update goes through ONE launch sequence: the
// recursion trees of all matrices are processed level by level (all merges of
// one height, over all matrices, in one launch per phase), and the whole
// sequence is captured into one hipGraph per buffer set -- no host round trip,
// no library call.  The algorithm is modelled step by step (same buffers and
// index conventions) in scripts/models/dc_model.py:
//
//   leaf     one workgroup per leaf (<= LEAF = 32 rows): the torn leaf block as a
//            dense matrix in LDS, cyclic parallel Jacobi in fp64, ascending
//   prep     one workgroup per merge: z from the children's boundary columns,
//            the 4 ascending runs of the two children merged by rank (binary
//            searches), LAPACK dlaed2 deflation (small rho |z|, Givens
//            rotations of close poles, deflated run kept ascending), surviving
//            poles grouped by type (1 left-only rows, 2 mixed, 3 right-only) so
//            the eigenvector GEMMs skip structural zeros; patches this merge's
//            two GEMM records in device memory (M = #roots, K per type range)
//   rotate   the recorded rotations, one thread per column, in order
//   gather   ZpT[c][j] = Z[src_j][c] (LDS-tiled transpose), deflated rows -> U
//   secular  one wave per root, fp64: Li's middle-way two-pole model with a
//            bracket safeguard (geometric bisection near a pole); fp64 roots of
//            the fp32 rank-one problem give eigenvectors orthogonal to fp32
//            precision (no Gu-Eisenstat recomputation needed); the eigenvector
//            row u_j = w_j / (d_j - lambda) / ||.|| goes to U in type order
//   gemm     Z[:, left] = U[:, t1+t2] ZpT[left]^T, Z[:, right] = U[:, t2+t3]
//            ZpT[right]^T: the grouped exact-f32 MFMA GEMM of
//            csrc/precond_gemm.hip, tile grid sized for the worst case, M / K
//            read from the records the prep kernel wrote
//   final    the root's two ascending runs merged by rank: eigenvalues
//            ascending, eigenvector ROWS permuted into the output
//
// Storage per matrix (workspace carved by the host): Zw (n x ldw fp32, row i of
// a node block = eigenvector i of that node in the node's own columns), ZpT, U
// (n x ldw), fp64 eigenvalues and scratch.  Output: d ascending, Zout row k =
// eigenvector k (the layout the compact-WY back-transformation reads).
// Reference semantics: kfac/layers/utils.py:45-74 (symeig, ascending).
#include "pgemm.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

// leaf rows: the fp64 cyclic Jacobi leaf costs ~rounds x sweeps LDS barriers
// (rows - 1 rounds per sweep); 32-row leaves halve the rounds for one more,
// cheap, merge level (ResNet-50 inverse update 159 -> 157 ms)
constexpr int LEAF = 32;
constexpr int PADK = 36;          // zero columns past k in U / ZpT rows (GEMM k-steps)
constexpr int LDS_M_MAX = 4800;   // merges up to this size scan in LDS (32 B per row)
constexpr double EPS32 = 5.9604644775390625e-08;   // 2^-24 (LAPACK slamch 'E')
constexpr double EPS64 = 1.1102230246251565e-16;   // 2^-53
constexpr int MAX_IT = 64;
constexpr int RPB = 4;            // secular: roots (waves) per block
constexpr int TILE_F32 = 0;       // pgemm 128 x 128, 4 waves (profiles/r2_pgemm_sweep.log)
// GEMM precision of the merge (eigenvector update Zw = U ZpT): both operands
// are orthogonal-matrix entries (|x| <= 1), so fp16x3 with a fixed 2^14
// scale (PREC_F16X3F: three fp16 MFMA products, 22 significand bits); or
// KFAC_EIG_GEMM=bf16x6 (six bf16 products) / fp32 (exact f32 MFMA)
const int g_dc_prec = [] {
  const char* e = getenv("KFAC_EIG_GEMM");
  if (e && !strcmp(e, "fp32")) return (int)PREC_F32;
  if (e && !strcmp(e, "bf16x6")) return (int)PREC_BF16X6F;
  return (int)PREC_F16X3F;
}();
// the wave-parallel deflation scan of dc_prep (KFAC_DC_SERIAL_SCAN=1: every
// chunk through the sequential path -- the reference for the bitwise test)
int g_dc_fast_scan = [] {
  const char* e = getenv("KFAC_DC_SERIAL_SCAN");
  return (e && e[0] == '1') ? 0 : 1;
}();
constexpr int TYP_SHIFT = 28;
constexpr int SRC_MASK = (1 << TYP_SHIFT) - 1;

inline long long rup(long long a, long long b) { return (a + b - 1) / b * b; }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// device pointers in the global address space: accesses through a record
// loaded from memory compile to global_* (not flat_*, which also waits on
// lgkmcnt)
struct DcMat {
  const AS1 float* d; const AS1 float* e;
  AS1 float* dout; AS1 float* Zout; long long ldz;
  AS1 float* Zw; AS1 float* ZpT; AS1 float* U; long long ldw;
  AS1 double* dval; AS1 double* dl; AS1 double* wv; AS1 double* defv; AS1 double* rho;
  AS1 double* gds; AS1 double* gzs; AS1 double* gdef;
  AS1 int* kk; AS1 int* k1a; AS1 int* nrot; AS1 int* typepos; AS1 int* gsrc; AS1 int* dsrc;
  AS1 int* gsrcx; AS1 int* gdefsrc;
  AS1 int* rp; AS1 float* rcs; AS1 int* info;
  int n; int pad;
};

struct DcNode { int mat, lo, mid, hi; };

__device__ inline double block_sum(double v, double* red) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__device__ inline double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ inline double block_max(double v, double* red) {
  v = wave_max_d(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s = fmax(s, red[w]);
  return s;
}

// ------------------------------------------------------------------- zero
__global__ __launch_bounds__(256) void dc_zero_kernel(const DcMat* __restrict__ mats) {
  const DcMat M = mats[blockIdx.y];
  const long long total = (long long)M.n * M.ldw / 4;
  float4* p = (float4*)M.Zw;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256)
    p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (blockIdx.x == 0 && threadIdx.x == 0) M.info[0] = 0;
}

// ------------------------------------------------------------------- leaf
// Cyclic parallel Jacobi (round-robin pairs) on the torn leaf block, fp64 in
// LDS; V rows are the eigenvectors.
__global__ __launch_bounds__(256) void dc_leaf_kernel(const DcMat* __restrict__ mats,
                                                      const DcNode* __restrict__ nodes) {
  __shared__ double S[LEAF][LEAF + 1];
  __shared__ double V[LEAF][LEAF + 1];
  __shared__ double rc[LEAF / 2], rs[LEAF / 2], rt[LEAF / 2], rpp[LEAF / 2], rqq[LEAF / 2],
      rpq[LEAF / 2];
  __shared__ int rpi[LEAF / 2], rqi[LEAF / 2];
  __shared__ int nrot;
  __shared__ double dsh[LEAF];
  const DcNode nd = nodes[blockIdx.x];
  const DcMat M = mats[nd.mat];
  const int lo = nd.lo, hi = nd.hi, nl = hi - lo, n = M.n;
  const int ne = nl + (nl & 1);
  const int npairs = ne / 2;
  const int tid = threadIdx.x;
  for (int x = tid; x < ne * ne; x += 256) {
    const int i = x / ne, j = x - i * ne;
    double v = 0.0;
    if (i < nl && j < nl) {
      if (i == j) {
        v = (double)M.d[lo + i];
        if (i == 0 && lo > 0) v -= fabs((double)M.e[lo - 1]);
        if (i == nl - 1 && hi < n) v -= fabs((double)M.e[hi - 1]);
      } else if (j == i + 1) {
        v = (double)M.e[lo + i];
      } else if (i == j + 1) {
        v = (double)M.e[lo + j];
      }
    }
    S[i][j] = v;
    V[i][j] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  const int mm = ne - 1;
  for (int sweep = 0; sweep < 40 && mm > 0; ++sweep) {
    if (tid == 0) nrot = 0;
    __syncthreads();
    for (int r = 0; r < mm; ++r) {
      for (int k = tid; k < npairs; k += 256) {
        int a, b;
        if (k == 0) { a = mm; b = r; }
        else { a = (r + k) % mm; b = (r - k + mm) % mm; }
        const int p = a < b ? a : b, q = a < b ? b : a;
        const double app = S[p][p], aqq = S[q][q], apq = S[p][q];
        double c = 1.0, s = 0.0, t = 0.0;
        if (fabs(apq) > 1e-300 && fabs(apq) > 1e-15 * sqrt(fabs(app) * fabs(aqq))) {
          const double theta = (aqq - app) / (2.0 * apq);
          t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(1.0 + theta * theta));
          c = 1.0 / sqrt(1.0 + t * t);
          s = t * c;
          atomicAdd(&nrot, 1);
        }
        rpi[k] = p; rqi[k] = q; rc[k] = c; rs[k] = s; rt[k] = t;
        rpp[k] = app; rqq[k] = aqq; rpq[k] = apq;
      }
      __syncthreads();
      for (int x = tid; x < npairs * ne; x += 256) {   // S <- S J, V rows p, q
        const int k = x / ne, i = x - k * ne;
        const double c = rc[k], s = rs[k];
        if (s == 0.0) continue;
        const int p = rpi[k], q = rqi[k];
        const double tau = s / (1.0 + c);
        const double sp = S[i][p], sq = S[i][q];
        S[i][p] = sp - s * (sq + tau * sp);
        S[i][q] = sq + s * (sp - tau * sq);
        const double vp = V[p][i], vq = V[q][i];
        V[p][i] = vp - s * (vq + tau * vp);
        V[q][i] = vq + s * (vp - tau * vq);
      }
      __syncthreads();
      for (int x = tid; x < npairs * ne; x += 256) {   // S <- J^T S
        const int k = x / ne, j = x - k * ne;
        const double c = rc[k], s = rs[k];
        if (s == 0.0) continue;
        const int p = rpi[k], q = rqi[k];
        const double tau = s / (1.0 + c);
        const double sp = S[p][j], sq = S[q][j];
        S[p][j] = sp - s * (sq + tau * sp);
        S[q][j] = sq + s * (sp - tau * sq);
      }
      __syncthreads();
      for (int k = tid; k < npairs; k += 256) {
        if (rs[k] != 0.0) {
          const int p = rpi[k], q = rqi[k];
          S[p][q] = 0.0; S[q][p] = 0.0;
          S[p][p] = rpp[k] - rt[k] * rpq[k];
          S[q][q] = rqq[k] + rt[k] * rpq[k];
        }
      }
      __syncthreads();
    }
    if (nrot == 0) break;
    __syncthreads();
  }
  for (int i = tid; i < nl; i += 256) dsh[i] = S[i][i];
  __syncthreads();
  for (int i = tid; i < nl; i += 256) {
    const double di = dsh[i];
    int rank = 0;
    for (int j = 0; j < nl; ++j) {
      const double dj = dsh[j];
      rank += (dj < di) || (dj == di && j < i);
    }
    M.dval[lo + rank] = di;
    AS1 float* row = M.Zw + (long long)(lo + rank) * M.ldw + lo;
    for (int c = 0; c < nl; ++c) row[c] = (float)V[i][c];
  }
  if (tid == 0) M.kk[lo] = nl;
}

// ------------------------------------------------------------------- prep
// count of elements of the ascending run a[s, e) below v (or <= v)
template <class P>
__device__ inline int run_count(P a, int s, int e, double v, bool le) {
  int lo = s, hi = e;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const bool below = le ? (a[mid] <= v) : (a[mid] < v);
    if (below) lo = mid + 1; else hi = mid;
  }
  return lo - s;
}

__global__ __launch_bounds__(256) void dc_prep_kernel(const DcMat* __restrict__ mats,
                                                      const DcNode* __restrict__ nodes,
                                                      PGemm* __restrict__ table, int use_lds,
                                                      int use_fast) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  __shared__ double red[4];
  __shared__ int sh_k, sh_nrot, sh_cnt[3][256];
  const DcNode nd = nodes[blockIdx.x];
  const DcMat M = mats[nd.mat];
  const int lo = nd.lo, mid = nd.mid, hi = nd.hi;
  const int n1 = mid - lo, n2 = hi - mid, m = hi - lo;
  const long long ldw = M.ldw;
  const int tid = threadIdx.x;
  // staging arrays in LDS (use_lds) or global scratch: the body is templated
  // on their address space (a pointer that may be either compiles to flat_*
  // accesses, slow in the serial deflation scan).  sd / sz / ssrc: unsorted
  // staging of steps 1-2; sd2 / sz2 / ssrc2: the sorted arrays from step 3 on
  auto body = [&](auto sd, auto sz, auto sdef, auto ssrc, auto sdefsrc, auto sd2, auto sz2,
                  auto ssrc2, bool copy_sorted) {
  const double beta = (double)M.e[mid - 1];
  const int kL = M.kk[lo], kR = M.kk[mid];
  // -- 1. z from the children's boundary columns, eigenvalues (unsorted staging)
  double nz = 0.0;
  for (int i = tid; i < m; i += 256) {
    const float zf = (i < n1) ? M.Zw[(long long)(lo + i) * ldw + (mid - 1)]
                              : M.Zw[(long long)(lo + i) * ldw + mid];
    double z = (double)zf;
    if (i >= n1 && beta < 0.0) z = -z;
    sz[i] = z;
    sd[i] = M.dval[lo + i];
    nz += z * z;
  }
  const double nz2 = block_sum(nz, red);    // has barriers: sd / sz visible
  const double zscale = nz2 > 0.0 ? 1.0 / sqrt(nz2) : 0.0;
  const double rho = fabs(beta) * nz2;
  // -- 2. merge of the runs [0,kL) [kL,n1) [n1,n1+kR) [n1+kR,m) by rank
  const int rs_[5] = {0, kL, n1, n1 + kR, m};
  for (int i = tid; i < m; i += 256) {
    const int r = (i < kL) ? 0 : (i < n1) ? 1 : (i < n1 + kR) ? 2 : 3;
    const double v = sd[i];
    int rank = i - rs_[r];
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2)
      if (r2 != r) rank += run_count(sd, rs_[r2], rs_[r2 + 1], v, r2 < r);
    rank = rank < 0 ? 0 : (rank >= m ? m - 1 : rank);
    M.gds[lo + rank] = v;
    M.gzs[lo + rank] = sz[i] * zscale;
    M.gsrcx[lo + rank] = i | ((i < n1 ? 1 : 3) << TYP_SHIFT);
  }
  __threadfence_block();
  __syncthreads();
  if (copy_sorted) {
    for (int p = tid; p < m; p += 256) {
      sd2[p] = M.gds[lo + p];
      sz2[p] = M.gzs[lo + p];
      ssrc2[p] = M.gsrcx[lo + p];
    }
  }
  __syncthreads();
  // -- 3. deflation tolerance
  double dmx = 0.0, zmx = 0.0;
  for (int p = tid; p < m; p += 256) {
    dmx = fmax(dmx, fabs(sd2[p]));
    zmx = fmax(zmx, fabs(sz2[p]));
  }
  dmx = block_max(dmx, red);
  zmx = block_max(zmx, red);
  const double tol = 8.0 * EPS32 * fmax(dmx, rho * zmx);
  // -- 4. deflation scan (LAPACK dlaed2 order); survivors compacted in place at
  // the front of sd2 / sz2 / ssrc2, deflated run ascending.  Wave 0 takes 64
  // elements at a time: z-deflation is per element, and with no Givens
  // deflation in the chunk (the rotation test of every surviving pole
  // against the one before it comes out false -- the usual case) the chunk's
  // effect is a compaction: survivors flushed in order, z-deflated values
  // appended (the run stays ascending: sd2 is sorted).  A chunk with a
  // rotation, or whose first appended value sorts below the run's end, runs
  // element by element on lane 0 (the exact sequential scan).  The serial
  // scan over up to 4608 elements was ~40 % of the divide and conquer.
  if (tid < 64) {
    const int lane = tid;
    int q = 0, t = 0, r = 0;
    bool have = false;
    double pd = 0.0, pz = 0.0;
    int ps = 0;
    AS1 int* rp = M.rp + 2LL * lo;
    AS1 float* rcs = M.rcs + 2LL * lo;
    const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int base = 0; base < m; base += 64) {
      const int p = base + lane;
      const bool in = p < m;
      const double dp = in ? (double)sd2[p] : 0.0, zp = in ? (double)sz2[p] : 0.0;
      const int sp = in ? (int)ssrc2[p] : 0;
      const bool zdef = in && rho * fabs(zp) <= tol;
      const bool cand = in && !zdef;
      const unsigned long long cmask = __ballot(cand), dmask = __ballot(zdef);
      const unsigned long long prevc = cmask & below;
      const int pl = prevc ? 63 - __clzll(prevc) : 0;
      const double ppd = __shfl(dp, pl, 64), ppz = __shfl(zp, pl, 64);
      bool rot = false;
      if (cand && (prevc || have)) {
        const double qd = prevc ? ppd : pd, qz = prevc ? ppz : pz;
        rot = fabs((dp - qd) * zp * qz) <= tol * fma(zp, zp, qz * qz);
      }
      bool fast = use_fast && __ballot(rot) == 0ull;
      if (fast && dmask && t > 0) {
        const double fdv = __shfl(dp, __ffsll((long long)dmask) - 1, 64);
        fast = !((double)sdef[t - 1] > fdv);
      }
      if (fast) {
        const int kc = __popcll(cmask);
        if (kc > 0) {
          const int f0 = have ? 1 : 0;
          if (lane == 0 && have) { sd2[q] = pd; sz2[q] = pz; ssrc2[q] = ps; }
          const int rank = __popcll(prevc);
          if (cand && rank < kc - 1) {
            sd2[q + f0 + rank] = dp; sz2[q + f0 + rank] = zp; ssrc2[q + f0 + rank] = sp;
          }
          const int last = 63 - __clzll(cmask);
          pd = __shfl(dp, last, 64); pz = __shfl(zp, last, 64); ps = __shfl(sp, last, 64);
          q += f0 + kc - 1;
          have = true;
        }
        if (zdef) {
          const int dr = t + __popcll(dmask & below);
          sdef[dr] = dp;
          sdefsrc[dr] = sp & SRC_MASK;
        }
        t += __popcll(dmask);
        continue;
      }
      // exact sequential semantics for this chunk
      if (lane == 0) {
        const int pend = base + 64 < m ? base + 64 : m;
        for (int pp = base; pp < pend; ++pp) {
          const double ed = sd2[pp], ez = sz2[pp];
          const int es = ssrc2[pp];
          double dv = 0.0;
          int dsrc_v = -1;
          if (rho * fabs(ez) <= tol) {
            dv = ed; dsrc_v = es & SRC_MASK;
          } else if (!have) {
            have = true; pd = ed; pz = ez; ps = es;
            continue;
          } else {
            const double tt = ed - pd;
            // |tt c s| <= tol with c = ez / tau, s = -pz / tau, tau = hypot(ez, pz),
            // tested as |tt ez pz| <= tol (ez^2 + pz^2): the square root and the
            // divisions only when a rotation deflates (rare)
            if (fabs(tt * ez * pz) <= tol * fma(ez, ez, pz * pz)) {
              const double tau = hypot(ez, pz);
              const double c = ez / tau, sn = -pz / tau;
              rp[2 * r] = ps & SRC_MASK;
              rp[2 * r + 1] = es & SRC_MASK;
              rcs[2 * r] = (float)c;
              rcs[2 * r + 1] = (float)sn;
              ++r;
              dv = pd * c * c + ed * sn * sn;
              dsrc_v = ps & SRC_MASK;
              const int ta = ps >> TYP_SHIFT, tb = es >> TYP_SHIFT;
              const int typ = (ta == tb) ? tb : 2;
              pd = pd * sn * sn + ed * c * c;
              pz = tau;
              ps = (es & SRC_MASK) | (typ << TYP_SHIFT);
            } else {
              sd2[q] = pd; sz2[q] = pz; ssrc2[q] = ps; ++q;
              pd = ed; pz = ez; ps = es;
              continue;
            }
          }
          // insertion into the ascending deflated run
          int j = t;
          while (j > 0 && sdef[j - 1] > dv) {
            sdef[j] = sdef[j - 1];
            sdefsrc[j] = sdefsrc[j - 1];
            --j;
          }
          sdef[j] = dv;
          sdefsrc[j] = dsrc_v;
          ++t;
        }
      }
      q = __shfl(q, 0, 64); t = __shfl(t, 0, 64); r = __shfl(r, 0, 64);
      have = __shfl((int)have, 0, 64) != 0;
      pd = __shfl(pd, 0, 64); pz = __shfl(pz, 0, 64); ps = __shfl(ps, 0, 64);
    }
    if (lane == 0) {
      if (have) { sd2[q] = pd; sz2[q] = pz; ssrc2[q] = ps; ++q; }
      sh_k = q;
      sh_nrot = r;
      M.kk[lo] = q;
      M.nrot[lo] = r;
      M.rho[lo] = rho;
    }
  }
  __syncthreads();
  const int k = sh_k;
  // -- 5. type positions (type 1, then 2, then 3; ascending within a type)
  const int chunk = (k + 255) / 256;
  const int q0 = tid * chunk, q1 = (q0 + chunk < k) ? q0 + chunk : k;
  int c1 = 0, c2 = 0, c3 = 0;
  for (int q = q0; q < q1; ++q) {
    const int ty = ssrc2[q] >> TYP_SHIFT;
    c1 += ty == 1; c2 += ty == 2; c3 += ty == 3;
  }
  sh_cnt[0][tid] = c1; sh_cnt[1][tid] = c2; sh_cnt[2][tid] = c3;
  __syncthreads();
  if (tid == 0) {
    int s1 = 0, s2 = 0, s3 = 0;
    for (int x = 0; x < 256; ++x) {
      const int a = sh_cnt[0][x], b = sh_cnt[1][x], c = sh_cnt[2][x];
      sh_cnt[0][x] = s1; sh_cnt[1][x] = s2; sh_cnt[2][x] = s3;
      s1 += a; s2 += b; s3 += c;
    }
    // offsets of the types: t1 at 0, t2 at s1, t3 at s1 + s2
    red[0] = (double)s1;
    red[1] = (double)s2;
    M.k1a[lo] = s1;
    // GEMM records of this merge (host-set: lda/ldb/ldc, tiles, epi)
    const int K1 = s1, K2 = s2, k1al = K1 & ~3;
    PGemm* L = table + 2 * blockIdx.x;
    PGemm* R = L + 1;
    L->a_hi = L->a_lo = (const void*)(M.U + (long long)lo * ldw);
    L->b_hi = L->b_lo = (const void*)(M.ZpT + (long long)lo * ldw);
    L->c_hi = L->c_lo = (void*)(M.Zw + (long long)lo * ldw + lo);
    L->M = k; L->N = n1; L->K = K1 + K2;
    R->a_hi = R->a_lo = (const void*)(M.U + (long long)lo * ldw + k1al);
    R->b_hi = R->b_lo = (const void*)(M.ZpT + (long long)(lo + n1) * ldw + k1al);
    R->c_hi = R->c_lo = (void*)(M.Zw + (long long)lo * ldw + lo + n1);
    R->M = k; R->N = n2; R->K = k - k1al;
  }
  __syncthreads();
  const int off2 = (int)red[0], off3 = (int)red[0] + (int)red[1];
  int p1 = sh_cnt[0][tid], p2 = off2 + sh_cnt[1][tid], p3 = off3 + sh_cnt[2][tid];
  for (int q = q0; q < q1; ++q) {
    const int s = ssrc2[q];
    const int ty = s >> TYP_SHIFT;
    const int pos = (ty == 1) ? p1++ : (ty == 2) ? p2++ : p3++;
    M.typepos[lo + q] = pos;
    M.gsrc[lo + pos] = s & SRC_MASK;
    M.dl[lo + q] = sd2[q];
    M.wv[lo + q] = sz2[q];
  }
  for (int t = tid; t < m - k; t += 256) {
    M.defv[lo + t] = sdef[t];
    M.dsrc[lo + t] = sdefsrc[t];
  }
  };
  if (use_lds) {
    typedef __attribute__((address_space(3))) double lds_d;
    typedef __attribute__((address_space(3))) int lds_i;
    lds_d* sd = (lds_d*)dyn;
    lds_d* sz = sd + m;
    lds_d* sdef = sz + m;
    lds_i* ssrc = (lds_i*)(sdef + m);
    lds_i* sdefsrc = ssrc + m;
    body(sd, sz, sdef, ssrc, sdefsrc, sd, sz, ssrc, true);
  } else {
    body(M.dl + lo, M.wv + lo, M.gdef + lo, M.gsrcx + lo, M.gdefsrc + lo, M.gds + lo, M.gzs + lo,
         M.gsrcx + lo, false);
  }
}

// ------------------------------------------------------------------- rotate
__global__ __launch_bounds__(256) void dc_rotate_kernel(const DcMat* __restrict__ mats,
                                                        const DcNode* __restrict__ nodes) {
  const DcNode nd = nodes[blockIdx.y];
  const DcMat M = mats[nd.mat];
  const int lo = nd.lo, m = nd.hi - nd.lo;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int nr = M.nrot[lo];
  if (c >= m || nr == 0) return;
  const AS1 int* rp = M.rp + 2LL * lo;
  const AS1 float* rcs = M.rcs + 2LL * lo;
  AS1 float* base = M.Zw + (long long)lo * M.ldw + lo + c;
  for (int r = 0; r < nr; ++r) {
    const int p = rp[2 * r], q = rp[2 * r + 1];
    const float cs = rcs[2 * r], sn = rcs[2 * r + 1];
    AS1 float* xp = base + (long long)p * M.ldw;
    AS1 float* yp = base + (long long)q * M.ldw;
    const float x = *xp, y = *yp;
    *xp = cs * x + sn * y;
    *yp = cs * y - sn * x;
  }
}

// ------------------------------------------------------------------- gather
// blocks [0, tiles): 64 x 64 transposed tiles ZpT[c][j] = Z[src_j][c] (zero
// past k up to k + PADK); blocks [tiles, tiles + mmax): deflated row t -> U
// row k + t (full m columns).
__global__ __launch_bounds__(256) void dc_gather_kernel(const DcMat* __restrict__ mats,
                                                        const DcNode* __restrict__ nodes,
                                                        int tiles_c, int tiles) {
  __shared__ float tile[64][65];
  const DcNode nd = nodes[blockIdx.y];
  const DcMat M = mats[nd.mat];
  const int lo = nd.lo, m = nd.hi - nd.lo;
  const long long ldw = M.ldw;
  const int k = M.kk[lo];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= tiles) {
    const int t = b - tiles;
    if (t >= m - k) return;
    const int src = M.dsrc[lo + t];
    const AS1 float* s = M.Zw + (long long)(lo + (src < 0 ? 0 : src)) * ldw + lo;
    AS1 float* o = M.U + (long long)(lo + k + t) * ldw;
    for (int c = tid; c < m; c += 256) o[c] = s[c];
    return;
  }
  const int ct = b % tiles_c, jt = b / tiles_c;
  const int c0 = ct * 64, j0 = jt * 64;
  if (c0 >= m || j0 >= k + PADK) return;
  const int tx = tid & 63, ty = tid >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int j = j0 + r, c = c0 + tx;
    float v = 0.f;
    if (j < k && c < m) {
      const int src = M.gsrc[lo + j];
      v = M.Zw[(long long)(lo + src) * ldw + lo + c];
    }
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, j = j0 + tx;
    if (c < m && j < k + PADK) M.ZpT[(long long)(lo + c) * ldw + j] = tile[tx][r];
  }
}

// ------------------------------------------------------------------- secular
__device__ inline double quad_root(double qa, double qb, double qc, double tl, double th) {
  if (qa == 0.0) return qb != 0.0 ? -qc / qb : __builtin_nan("");
  double disc = qb * qb - 4.0 * qa * qc;
  if (disc < 0.0) disc = 0.0;
  const double sq = sqrt(disc);
  const double q = -0.5 * (qb + (qb >= 0.0 ? sq : -sq));
  const double r1 = q / qa;
  const double r2 = q != 0.0 ? qc / q : __builtin_nan("");
  if (tl < r1 && r1 < th) return r1;
  return r2;
}

__global__ __launch_bounds__(64 * RPB) void dc_secular_kernel(const DcMat* __restrict__ mats,
                                                               const DcNode* __restrict__ nodes,
                                                               int use_lds) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  const DcNode nd = nodes[blockIdx.y];
  const DcMat M = mats[nd.mat];
  const int lo = nd.lo, m = nd.hi - nd.lo;
  const long long ldw = M.ldw;
  const int k = M.kk[lo];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * RPB + wave;
  if (blockIdx.x * RPB >= m) return;   // uniform per block
  const AS1 double* Dg = M.dl + lo;
  const AS1 double* Wg = M.wv + lo;
  // the solve, templated on where D / W live (LDS or global): a pointer that
  // may be either compiles to flat_* loads in the innermost loop
  auto solve = [&](auto D, auto W) {
  if (i >= m) return;
  if (i >= k) {   // deflated row: U row (staged by the gather) -> Z row, its eigenvalue
    const AS1 float* s = M.U + (long long)(lo + i) * ldw;
    AS1 float* o = M.Zw + (long long)(lo + i) * ldw + lo;
    for (int c = lane; c < m; c += 64) o[c] = s[c];
    if (lane == 0) M.dval[lo + i] = M.defv[lo + i - k];
    return;
  }
  const double rho = M.rho[lo];
  int o;
  double tlo, thi;
  if (i < k - 1) {
    const double mid = 0.5 * (D[i + 1] - D[i]);
    const double Di = D[i];
    double f = 0.0;
    for (int q = lane; q < k; q += 64) f += rho * W[q] * W[q] / ((D[q] - Di) - mid);
    f = 1.0 + wave_sum_d(f);
    if (f >= 0.0) { o = i; tlo = 0.0; thi = mid; }
    else { o = i + 1; tlo = -mid; thi = 0.0; }
  } else {
    double s = 0.0;
    for (int q = lane; q < k; q += 64) s += rho * W[q] * W[q];
    o = k - 1; tlo = 0.0; thi = wave_sum_d(s);
  }
  const double Do = D[o];
  const int left = (o == i) ? o : o - 1;
  const int right = (left + 1 < k) ? left + 1 : -1;
  const double a = D[left] - Do;
  const double bpole = right >= 0 ? D[right] - Do : 0.0;
  double x = 0.5 * (tlo + thi);
  int it = 0;
  for (; it < MAX_IT; ++it) {
    double f = 0.0, fa = 0.0, psi = 0.0, dpsi = 0.0, phi = 0.0, dphi = 0.0;
    for (int q = lane; q < k; q += 64) {
      const double rden = 1.0 / ((D[q] - Do) - x);
      const double term = rho * W[q] * W[q] * rden;
      const double dterm = term * rden;
      f += term;
      fa += fabs(term);
      if (q <= left) { psi += term; dpsi += dterm; }
      else { phi += term; dphi += dterm; }
    }
    f = 1.0 + wave_sum_d(f);
    fa = wave_sum_d(fa);
    psi = wave_sum_d(psi);
    dpsi = wave_sum_d(dpsi);
    phi = wave_sum_d(phi);
    dphi = wave_sum_d(dphi);
    if (fabs(f) <= 16.0 * EPS64 * (1.0 + fa)) break;
    if (f < 0.0) tlo = x; else thi = x;
    if (thi - tlo <= 4.0 * EPS64 * fmax(fabs(tlo), fabs(thi))) break;
    const double B = dpsi * (a - x) * (a - x);
    const double A = psi - B / (a - x);
    double y;
    if (right >= 0) {
      const double E = dphi * (bpole - x) * (bpole - x);
      const double C = phi - E / (bpole - x);
      const double K = 1.0 + A + C;
      const double g = bpole - a;
      if (o == left) y = quad_root(K, -(K * g + B + E), B * g, 0.0, g);
      else y = quad_root(K, K * g - B - E, -E * g, -g, 0.0);
    } else {
      const double K = 1.0 + A;
      y = K > 0.0 ? a + B / K : __builtin_nan("");
    }
    const bool fin = isfinite(y);
    if (fin && fabs(y - x) <= 4.0 * EPS64 * fabs(x)) { x = y; break; }
    if (!fin || !(tlo < y && y < thi)) {
      if (tlo == 0.0) y = thi > 0.0 ? thi * 0.0625 : 0.5 * (tlo + thi);
      else if (thi == 0.0) y = tlo * 0.0625;
      else if (tlo > 0.0 && thi > 8.0 * tlo) y = sqrt(tlo * thi);
      else if (thi < 0.0 && tlo < 8.0 * thi) y = -sqrt(tlo * thi);
      else y = 0.5 * (tlo + thi);
    }
    x = y;
  }
  if (it == MAX_IT && lane == 0) atomicAdd((int*)M.info, 1);
  // eigenvector row i: u_q = w_q / (d_q - lambda), normalised, in type order
  double nrm = 0.0;
  for (int q = lane; q < k; q += 64) {
    const double u = W[q] / ((D[q] - Do) - x);
    nrm += u * u;
  }
  nrm = wave_sum_d(nrm);
  const double inv = nrm > 0.0 ? 1.0 / sqrt(nrm) : 0.0;
  AS1 float* urow = M.U + (long long)(lo + i) * ldw;
  const AS1 int* tp = M.typepos + lo;
  for (int q = lane; q < k; q += 64) {
    const double u = W[q] / ((D[q] - Do) - x);
    urow[tp[q]] = (float)(u * inv);
  }
  for (int q = k + lane; q < k + PADK; q += 64) urow[q] = 0.f;
  if (lane == 0) M.dval[lo + i] = Do + x;
  };
  if (use_lds) {
    typedef __attribute__((address_space(3))) double lds_double;
    lds_double* sD = (lds_double*)dyn;
    lds_double* sW = sD + k;
    for (int q = threadIdx.x; q < k; q += 64 * RPB) {
      sD[q] = Dg[q];
      sW[q] = Wg[q];
    }
    __syncthreads();
    solve((const lds_double*)sD, (const lds_double*)sW);
  } else {
    solve(Dg, Wg);
  }
}

// ------------------------------------------------------------------- final
__global__ __launch_bounds__(256) void dc_final_kernel(const DcMat* __restrict__ mats) {
  const DcMat M = mats[blockIdx.y];
  const int n = M.n, i = blockIdx.x;
  if (i >= n) return;
  __shared__ int sh_rank;
  if (threadIdx.x == 0) {
    const int k = M.kk[0];
    const double v = M.dval[i];
    int rank;
    if (i < k) rank = i + run_count(M.dval, k, n, v, false);
    else rank = (i - k) + run_count(M.dval, 0, k, v, true);
    rank = rank < 0 ? 0 : (rank >= n ? n - 1 : rank);
    M.dout[rank] = (float)v;
    sh_rank = rank;
  }
  __syncthreads();
  const AS1 float* s = M.Zw + (long long)i * M.ldw;
  AS1 float* o = M.Zout + (long long)sh_rank * M.ldz;
  for (int c = threadIdx.x; c < n; c += 256) o[c] = s[c];
}

// ------------------------------------------------------------------- host
struct DcLevel {
  int first, count;       // merges (device node table)
  int mmax;
  int tables_off;         // PGemm records (2 per merge)
  int gemm_tiles;
};

struct DcPlan {
  DcMat* d_mats = nullptr;
  DcNode* d_nodes = nullptr;
  PGemm* d_tables = nullptr;
  int nleaves = 0, nmats = 0, nmax = 0;
  std::vector<DcLevel> levels;
  hipGraphExec_t exec = nullptr;
};

struct HostNode { int lo, mid, hi, h; };

int build_tree(std::vector<HostNode>& out, int lo, int hi) {
  if (hi - lo <= LEAF) {
    out.push_back(HostNode{lo, -1, hi, 0});
    return 0;
  }
  const int mid = lo + (hi - lo) / 2;
  const int h1 = build_tree(out, lo, mid);
  const int h2 = build_tree(out, mid, hi);
  const int h = 1 + (h1 > h2 ? h1 : h2);
  out.push_back(HostNode{lo, mid, hi, h});
  return h;
}

size_t al256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace

// workspace layout per matrix (bytes): see carve()
// run-time switch of the deflation scan (eager launches; a captured plan keeps
// the mode it was captured with): 1 wave-parallel, 0 sequential
KFAC_API int kfac_dc_set_fast_scan(int on) {
  const int prev = g_dc_fast_scan;
  g_dc_fast_scan = on ? 1 : 0;
  return prev;
}

KFAC_API long long kfac_dc_ws_bytes(int n) {
  const long long ldw = rup(n + PADK, 64);
  size_t b = 0;
  b += 3 * al256((size_t)n * ldw * 4);      // Zw, ZpT, U
  b += 8 * al256((size_t)n * 8);            // dval dl wv defv rho gds gzs gdef
  b += 8 * al256((size_t)n * 4);            // kk k1a nrot typepos gsrc dsrc gsrcx gdefsrc
  b += al256((size_t)2 * n * 4);            // rp
  b += al256((size_t)2 * n * 4);            // rcs
  b += 256;                                 // info
  return (long long)b;
}

namespace {

DcMat carve(const float* d, const float* e, float* dout, float* Zout, long long ldz,
            unsigned char* ws, int n) {
  DcMat M;
  memset(&M, 0, sizeof(M));
  M.d = (const AS1 float*)d; M.e = (const AS1 float*)e;
  M.dout = (AS1 float*)dout; M.Zout = (AS1 float*)Zout; M.ldz = ldz; M.n = n;
  M.ldw = rup(n + PADK, 64);
  size_t off = 0;
  auto take = [&](size_t bytes) { unsigned char* p = ws + off; off += al256(bytes); return p; };
  const size_t mat = (size_t)n * M.ldw * 4;
  M.Zw = (AS1 float*)take(mat); M.ZpT = (AS1 float*)take(mat); M.U = (AS1 float*)take(mat);
  M.dval = (AS1 double*)take(n * 8); M.dl = (AS1 double*)take(n * 8);
  M.wv = (AS1 double*)take(n * 8); M.defv = (AS1 double*)take(n * 8);
  M.rho = (AS1 double*)take(n * 8); M.gds = (AS1 double*)take(n * 8);
  M.gzs = (AS1 double*)take(n * 8); M.gdef = (AS1 double*)take(n * 8);
  M.kk = (AS1 int*)take(n * 4); M.k1a = (AS1 int*)take(n * 4); M.nrot = (AS1 int*)take(n * 4);
  M.typepos = (AS1 int*)take(n * 4); M.gsrc = (AS1 int*)take(n * 4);
  M.dsrc = (AS1 int*)take(n * 4); M.gsrcx = (AS1 int*)take(n * 4);
  M.gdefsrc = (AS1 int*)take(n * 4);
  M.rp = (AS1 int*)take(2 * n * 4); M.rcs = (AS1 float*)take(2 * n * 4);
  M.info = (AS1 int*)take(4);
  return M;
}

std::mutex g_dc_mu;
std::map<std::string, DcPlan> g_dc_plans;

int build_plan(const std::vector<DcMat>& mats, DcPlan& P) {
  P.nmats = (int)mats.size();
  std::vector<DcNode> leaves;
  std::vector<std::vector<DcNode>> by_h;
  for (int mi = 0; mi < P.nmats; ++mi) {
    std::vector<HostNode> t;
    build_tree(t, 0, mats[mi].n);
    if (mats[mi].n > P.nmax) P.nmax = mats[mi].n;
    for (const HostNode& h : t) {
      const DcNode d{mi, h.lo, h.mid, h.hi};
      if (h.h == 0) {
        leaves.push_back(d);
      } else {
        if ((int)by_h.size() < h.h) by_h.resize(h.h);
        by_h[h.h - 1].push_back(d);
      }
    }
  }
  P.nleaves = (int)leaves.size();
  std::vector<DcNode> all = leaves;
  std::vector<PGemm> recs;
  for (auto& lv : by_h) {
    DcLevel L;
    L.first = (int)all.size();
    L.count = (int)lv.size();
    L.mmax = 0;
    L.tables_off = (int)recs.size();
    int tiles = 0;
    for (const DcNode& nd : lv) {
      const DcMat& M = mats[nd.mat];
      const int m = nd.hi - nd.lo, n1 = nd.mid - nd.lo, n2 = nd.hi - nd.mid;
      if (m > L.mmax) L.mmax = m;
      for (int side = 0; side < 2; ++side) {
        PGemm r;
        memset(&r, 0, sizeof(r));
        r.lda = M.ldw; r.ldb = M.ldw; r.ldc = M.ldw;
        r.M = 0; r.N = side ? n2 : n1; r.K = 0; r.epi = EPI_STORE;
        r.ea = r.eb = LP_QEXP;             // |U|, |ZpT| <= 1 (PREC_F16X3F)
        // placeholders until the prep kernel patches them (never read with M = 0)
        r.a_hi = r.a_lo = (const void*)M.U; r.b_hi = r.b_lo = (const void*)M.ZpT;
        r.c_hi = r.c_lo = (void*)M.Zw;
        r.tiles_n = cdiv(r.N, 128);
        r.tile_begin = tiles;
        tiles += cdiv(m, 128) * r.tiles_n;
        recs.push_back(r);
      }
      all.push_back(nd);
    }
    L.gemm_tiles = tiles;
    P.levels.push_back(L);
  }
  int err;
  if ((err = (int)hipMalloc(&P.d_mats, sizeof(DcMat) * mats.size()))) return err;
  if ((err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(DcMat) * mats.size(),
                            hipMemcpyHostToDevice)))
    return err;
  if ((err = (int)hipMalloc(&P.d_nodes, sizeof(DcNode) * (all.size() + 1)))) return err;
  if ((err = (int)hipMemcpy(P.d_nodes, all.data(), sizeof(DcNode) * all.size(),
                            hipMemcpyHostToDevice)))
    return err;
  if (!recs.empty()) {
    if ((err = (int)hipMalloc(&P.d_tables, sizeof(PGemm) * recs.size()))) return err;
    if ((err = (int)hipMemcpy(P.d_tables, recs.data(), sizeof(PGemm) * recs.size(),
                              hipMemcpyHostToDevice)))
      return err;
  }
  return 0;
}

int enqueue(const DcPlan& P, hipStream_t stream) {
  hipLaunchKernelGGL(dc_zero_kernel, dim3(256, P.nmats), dim3(256), 0, stream, P.d_mats);
  hipLaunchKernelGGL(dc_leaf_kernel, dim3(P.nleaves), dim3(256), 0, stream, P.d_mats, P.d_nodes);
  for (const DcLevel& L : P.levels) {
    const DcNode* nodes = P.d_nodes + L.first;
    PGemm* tab = P.d_tables + L.tables_off;
    const int prep_lds = L.mmax <= LDS_M_MAX;
    hipLaunchKernelGGL(dc_prep_kernel, dim3(L.count), dim3(256),
                       prep_lds ? (size_t)L.mmax * 32 : 0, stream, P.d_mats, nodes, tab, prep_lds,
                       g_dc_fast_scan);
    hipLaunchKernelGGL(dc_rotate_kernel, dim3(cdiv(L.mmax, 256), L.count), dim3(256), 0, stream,
                       P.d_mats, nodes);
    const int tiles_c = cdiv(L.mmax, 64), tiles_j = cdiv(L.mmax + PADK, 64);
    const int tiles = tiles_c * tiles_j;
    hipLaunchKernelGGL(dc_gather_kernel, dim3(tiles + L.mmax, L.count), dim3(256), 0, stream,
                       P.d_mats, nodes, tiles_c, tiles);
    const int sec_lds = L.mmax <= LDS_M_MAX;
    hipLaunchKernelGGL(dc_secular_kernel, dim3(cdiv(L.mmax, RPB), L.count), dim3(64 * RPB),
                       sec_lds ? (size_t)L.mmax * 16 : 0, stream, P.d_mats, nodes, sec_lds);
    int err = kfac_pgemm(g_dc_prec, TILE_F32, tab, 2 * L.count, L.gemm_tiles, nullptr, stream);
    if (err) return err;
  }
  hipLaunchKernelGGL(dc_final_kernel, dim3(P.nmax, P.nmats), dim3(256), 0, stream, P.d_mats);
  return (int)hipGetLastError();
}

}  // namespace

struct KfacDcRecord {
  const float* d; const float* e; float* dout; float* Zout; long long ldz;
  void* ws; long long n;
};

namespace {

// The plan of a record set (built and uploaded on first use) and, with
// `capture`, its instantiated graph (captured on a private non-blocking
// stream).  nullptr on failure (*err set).
DcPlan* plan_for(const KfacDcRecord* recs, int count, bool capture, int* err) {
  std::vector<DcMat> mats;
  for (int i = 0; i < count; ++i) {
    const KfacDcRecord& r = recs[i];
    if (r.n < 2 || r.n > SRC_MASK || (r.ldz & 3)) {
      *err = -2;
      return nullptr;
    }
    mats.push_back(carve(r.d, r.e, r.dout, r.Zout, r.ldz, (unsigned char*)r.ws, (int)r.n));
  }
  const std::string key((const char*)mats.data(), sizeof(DcMat) * mats.size());
  std::lock_guard<std::mutex> lk(g_dc_mu);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)dc_prep_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_M_MAX * 32);
    (void)hipFuncSetAttribute((const void*)dc_secular_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_M_MAX * 16);
    attr = true;
  }
  auto it = g_dc_plans.find(key);
  if (it == g_dc_plans.end()) {
    DcPlan P;
    if ((*err = build_plan(mats, P)) != 0) return nullptr;
    it = g_dc_plans.emplace(key, P).first;
  }
  DcPlan* plan = &it->second;
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

// Eigen-decompose `count` symmetric tridiagonal matrices (d, e: n floats each,
// e[i] couples rows i, i+1).  Output: dout ascending, Zout row k = eigenvector
// k (ldz floats per row).  ws: kfac_dc_ws_bytes(n) bytes per matrix.  The
// launch sequence for a record set is built once, captured into a hipGraph
// (use_graph) and replayed.
KFAC_API int kfac_dc_batched(const KfacDcRecord* recs, int count, int use_graph,
                             hipStream_t stream) {
  if (count <= 0) return 0;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cs == hipStreamCaptureStatusNone;
  int err = 0;
  DcPlan* plan = plan_for(recs, count, graph, &err);
  if (!plan) return err ? err : -4;
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}

// Build (upload + capture) the plan of a record set without running it: call
// before concurrent solves start (a capture must not overlap other threads'
// library calls).
KFAC_API int kfac_dc_prepare(const KfacDcRecord* recs, int count) {
  int err = 0;
  return plan_for(recs, count, true, &err) ? 0 : (err ? err : -4);
}

// info (device int, per matrix): secular roots that hit the iteration cap.
KFAC_API int kfac_dc_info_offset(int n) {
  const long long ldw = rup(n + PADK, 64);
  size_t b = 3 * al256((size_t)n * ldw * 4) + 8 * al256((size_t)n * 8) +
             8 * al256((size_t)n * 4) + 2 * al256((size_t)2 * n * 4);
  return (int)b;
}
