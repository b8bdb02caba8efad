// Batched compact-WY back-transformation of the hand-written tridiagonal
// eigensolver (reference semantics kfac/layers/utils.py:45-74:
// the eigenvectors of a symmetric factor, eigenvalues ascending).
//
// Stage 3 of ops/eigen.py's fused path: after the ragged tridiagonal
// reduction (csrc/eig_reduce.hip) and the batched divide and conquer
// (csrc/eig_dc.hip), Z (eigenvectors of the tridiagonal matrices) becomes
// Q Z.  Every GEMM is the grouped MFMA kernel of csrc/precond_gemm.hip; no
// vendor library is linked.
#include "pgemm.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

// ---------------------------------------------------------------------------
// Batched blocked back-transformation Z <- Q Z for the hand-written reduction
// (round 1 called rocSOLVER ormtr per matrix: 13 ms at n = 4608).
// Q = H_0 H_1 ... H_{n-2} is applied as compact-WY blocks of BT reflectors,
// last block first:  Z[j0:, :] -= V_k (T_k (V_k^T Z[j0:, :])).  Every GEMM is
// the grouped MFMA kernel of csrc/precond_gemm.hip (exact f32 MFMA) over all
// matrices of the size class; the long-K product V_k^T Z is split over K
// into per-chunk slabs summed in a fixed order by a small reduction kernel
// (bitwise reproducible; round 3 accumulated the chunks with f32 atomics).
// The whole sequence (~6 launches per block) is
// captured once per buffer set into a hipGraph (no library GEMM, nothing on
// the legacy stream).
//
// Layouts (all fp32): A row j = reflector j (made explicit: zeros up to j, 1
// at j+1); Z column-major (row `col` of the row-major view = eigenvector
// `col`); lda = ldz a multiple of 64 with zero padding past n, so every GEMM
// operand is k-contiguous and zero-padded to the kernel's 64-wide k-steps.
//   S1  W1t_s[col][c] = sum_{i in chunk s} Z[col][i] V_k[c][i]   (split-K slabs)
//   R   W1t = ((W1t_0 + W1t_1) + W1t_2) + ...                  (fixed order, in slab 0)
//   S2  W2t[col][c] = sum_c' W1t[col][c'] T_k[c][c']
//   S3  Z[col][j0+i] -= sum_c W2t[col][c] Vt_k[i][c]       (Vt_k = V_k^T copy)
namespace {

// reflectors per block: 256 (round 5; 128 before): each block is one pass
// over Z for its update and one for V_k^T Z, so the block width halves the
// Z traffic of the sequence, and the Z update's k-loop doubles.  T_k is
// built from its two 128-row halves (larft_kernel) and their coupling
// (t_merge_kernel).
constexpr int BT = 256;
constexpr int LB = 128;       // larft sub-block
constexpr int KCH = 512;      // split-K chunk of S1
constexpr int TILE_F32 = 0;   // pgemm 128 x 128 fp32, 4 waves (best since round 2: profiles/r2_pgemm_sweep.log)
// GEMM precision of the back-transformation: bf16x6 on the fp32 operands
// (PREC_BF16X6F: six bf16 MFMA products, fp32-level error, at the bf16 MFMA
// rate) unless KFAC_EIG_GEMM=fp32 (exact f32 MFMA)
const int g_bt_prec = [] {
  const char* e = getenv("KFAC_EIG_GEMM");
  return (e && !strcmp(e, "fp32")) ? (int)PREC_F32 : (int)PREC_BF16X6F;
}();
// the products whose operands are bounded by 1 -- G_k = V_k V_k^T and
// W1 = Z^T V_k (reflector entries |v| <= 1, eigenvector entries |z| <= 1) --
// run fp16x3 with a fixed 2^14 scale (PREC_F16X3F) unless KFAC_EIG_GEMM
// names bf16x6 / fp32; T_k (S2) and the update with W2 (S3) keep bf16x6
const int g_bt_prec_bounded = [] {
  const char* e = getenv("KFAC_EIG_GEMM");
  if (e && !strcmp(e, "fp32")) return (int)PREC_F32;
  if (e && !strcmp(e, "bf16x6")) return (int)PREC_BF16X6F;
  return (int)PREC_F16X3F;
}();

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// split-K slabs per matrix (the most any block needs: K = lda - j0 <= lda)
inline int nslab(int lda) { return cdiv(lda, KCH); }

// R: slab 0 of every matrix <- the sum of its first `ns` slabs, in slab order
__global__ __launch_bounds__(256) void slab_sum_kernel(float4* W1, long long slab4, int nsl,
                                                       int ns) {
  float4* base = W1 + (long long)blockIdx.y * nsl * slab4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < slab4; i += (long long)gridDim.x * 256) {
    float4 acc = base[i];
    for (int s = 1; s < ns; ++s) {
      const float4 x = base[(long long)s * slab4 + i];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    base[i] = acc;
  }
}

// Zero fill as a kernel (captured memset nodes misbehaved for multi-matrix
// batches on ROCm 7.2).
__global__ __launch_bounds__(256) void zero_kernel(float4* p, long long n4) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
    p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Row j of the reduced matrix (== reflector j in column-major) made explicit:
// zeros up to j, the implicit 1 at j+shift (shift 1: tridiagonalisation),
// v[1:] after.
__global__ __launch_bounds__(256) void make_v_kernel(float* A, int lda, long long sA, int n,
                                                     int shift) {
  float* row = A + blockIdx.y * sA + (long long)blockIdx.x * lda;
  const int j = blockIdx.x;
  for (int i = threadIdx.x; i <= j + shift && i < n; i += 256) row[i] = (i == j + shift) ? 1.f : 0.f;
}

// The two diagonal LB x LB sub-blocks of T_k (upper triangular, ROW-major
// BT x BT, zero beyond kb) from G_k = V_k V_k^T (row-major, ld BT) and tau
// (LAPACK larft, forward / columnwise), one workgroup per sub-block.  larft's column recursion T(0:i, i) = -tau_i T(0:i, 0:i)
// G(0:i, i) is BT dependent steps (~320 us per launch at BT = 128,
// profiles/r3_eig_kernel_stats.csv); the same T is the inverse of the upper
// triangular U = diag(1 / tau) + striu(G), computed here by recursive
// doubling: T12 = -T11 U12 T22 for diagonal blocks of 1, 2, 4, .. 64 --
// seven levels of two small products, all 256 threads busy.  A reflector
// with tau = 0 (H_i = I) has row and column i of T zero: its row / column of
// U is decoupled (U_ii = 1) and zeroed in T afterwards.
constexpr int LT = 256;   // larft threads
__global__ __launch_bounds__(LT) void larft_kernel(const float* G, float* T, const float* tau,
                                                   int n, int nblk) {
  __shared__ float sU[LB][LB + 1];
  __shared__ float sT[LB][LB + 1];
  __shared__ float sW[LB / 2][LB / 2 + 1];
  __shared__ int live[LB];
  const int k = blockIdx.x / (BT / LB), sb = blockIdx.x % (BT / LB);
  const int mat = blockIdx.y, tid = threadIdx.x;
  // sub-block sb: rows / columns sb LB .. sb LB + LB - 1 of block k
  const long long off = ((long long)mat * nblk + k) * BT * BT + (long long)sb * LB * (BT + 1);
  const int j0 = k * BT + sb * LB;
  const int kb = (n - j0) < LB ? (n - j0 > 0 ? n - j0 : 0) : LB;
  const float* tj = tau + (long long)mat * n + j0;
  for (int r = tid; r < LB; r += LT) live[r] = (r < kb) && (tj[r] != 0.f);
  __syncthreads();
  for (int e = tid; e < LB * LB; e += LT) {
    const int r = e / LB, c = e % LB;
    float u = 0.f;
    if (r == c) u = live[r] ? 1.f / tj[r] : 1.f;
    else if (c > r && live[r] && live[c]) u = G[off + (long long)r * BT + c];
    sU[r][c] = u;
    sT[r][c] = (r == c) ? 1.f / u : 0.f;
  }
  __syncthreads();
  for (int b = 1; b < LB; b *= 2) {
    const int pairs = LB / (2 * b), per = b * b;
    // W = U12 T22 for every pair (U12: rows p0 .. p0+b, cols p0+b .. p0+2b)
    for (int e = tid; e < pairs * per; e += LT) {
      const int p = e / per, w = e % per, r = w / b, c = w % b;
      const int p0 = 2 * p * b;
      float acc = 0.f;
      for (int q = 0; q <= c; ++q) acc = fmaf(sU[p0 + r][p0 + b + q], sT[p0 + b + q][p0 + b + c], acc);
      sW[(p * b + r) % (LB / 2)][c] = acc;
    }
    __syncthreads();
    // T12 = -T11 W
    for (int e = tid; e < pairs * per; e += LT) {
      const int p = e / per, w = e % per, r = w / b, c = w % b;
      const int p0 = 2 * p * b;
      float acc = 0.f;
      for (int q = r; q < b; ++q) acc = fmaf(sT[p0 + r][p0 + q], sW[(p * b + q) % (LB / 2)][c], acc);
      sT[p0 + r][p0 + b + c] = -acc;
    }
    __syncthreads();
  }
  for (int e = tid; e < LB * LB; e += LT) {
    const int r = e / LB, c = e % LB;
    T[off + (long long)r * BT + c] = (live[r] && live[c]) ? sT[r][c] : 0.f;
  }
}

// The coupling of T_k's two halves: T = U^-1 for the block upper-triangular
// U = [U11 U12; 0 U22] with U12 = G12 (the strict upper part of G_k), so
// T12 = -T11 G12 T22, and T21 = 0.  One workgroup per block, operands in LDS,
// 8 x 8 outputs per thread: W = G12 T22, then T12 = -T11 W.  Full-length
// k-loops: T22 (T11) is zero below (left of) its diagonal, and dead rows /
// columns of T11 / T22 are zero already, so the extra terms add exact zeros
// (the sums are those of the triangular loops, bit for bit).  A first
// version reading T22 from memory inside a triangular loop took 371 us per
// 3 x 4608 back-transformation.
__global__ __launch_bounds__(256) void t_merge_kernel(const float* G, float* T, int nblk) {
  __shared__ float s0[LB][LB + 1];
  __shared__ float s1[LB][LB + 1];
  const int k = blockIdx.x, mat = blockIdx.y, tid = threadIdx.x;
  const long long off = ((long long)mat * nblk + k) * BT * BT;
  const float* G12 = G + off + LB;                        // rows 0.., columns LB..
  const float* T11 = T + off;
  const float* T22 = T + off + (long long)LB * BT + LB;
  float* T12 = T + off + LB;
  for (int e = tid; e < LB * LB; e += 256) {
    const int r = e / LB, c = e % LB;
    s0[r][c] = G12[(long long)r * BT + c];
    s1[r][c] = T22[(long long)r * BT + c];
  }
  __syncthreads();
  const int ty = tid >> 4, tx = tid & 15;                 // rows ty + 16 i, columns tx + 16 j
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc[i][jj] = 0.f;
  for (int q = 0; q < LB; ++q) {
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = s0[ty + 16 * i][q];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) b[jj] = s1[q][tx + 16 * jj];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc[i][jj] = fmaf(a[i], b[jj], acc[i][jj]);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) s0[ty + 16 * i][tx + 16 * jj] = acc[i][jj];   // W
  for (int e = tid; e < LB * LB; e += 256) {
    const int r = e / LB, c = e % LB;
    s1[r][c] = T11[(long long)r * BT + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc[i][jj] = 0.f;
  for (int p = 0; p < LB; ++p) {
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = s1[ty + 16 * i][p];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) b[jj] = s0[p][tx + 16 * jj];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc[i][jj] = fmaf(a[i], b[jj], acc[i][jj]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
      T12[(long long)(ty + 16 * i) * BT + tx + 16 * jj] = -acc[i][jj];
}

struct BtArgs {
  float* A; int lda; long long sA; const float* tau; float* Z; int ldz; long long sZ; int n;
  int batch; float* Tbuf; float* W1; float* W2; float* Vt; int shift;
};

// One recorded operation of the back-transformation.
struct BtOp {
  int kind;              // 0 pgemm, 1 split copy, 2 memset, 3 make_v, 4 larft, 5 slab sum (count = slabs),
                         // 6 pgemm of bounded operands (g_bt_prec_bounded)
  size_t off; int count; int tiles;    // table offset (bytes) / records / tiles
  void* ptr; size_t bytes;             // memset
};

struct BtPlan {
  std::vector<BtOp> ops;
  void* tables = nullptr;
  hipGraphExec_t exec = nullptr;
};

void add_pgemm(std::vector<unsigned char>& host, std::vector<BtOp>& ops, std::vector<PGemm>& recs,
               bool bounded = false) {
  int tiles = 0;
  for (auto& r : recs) {
    r.tiles_n = cdiv(r.N, 128);
    r.tile_begin = tiles;
    tiles += cdiv(r.M, 128) * r.tiles_n;
    if (bounded) r.ea = r.eb = LP_QEXP;
  }
  BtOp op{bounded ? 6 : 0, host.size(), (int)recs.size(), tiles, nullptr, 0};
  const unsigned char* p = (const unsigned char*)recs.data();
  host.insert(host.end(), p, p + recs.size() * sizeof(PGemm));
  while (host.size() % 256) host.push_back(0);
  ops.push_back(op);
  recs.clear();
}

PGemm rec(const float* a, long long lda, const float* b, long long ldb, float* c, long long ldc,
          int M, int N, int K, int epi) {
  PGemm r;
  memset(&r, 0, sizeof(r));
  r.a_hi = r.a_lo = a; r.lda = lda;
  r.b_hi = r.b_lo = b; r.ldb = ldb;
  r.c_hi = r.c_lo = c; r.ldc = ldc;
  r.M = M; r.N = N; r.K = K; r.epi = epi;
  return r;
}

// Host-side plan: the op list and every GEMM / copy table of the sequence.
void build_plan(const BtArgs& a, BtPlan& plan, std::vector<unsigned char>& host) {
  const int n = a.n, b = a.batch, nblk = cdiv(n, BT);
  const long long tstride = (long long)nblk * BT * BT;
  float* G = a.Tbuf;
  float* T = a.Tbuf + tstride * b;
  const long long w1s = (long long)n * BT, vts = (long long)a.lda * BT;
  std::vector<PGemm> recs;
  plan.ops.push_back(BtOp{3, 0, 0, 0, nullptr, 0});
  // G_k = V_k V_k^T for every block of every matrix (one grouped launch)
  for (int m = 0; m < b; ++m)
    for (int k = 0; k < nblk; ++k) {
      const int j0 = k * BT, kb = n - j0 < BT ? n - j0 : BT;
      const float* Vk = a.A + m * a.sA + (long long)j0 * a.lda + j0;
      recs.push_back(rec(Vk, a.lda, Vk, a.lda, G + m * tstride + (long long)k * BT * BT, BT, kb,
                         kb, a.lda - j0, EPI_STORE));
    }
  add_pgemm(host, plan.ops, recs, true);
  plan.ops.push_back(BtOp{4, 0, 0, 0, nullptr, 0});
  for (int k = nblk - 1; k >= 0; --k) {
    const int j0 = k * BT, kb = n - j0 < BT ? n - j0 : BT, Kn = a.lda - j0;
    if (kb < BT) {   // partial block: stale columns >= kb must read as zero
      plan.ops.push_back(BtOp{2, 0, 0, 0, a.W2, (size_t)b * w1s * 4});
      plan.ops.push_back(BtOp{2, 0, 0, 0, a.Vt, (size_t)b * vts * 4});
      plan.ops.push_back(BtOp{2, 0, 0, 0, a.W1, (size_t)b * nslab(a.lda) * w1s * 4});
    }
    const int ns = cdiv(Kn, KCH), nsl = nslab(a.lda);
    for (int m = 0; m < b; ++m) {
      const float* Zm = a.Z + m * a.sZ;
      const float* Vk = a.A + m * a.sA + (long long)j0 * a.lda;
      for (int s = 0; s < ns; ++s) {
        const int k0 = s * KCH, kc = Kn - k0 < KCH ? Kn - k0 : KCH;
        recs.push_back(rec(Zm + j0 + k0, a.ldz, Vk + j0 + k0, a.lda,
                           a.W1 + ((long long)m * nsl + s) * w1s, BT, n, kb, kc, EPI_STORE));
      }
    }
    add_pgemm(host, plan.ops, recs, true);
    if (ns > 1) plan.ops.push_back(BtOp{5, 0, ns, 0, nullptr, 0});
    for (int m = 0; m < b; ++m)
      recs.push_back(rec(a.W1 + (long long)m * nsl * w1s, BT, T + m * tstride + (long long)k * BT * BT, BT,
                         a.W2 + m * w1s, BT, n, kb, BT, EPI_STORE));
    add_pgemm(host, plan.ops, recs);
    {  // Vt_k = V_k^T (rows j0.., kb columns)
      std::vector<SplitJob> jobs(b);
      int tiles = 0;
      for (int m = 0; m < b; ++m) {
        SplitJob& J = jobs[m];
        J.src = a.A + m * a.sA + (long long)j0 * a.lda + j0; J.lds = a.lda;
        J.o_hi = J.o_lo = a.Vt + m * vts; J.ldo = BT;
        J.rows = kb; J.cols = n - j0; J.trans = 1;
        J.tiles_c = cdiv(J.cols, 64); J.tile_begin = tiles;
        tiles += cdiv(J.rows, 64) * J.tiles_c;
      }
      BtOp op{1, host.size(), b, tiles, nullptr, 0};
      const unsigned char* p = (const unsigned char*)jobs.data();
      host.insert(host.end(), p, p + jobs.size() * sizeof(SplitJob));
      while (host.size() % 256) host.push_back(0);
      plan.ops.push_back(op);
    }
    for (int m = 0; m < b; ++m)
      recs.push_back(rec(a.W2 + m * w1s, BT, a.Vt + m * vts, BT, a.Z + m * a.sZ + j0, a.ldz, n,
                         n - j0, BT, EPI_SUB));
    add_pgemm(host, plan.ops, recs);
  }
}

int run_plan(const BtArgs& a, const BtPlan& plan, hipStream_t stream) {
  const int nblk = cdiv(a.n, BT);
  const long long tstride = (long long)nblk * BT * BT;
  for (const BtOp& op : plan.ops) {
    int err = 0;
    const unsigned char* t = (const unsigned char*)plan.tables + op.off;
    switch (op.kind) {
      case 0: err = kfac_pgemm(g_bt_prec, TILE_F32, t, op.count, op.tiles, nullptr, stream); break;
      case 6:
        err = kfac_pgemm(g_bt_prec_bounded, TILE_F32, t, op.count, op.tiles, nullptr, stream);
        break;
      case 1: err = kfac_split_copy(PREC_F32, t, op.count, op.tiles, stream); break;
      case 2: {
        const long long n4 = (long long)(op.bytes / 16);
        const int grid = (int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048);
        hipLaunchKernelGGL(zero_kernel, dim3(grid), dim3(256), 0, stream, (float4*)op.ptr, n4);
        err = (int)hipGetLastError();
        break;
      }
      case 5: {
        const long long slab4 = (long long)a.n * BT / 4;
        const int grid = (int)((slab4 + 255) / 256 < 1024 ? (slab4 + 255) / 256 : 1024);
        hipLaunchKernelGGL(slab_sum_kernel, dim3(grid, a.batch), dim3(256), 0, stream,
                           (float4*)a.W1, slab4, nslab(a.lda), op.count);
        err = (int)hipGetLastError();
        break;
      }
      case 3:
        hipLaunchKernelGGL(make_v_kernel, dim3(a.n, a.batch), dim3(256), 0, stream, a.A, a.lda,
                           a.sA, a.n, a.shift);
        err = (int)hipGetLastError();
        break;
      default:
        hipLaunchKernelGGL(larft_kernel, dim3(nblk * (BT / LB), a.batch), dim3(LT), 0, stream,
                           a.Tbuf, a.Tbuf + tstride * a.batch, a.tau, a.n, nblk);
        hipLaunchKernelGGL(t_merge_kernel, dim3(nblk, a.batch), dim3(256), 0, stream, a.Tbuf,
                           a.Tbuf + tstride * a.batch, nblk);
        err = (int)hipGetLastError();
    }
    if (err) return err;
  }
  return 0;
}

typedef std::tuple<float*, float*, int, int, float*, float*, float*, float*, int> BtKey;
std::mutex g_bt_mu;
std::map<BtKey, BtPlan> g_bt;

// The plan (tables uploaded, graph captured on a private non-blocking
// stream) of this buffer set; built on first use.  Call it from one thread
// while no other thread issues library work (kfac_backtransform_prepare).
BtPlan* plan_for(const BtArgs& a, int* err) {
  const BtKey key(a.A, a.Z, a.n, a.batch, a.Tbuf, a.W1, a.W2, a.Vt, a.shift);
  std::lock_guard<std::mutex> lk(g_bt_mu);
  auto it = g_bt.find(key);
  if (it != g_bt.end()) return &it->second;
  BtPlan plan;
  std::vector<unsigned char> host;
  build_plan(a, plan, host);
  if ((*err = (int)hipMalloc(&plan.tables, host.size())) != 0) return nullptr;
  if ((*err = (int)hipMemcpy(plan.tables, host.data(), host.size(), hipMemcpyHostToDevice)) != 0)
    return nullptr;
  static hipStream_t cap = nullptr;
  if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
  if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
    hipGraph_t graph = nullptr;
    const int e1 = run_plan(a, plan, cap);
    const hipError_t e2 = hipStreamEndCapture(cap, &graph);
    if (!e1 && e2 == hipSuccess && graph &&
        hipGraphInstantiate(&plan.exec, graph, nullptr, nullptr, 0) != hipSuccess)
      plan.exec = nullptr;
    if (graph) hipGraphDestroy(graph);
  }
  (void)hipGetLastError();
  return &(g_bt[key] = plan);
}

}  // namespace

// A: the reduced matrices (reflectors in rows, made explicit in place),
// Z: tridiagonal eigenvectors (column-major, ldz) -> eigenvectors of A.
// lda == ldz, a multiple of 64 (zero padding past n).  Tbuf: 2 x batch x
// nblk x BT x BT, W1: batch x kfac_backtransform_slabs(lda) x n x BT, W2: batch
// x n x BT, Vt: batch x lda x BT.
KFAC_API int kfac_tridiag_backtransform(float* A, int lda, long long strideA, const float* tau,
                                        float* Z, int ldz, long long strideZ, int n, int batch,
                                        float* Tbuf, float* W1, float* W2, float* Vt,
                                        int use_graph, hipStream_t stream) {
  if (lda % 64 || ldz % 64 || lda != ldz || n < 2) return -2;
  const BtArgs a{A, lda, strideA, tau, Z, ldz, strideZ, n, batch, Tbuf, W1, W2, Vt, 1};
  int err = 0;
  BtPlan* plan = plan_for(a, &err);
  if (!plan) return err ? err : -4;
  if (use_graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return run_plan(a, *plan, stream);
}

// The same for the two-stage solver's stage 1 (csrc/eig_sy2sb.hip): reflector
// j has its implicit 1 at column j + shift (shift = the band's half-bandwidth)
KFAC_API int kfac_band_backtransform(float* A, int lda, long long strideA, const float* tau,
                                     float* Z, int ldz, long long strideZ, int n, int batch,
                                     float* Tbuf, float* W1, float* W2, float* Vt, int shift,
                                     int use_graph, hipStream_t stream) {
  if (lda % 64 || ldz % 64 || lda != ldz || n < 2 || shift < 1) return -2;
  const BtArgs a{A, lda, strideA, tau, Z, ldz, strideZ, n, batch, Tbuf, W1, W2, Vt, shift};
  int err = 0;
  BtPlan* plan = plan_for(a, &err);
  if (!plan) return err ? err : -4;
  if (use_graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return run_plan(a, *plan, stream);
}

KFAC_API int kfac_backtransform_slabs(int lda) { return nslab(lda); }
KFAC_API int kfac_backtransform_block() { return BT; }

KFAC_API int kfac_backtransform_prepare(float* A, int lda, long long strideA, const float* tau,
                                        float* Z, int ldz, long long strideZ, int n, int batch,
                                        float* Tbuf, float* W1, float* W2, float* Vt) {
  if (lda % 64 || ldz % 64 || lda != ldz || n < 2) return -2;
  const BtArgs a{A, lda, strideA, tau, Z, ldz, strideZ, n, batch, Tbuf, W1, W2, Vt, 1};
  int err = 0;
  return plan_for(a, &err) ? 0 : (err ? err : -4);
}
