// Preconditioning epilogue kernels for gfx950.
//
//   outer_recip     K7: dGdA[i][j] = 1 / (dG[i] * dA[j] + damping)
//                   (reference kfac/layers/base.py:300-306)
//   hadamard        K8 middle step, in place on v1 (nG x nA, f32):
//                   mode 0: v1 *= dGdA ; mode 1: v1 /= (dG[i]*dA[j] + damping)
//                   (reference kfac/layers/base.py:459-470)
//   grouped_kl_dot  K10: vg = sum over ALL layers of <v, g>: one launch writes a
//                   f64 partial per workgroup, kl_finalize sums them in a fixed
//                   order -- deterministic, so every data-parallel rank derives
//                   the bit-identical clip scale (the reference does one .item()
//                   per layer: kfac/preconditioner.py:661-682).
//   grouped_apply   K11: g = nu * v for ALL layers in ONE launch, where nu is
//                   computed on the device from vg (no host sync):
//                   nu = vg==0 ? 1 : min(1, sqrt(kl_clip / |vg * lr^2|)).
//                   (reference kfac/layers/base.py:419-430,477-483; the .grad
//                   tensors are written in place so DDP bucket views survive)
// Descriptor tables travel by value in the kernel arguments (< 4 KB), so a
// table can be rebuilt every step without any H2D copy.
#include "common.h"
#include "devtable.h"

namespace {

constexpr int MAXG = 40;

// v: (rows x cols) f32 with row stride ldv.  g: the parameter's .grad in ANY
// memory layout: column `col` of the K-FAC matrix is (c, i, j) =
// (col / kk, (col % kk) / kw, col % kw) -> element r*gs0 + c*gs1 + i*gs2 + j*gs3
// (conv weights in channels_last, linear weights, bias vectors alike).
struct Mat2D {
  const float* v;
  void* g;
  long long gs0, gs1, gs2, gs3;
  int ldv;
  int rows, cols;
  int gdtype;
  int kk, kw;
};

struct GroupTable {
  int count;
  int block_prefix[MAXG + 1];   // exclusive prefix sum of blocks per entry
  Mat2D m[MAXG];
};

constexpr int ELEMS_PER_BLOCK = 256 * 8;

__device__ __forceinline__ int find_entry(const GroupTable& t, int blk) {
  int lo = 0, hi = t.count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t.block_prefix[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ long long g_index(const Mat2D& m, int r, int col) {
  int c = col / m.kk;
  int rem = col - c * m.kk;
  int i = rem / m.kw;
  int j = rem - i * m.kw;
  return (long long)r * m.gs0 + (long long)c * m.gs1 + (long long)i * m.gs2 + (long long)j * m.gs3;
}

__device__ __forceinline__ void part_out(double* part, int i, double v) { part[i] = v; }

__device__ __forceinline__ float load_g(const Mat2D& m, long long idx) {
  if (m.gdtype == KDT_F32) return ((const float*)m.g)[idx];
  if (m.gdtype == KDT_BF16) return bf16_bits_to_f32(((const uint16_t*)m.g)[idx]);
  return f16_bits_to_f32(((const uint16_t*)m.g)[idx]);
}

__device__ __forceinline__ void store_g(const Mat2D& m, long long idx, float v) {
  if (m.gdtype == KDT_F32) ((float*)m.g)[idx] = v;
  else if (m.gdtype == KDT_BF16) ((uint16_t*)m.g)[idx] = f32_to_bf16_bits(v);
  else ((uint16_t*)m.g)[idx] = f32_to_f16_bits(v);
}

__global__ __launch_bounds__(256) void grouped_kl_dot_kernel(const GroupTable* __restrict__ tp,
                                                             double* part) {
  const GroupTable& t = *tp;
  const int e = find_entry(t, blockIdx.x);
  const Mat2D m = t.m[e];
  const long long n = (long long)m.rows * m.cols;
  const long long start = (long long)(blockIdx.x - t.block_prefix[e]) * ELEMS_PER_BLOCK;
  float acc = 0.f;
  for (long long i = start + threadIdx.x; i < n && i < start + ELEMS_PER_BLOCK; i += 256) {
    int r = (int)(i / m.cols), c = (int)(i - (long long)r * m.cols);
    acc += m.v[(long long)r * m.ldv + c] * load_g(m, g_index(m, r, c));
  }
  double d = wave_reduce_sum_d((double)acc);
  __shared__ double part4[4];
  if ((threadIdx.x & 63) == 0) part4[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) part_out(part, blockIdx.x, part4[0] + part4[1] + part4[2] + part4[3]);
}

__global__ __launch_bounds__(256) void grouped_apply_kernel(const GroupTable* __restrict__ tp,
                                                            const double* vg,
                                                            double lr2, double kl_clip,
                                                            int use_clip) {
  const GroupTable& t = *tp;
  float nu = 1.f;
  if (use_clip) {
    double s = (*vg) * lr2;
    if (s != 0.0) {
      double q = sqrt(kl_clip / fabs(s));
      nu = (float)(q < 1.0 ? q : 1.0);
    }
  }
  const int e = find_entry(t, blockIdx.x);
  const Mat2D m = t.m[e];
  const long long n = (long long)m.rows * m.cols;
  const long long start = (long long)(blockIdx.x - t.block_prefix[e]) * ELEMS_PER_BLOCK;
  for (long long i = start + threadIdx.x; i < n && i < start + ELEMS_PER_BLOCK; i += 256) {
    int r = (int)(i / m.cols), c = (int)(i - (long long)r * m.cols);
    store_g(m, g_index(m, r, c), nu * m.v[(long long)r * m.ldv + c]);
  }
}

__global__ __launch_bounds__(256) void outer_recip_kernel(const float* __restrict__ dG,
                                                          const float* __restrict__ dA,
                                                          float* __restrict__ out, int nG, int nA,
                                                          float damping) {
  const int i = blockIdx.y;
  const float g = dG[i];
  for (int j = blockIdx.x * 256 + threadIdx.x; j < nA; j += gridDim.x * 256)
    out[(long long)i * nA + j] = 1.0f / (g * dA[j] + damping);
}

__global__ __launch_bounds__(256) void hadamard_kernel(float* __restrict__ v, int ldv,
                                                       const float* __restrict__ dGdA,
                                                       const float* __restrict__ dG,
                                                       const float* __restrict__ dA, int nG,
                                                       int nA, float damping, int mode) {
  const int i = blockIdx.y;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < nA; j += gridDim.x * 256) {
    long long o = (long long)i * ldv + j;
    if (mode == 0) v[o] *= dGdA[(long long)i * nA + j];
    else v[o] /= (dG[i] * dA[j] + damping);
  }
}

// out = sum of part[0, n) in a fixed order (one workgroup)
__global__ __launch_bounds__(256) void kl_finalize_kernel(const double* __restrict__ part, int n,
                                                          double* out) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

}  // namespace

KFAC_API int kfac_kl_finalize(const double* part, int n, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(kl_finalize_kernel, dim3(1), dim3(256), 0, stream, part, n, out);
  return (int)hipGetLastError();
}

KFAC_API int kfac_kl_elems_per_block() { return ELEMS_PER_BLOCK; }

// entries: flat array of `count` records (ops/_lib.py MatRecord)
struct KfacMatRecord {
  const float* v;
  void* g;
  long long ldv, rows, cols, gdtype;
  long long gs0, gs1, gs2, gs3, kk, kw;
};

static int build_tables_and_launch(const KfacMatRecord* recs, int count, bool dot, double* vg,
                                   double lr2, double kl_clip, int use_clip, hipStream_t stream) {
  int part_off = 0;   // dot: per-workgroup partial slots at vg + 1 + part_off
  for (int base = 0; base < count; base += MAXG) {
    GroupTable t;
    memset(&t, 0, sizeof(t));   // deterministic table bytes (devtable key)
    t.count = count - base < MAXG ? count - base : MAXG;
    int blocks = 0;
    for (int k = 0; k < t.count; ++k) {
      const KfacMatRecord& r = recs[base + k];
      t.m[k].v = r.v; t.m[k].g = r.g; t.m[k].ldv = (int)r.ldv;
      t.m[k].rows = (int)r.rows; t.m[k].cols = (int)r.cols; t.m[k].gdtype = (int)r.gdtype;
      t.m[k].gs0 = r.gs0; t.m[k].gs1 = r.gs1; t.m[k].gs2 = r.gs2; t.m[k].gs3 = r.gs3;
      t.m[k].kk = (int)r.kk; t.m[k].kw = (int)r.kw;
      t.block_prefix[k] = blocks;
      long long n = r.rows * r.cols;
      blocks += (int)((n + ELEMS_PER_BLOCK - 1) / ELEMS_PER_BLOCK);
    }
    t.block_prefix[t.count] = blocks;
    if (blocks == 0) continue;
    int terr = 0;
    const GroupTable* d = (const GroupTable*)kfac_devtable::get(&t, sizeof(t), stream, &terr);
    if (!d) return terr;
    if (dot) {
      hipLaunchKernelGGL(grouped_kl_dot_kernel, dim3(blocks), dim3(256), 0, stream, d,
                         vg + 1 + part_off);
      part_off += blocks;
    } else
      hipLaunchKernelGGL(grouped_apply_kernel, dim3(blocks), dim3(256), 0, stream, d, vg, lr2,
                         kl_clip, use_clip);
    int err = (int)hipGetLastError();
    if (err) return err;
  }
  if (dot) return kfac_kl_finalize(vg + 1, part_off, vg, stream);
  return 0;
}

// vg: 1 + sum_k ceil(rows_k cols_k / kfac_kl_elems_per_block()) doubles; the
// result lands in vg[0], the per-workgroup partials after it.
KFAC_API int kfac_grouped_kl_dot(const KfacMatRecord* recs, int count, double* vg,
                                 hipStream_t stream) {
  return build_tables_and_launch(recs, count, true, vg, 0.0, 0.0, 0, stream);
}

KFAC_API int kfac_grouped_apply(const KfacMatRecord* recs, int count, const double* vg,
                                double lr2, double kl_clip, int use_clip, hipStream_t stream) {
  return build_tables_and_launch(recs, count, false, const_cast<double*>(vg), lr2, kl_clip,
                                 use_clip, stream);
}

KFAC_API int kfac_outer_recip(const float* dG, const float* dA, float* out, int nG, int nA,
                              float damping, hipStream_t stream) {
  dim3 grid((nA + 255) / 256 < 16 ? (nA + 255) / 256 : 16, nG);
  hipLaunchKernelGGL(outer_recip_kernel, grid, dim3(256), 0, stream, dG, dA, out, nG, nA, damping);
  return (int)hipGetLastError();
}

KFAC_API int kfac_hadamard(float* v, int ldv, const float* dGdA, const float* dG, const float* dA,
                           int nG, int nA, float damping, int mode, hipStream_t stream) {
  dim3 grid((nA + 255) / 256 < 16 ? (nA + 255) / 256 : 16, nG);
  hipLaunchKernelGGL(hadamard_kernel, grid, dim3(256), 0, stream, v, ldv, dGdA, dG, dA, nG, nA,
                     damping, mode);
  return (int)hipGetLastError();
}
