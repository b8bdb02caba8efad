// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels_last
// bf16 activations on gfx950: the ResNet-50 normalisation layers of the
// headline benchmark.
//
// The stock path runs, per BN layer and step, 3 MIOpen forward kernels, a
// clamp (ReLU) kernel, an add kernel (residual), a num_batches_tracked
// increment, and in backward 3 MIOpen kernels plus the ReLU mask and the add's
// gradient split: ~3.6 ms of a 12.3 ms ResNet-50 step at batch 32, memory-bound
// work at a fraction of HBM bandwidth (profiles/README.md).  Here:
//
//   forward   stats     per (channel group, row chunk) block: shifted sums of
//                       x - x[first row] and their squares (one 16-byte load =
//                       8 channels per thread), block-reduced in a fixed
//                       order -> chunk (mean, M2)
//             finalize  one workgroup per channel: the chunks merged in fp64
//                       about a common shift -> mean, 1/sqrt(var + eps); running
//                       stats (unbiased var) and num_batches_tracked updated
//                       in place; scale = w / sigma, shift = b - mean scale
//             apply     y = relu(x scale + shift [+ z]) in bf16
//   backward  reduce    per chunk: sum g and sum g x_hat, g = dy masked by
//                       y > 0 (ReLU) -- x_hat recomputed from x, mean, invstd
//             finalize  fp64 chunk sums -> dbias, dweight and the dx
//                       coefficients
//             apply     dx = (w / sigma) (g - sum g / M - x_hat sum g x_hat / M),
//                       dz = g for the residual branch
//
// Every reduction runs in a fixed order (no atomics): bitwise reproducible.
// Layout: x[m * C + c], m < M = N H W, C % 8 == 0, 16-byte aligned rows.
#include "common.h"

namespace {

typedef unsigned u32x4n __attribute__((ext_vector_type(4)));
typedef float fx2 __attribute__((ext_vector_type(2)));

constexpr int NT = 256;              // threads per block
constexpr int TARGET_BLOCKS = 1024;  // stats / reduce grid (4 per CU; fewer chunk partials)

__device__ __forceinline__ void unpack8(const u32x4n v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4n pack8(const float* f) {
  u32x4n v;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = (uint32_t)f32_to_bf16_bits(f[2 * i]) | ((uint32_t)f32_to_bf16_bits(f[2 * i + 1]) << 16);
  return v;
}

struct Geo {
  int cb, tpr, rpi, ncg, rows, nchunks;
};

// channel group width, threads per row, rows per iteration and the row chunks
// of an (M, C) problem (host and device agree: computed on the host only)
Geo geometry(long long M, int C) {
  Geo g;
  // a power of two (threads per row must divide the block), C % 8 == 0
  g.cb = 256;
  while (g.cb > 8 && C % g.cb) g.cb >>= 1;
  g.tpr = g.cb / 8;
  g.rpi = NT / g.tpr;
  g.ncg = C / g.cb;
  long long per = (M * g.ncg + TARGET_BLOCKS - 1) / TARGET_BLOCKS;
  if (per < g.rpi) per = g.rpi;
  per = (per + g.rpi - 1) / g.rpi * g.rpi;
  g.rows = (int)per;
  g.nchunks = (int)((M + per - 1) / per);
  return g;
}

// sums over this block's chunk of rows for 8 channels per thread, reduced
// over the block's row lanes into the lanes of row 0 (fixed order).
// Lanes of one wave that share a channel octet (lane % tpr) are folded by xor
// shuffles at distances tpr .. 32 (every lane ends with its octet's wave sum),
// then the four wave sums are added in wave order through LDS.  The round-4
// form -- every row's 16 sums through LDS, then the row-0 lanes adding all
// rpi rows one after another (31 dependent LDS steps at 64 channels) -- held
// the C = 64 statistics launches at ~15 us for 13 MB.
__device__ __forceinline__ void block_reduce16(float* acc, float (*red)[32][17], int cv, int tpr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = tpr; d < 64; d <<= 1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += __shfl_xor(acc[i], d, 64);
  }
  if (lane < tpr) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[w][lane][i] = acc[i];
  }
  __syncthreads();
  if (w == 0 && lane < tpr) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      acc[i] = (red[0][cv][i] + red[1][cv][i]) + (red[2][cv][i] + red[3][cv][i]);
  }
}

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(NT) void bn_stats_kernel(const uint16_t* __restrict__ x, long long M,
                                                      int C, Geo g, float* __restrict__ part) {
  __shared__ float red[NT / 64][32][17];
  const int cg = blockIdx.x, chunk = blockIdx.y;
  const int t = threadIdx.x, cv = t % g.tpr, rr = t / g.tpr;
  const int c0 = cg * g.cb + cv * 8;
  const long long m0 = (long long)chunk * g.rows;
  const long long m1 = m0 + g.rows < M ? m0 + g.rows : M;
  const AS1 u32x4n* X = (const AS1 u32x4n*)x;
  float k[8];
  unpack8(X[(m0 * C + c0) / 8], k);      // shift: the chunk's first row
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // 4 rows' loads in flight per thread before the (in-order) accumulation:
  // one 16-byte load at a time left the pass latency bound
  const long long cs = (long long)C / 8, step = (long long)g.rpi * cs;
  long long m = m0 + rr;
  const AS1 u32x4n* Xp = X + (m * C + c0) / 8;
  for (; m + 3 * g.rpi < m1; m += 4 * g.rpi, Xp += 4 * step) {
    u32x4n q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = Xp[u * step];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(q[u], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = f[i] - k[i];
        acc[i] += d;
        acc[8 + i] = fmaf(d, d, acc[8 + i]);
      }
    }
  }
  for (; m < m1; m += g.rpi, Xp += step) {
    float f[8];
    unpack8(*Xp, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = f[i] - k[i];
      acc[i] += d;
      acc[8 + i] = fmaf(d, d, acc[8 + i]);
    }
  }
  block_reduce16(acc, red, cv, g.tpr);
  if (rr == 0) {
    const float n = (float)(m1 - m0);
    // channel-major partials [c][chunk][2]: the finalize wave of a channel
    // reads its chunks as one contiguous run (chunk-major put each lane of
    // that wave on its own cache line)
    AS1 float* o = gptr(part) + ((long long)c0 * g.nchunks + chunk) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float s1 = acc[i], s2 = acc[8 + i];
      fx2 v;
      v.x = k[i] + s1 / n;                        // chunk mean
      v.y = fmaxf(s2 - s1 * (s1 / n), 0.f);       // chunk M2
      *(AS1 fx2*)(o + (long long)i * g.nchunks * 2) = v;
    }
  }
}

// fp64 sums of a workgroup (one channel per workgroup): waves reduced in
// lane order, then the 4 wave sums in wave order -- fixed, deterministic
__device__ __forceinline__ void block_sum2_d(double& a, double& b) {
  __shared__ double sh[2][NT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = wave_reduce_sum_d(a);
  b = wave_reduce_sum_d(b);
  if (lane == 0) { sh[0][w] = a; sh[1][w] = b; }
  __syncthreads();
  a = 0.0; b = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) { a += sh[0][i]; b += sh[1][i]; }
}

// one workgroup per channel (the chunks of a channel spread over 256 lanes:
// the chunk loop is 4 iterations at ResNet-50's 1024 chunks, not 16 on one
// wave): the chunk (mean, M2) pairs merged in fp64 about a common shift (the
// first chunk's mean): S1 = sum n_k (mean_k - K), S2 = sum M2_k + n_k
// (mean_k - K)^2 -- FMAs only, no per-chunk divisions
__global__ __launch_bounds__(NT) void bn_finalize_kernel(
    const float* __restrict__ part, long long M, int C, Geo g, float eps, float momentum,
    const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ rmean,
    float* __restrict__ rvar, long long* __restrict__ nbt, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x, t = threadIdx.x;
  if (c == 0 && t == 0 && nbt != nullptr) nbt[0] += 1;
  const AS1 fx2* pc = (const AS1 fx2*)(gptr(part) + (long long)c * g.nchunks * 2);
  const double K = (double)pc[0].x;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll 4
  for (int k = t; k < g.nchunks; k += NT) {
    const long long r0 = (long long)k * g.rows;
    const double nb = (double)((M - r0) < g.rows ? (M - r0) : g.rows);
    const fx2 e = pc[k];
    const double d = (double)e.x - K;
    s1 = fma(nb, d, s1);
    s2 += (double)e.y + nb * d * d;
  }
  block_sum2_d(s1, s2);
  if (t == 0) {
    const double mean = K + s1 / (double)M;
    const double m2 = s2 - s1 * (s1 / (double)M);
    const double var = m2 / (double)M;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    if (rmean != nullptr) {
      const double unb = M > 1 ? m2 / (double)(M - 1) : var;
      rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mean);
      rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
    }
    const float sc = (w ? w[c] : 1.f) * invstd;
    scale[c] = sc;
    shift[c] = (b ? b[c] : 0.f) - (float)mean * sc;
  }
}

__device__ __forceinline__ void load8(const float* __restrict__ p, int c0, float* o) {
  const fx4 a = *(const AS1 fx4*)(gptr(p) + c0), b = *(const AS1 fx4*)(gptr(p) + c0 + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

template <bool RELU, bool ADD>
__device__ __forceinline__ void apply8(const AS1 u32x4n* X, const AS1 u32x4n* Z, AS1 u32x4n* Y,
                                       long long v, const float* sc, const float* sh) {
  float f[8], o[8], zz[8];
  unpack8(X[v], f);
  if (ADD) unpack8(Z[v], zz);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float r = fmaf(f[i], sc[i], sh[i]);
    if (ADD) r += zz[i];
    o[i] = RELU ? fmaxf(r, 0.f) : r;
  }
  Y[v] = pack8(o);
}

// Grid-stride elementwise pass.  When C / 8 divides the block size (every
// power-of-two C <= 2048: all of ResNet-50) the stride is a multiple of C / 8,
// so each thread keeps ONE channel octet: its per-channel operands are loaded
// once, and no per-element 64-bit modulo is issued (the pass is VALU-heavy
// enough at 16 bytes per lane for that to matter).
template <bool RELU, bool ADD>
__global__ __launch_bounds__(NT) void bn_apply_kernel(const uint16_t* __restrict__ x,
                                                      const uint16_t* __restrict__ z,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      uint16_t* __restrict__ y, long long nvec,
                                                      int C) {
  const AS1 u32x4n* X = (const AS1 u32x4n*)x;
  const AS1 u32x4n* Z = (const AS1 u32x4n*)z;
  AS1 u32x4n* Y = (AS1 u32x4n*)y;
  const int cvec = C / 8;
  const long long stride = (long long)gridDim.x * NT;
  const long long v0 = blockIdx.x * (long long)NT + threadIdx.x;
  float sc[8], sh[8];
  if (NT % cvec == 0) {
    const int c0 = (threadIdx.x % cvec) * 8;
    load8(scale, c0, sc);
    load8(shift, c0, sh);
    for (long long v = v0; v < nvec; v += stride) apply8<RELU, ADD>(X, Z, Y, v, sc, sh);
  } else {
    for (long long v = v0; v < nvec; v += stride) {
      const int c0 = (int)(v % cvec) * 8;
      load8(scale, c0, sc);
      load8(shift, c0, sh);
      apply8<RELU, ADD>(X, Z, Y, v, sc, sh);
    }
  }
}

// --------------------------------------------------------------- backward
template <bool RELU>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
    const uint16_t* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, long long M, int C, Geo g, float* __restrict__ part) {
  __shared__ float red[NT / 64][32][17];
  const int cg = blockIdx.x, chunk = blockIdx.y;
  const int t = threadIdx.x, cv = t % g.tpr, rr = t / g.tpr;
  const int c0 = cg * g.cb + cv * 8;
  const long long m0 = (long long)chunk * g.rows;
  const long long m1 = m0 + g.rows < M ? m0 + g.rows : M;
  const AS1 u32x4n* DY = (const AS1 u32x4n*)dy;
  const AS1 u32x4n* Y = (const AS1 u32x4n*)y;
  const AS1 u32x4n* X = (const AS1 u32x4n*)x;
  float mu[8], is[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { mu[i] = mean[c0 + i]; is[i] = invstd[c0 + i]; }
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // 2 rows (up to 6 loads) in flight per thread, accumulated in row order
  const long long step = (long long)g.rpi * (C / 8);
  long long m = m0 + rr, v = (m * C + c0) / 8;
  for (; m + g.rpi < m1; m += 2 * g.rpi, v += 2 * step) {
    u32x4n qg[2], qx[2], qy[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      qg[u] = DY[v + u * step];
      qx[u] = X[v + u * step];
      if (RELU) qy[u] = Y[v + u * step];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float gv[8], xv[8], yv[8];
      unpack8(qg[u], gv);
      unpack8(qx[u], xv);
      if (RELU) unpack8(qy[u], yv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gg = (!RELU || yv[i] > 0.f) ? gv[i] : 0.f;
        acc[i] += gg;
        acc[8 + i] = fmaf(gg, (xv[i] - mu[i]) * is[i], acc[8 + i]);
      }
    }
  }
  for (; m < m1; m += g.rpi, v += step) {
    float gv[8], xv[8], yv[8];
    unpack8(DY[v], gv);
    unpack8(X[v], xv);
    if (RELU) unpack8(Y[v], yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float gg = (!RELU || yv[i] > 0.f) ? gv[i] : 0.f;
      acc[i] += gg;
      acc[8 + i] = fmaf(gg, (xv[i] - mu[i]) * is[i], acc[8 + i]);
    }
  }
  block_reduce16(acc, red, cv, g.tpr);
  if (rr == 0) {
    AS1 float* o = gptr(part) + ((long long)c0 * g.nchunks + chunk) * 2;   // [c][chunk][2]
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fx2 v;
      v.x = acc[i];
      v.y = acc[8 + i];
      *(AS1 fx2*)(o + (long long)i * g.nchunks * 2) = v;
    }
  }
}

// one workgroup per channel: fp64 chunk sums -> dw, db and the planar
// (A, B, X) of dx = a (g - k1 - x_hat k2) = A g + B + X x
__global__ __launch_bounds__(NT) void bn_bwd_finalize_kernel(
    const float* __restrict__ part, long long M, int C, Geo g, const float* __restrict__ w,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ dw, float* __restrict__ db,
    float* __restrict__ coef) {
  const int c = blockIdx.x, t = threadIdx.x;
  const AS1 fx2* pc = (const AS1 fx2*)(gptr(part) + (long long)c * g.nchunks * 2);
  double sg = 0.0, sgx = 0.0;
#pragma unroll 4
  for (int k = t; k < g.nchunks; k += NT) {
    const fx2 e = pc[k];
    sg += (double)e.x;
    sgx += (double)e.y;
  }
  block_sum2_d(sg, sgx);
  if (t == 0) {
    if (dw) dw[c] = (float)sgx;
    if (db) db[c] = (float)sg;
    // dx = a (g - k1 - (x - mean) invstd k2) as an affine map of (g, x):
    // A g + B + X x, planar per channel (float4 loads in the apply pass)
    const double a = (double)(w ? w[c] : 1.f) * (double)invstd[c];
    const double k1 = sg / (double)M, k2 = sgx / (double)M;
    const double ak = a * k2 * (double)invstd[c];
    coef[c] = (float)a;
    coef[C + c] = (float)(ak * (double)mean[c] - a * k1);
    coef[2 * C + c] = (float)(-ak);
  }
}

template <bool RELU, bool ADD>
__device__ __forceinline__ void bwd_apply8(const AS1 u32x4n* DY, const AS1 u32x4n* Y,
                                           const AS1 u32x4n* X, AS1 u32x4n* DX, AS1 u32x4n* DZ,
                                           long long v, const float* ca, const float* cb,
                                           const float* cx) {
  float gv[8], xv[8], yv[8], o[8], gz[8];
  unpack8(DY[v], gv);
  unpack8(X[v], xv);
  if (RELU) unpack8(Y[v], yv);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float gg = (!RELU || yv[i] > 0.f) ? gv[i] : 0.f;
    o[i] = fmaf(xv[i], cx[i], fmaf(gg, ca[i], cb[i]));
    gz[i] = gg;
  }
  DX[v] = pack8(o);
  if (ADD) DZ[v] = pack8(gz);
}

// same one-octet-per-thread scheme as bn_apply_kernel
template <bool RELU, bool ADD>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
    const uint16_t* __restrict__ x, const float* __restrict__ coef,
    uint16_t* __restrict__ dx, uint16_t* __restrict__ dz, long long nvec, int C) {
  const AS1 u32x4n* DY = (const AS1 u32x4n*)dy;
  const AS1 u32x4n* Y = (const AS1 u32x4n*)y;
  const AS1 u32x4n* X = (const AS1 u32x4n*)x;
  AS1 u32x4n* DX = (AS1 u32x4n*)dx;
  AS1 u32x4n* DZ = (AS1 u32x4n*)dz;
  const int cvec = C / 8;
  const long long stride = (long long)gridDim.x * NT;
  const long long v0 = blockIdx.x * (long long)NT + threadIdx.x;
  float ca[8], cb[8], cx[8];
  if (NT % cvec == 0) {
    const int c0 = (threadIdx.x % cvec) * 8;
    load8(coef, c0, ca);
    load8(coef + C, c0, cb);
    load8(coef + 2 * C, c0, cx);
    for (long long v = v0; v < nvec; v += stride)
      bwd_apply8<RELU, ADD>(DY, Y, X, DX, DZ, v, ca, cb, cx);
  } else {
    for (long long v = v0; v < nvec; v += stride) {
      const int c0 = (int)(v % cvec) * 8;
      load8(coef, c0, ca);
      load8(coef + C, c0, cb);
      load8(coef + 2 * C, c0, cx);
      bwd_apply8<RELU, ADD>(DY, Y, X, DX, DZ, v, ca, cb, cx);
    }
  }
}

int apply_grid(long long nvec) {
  long long b = (nvec + NT - 1) / NT;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

// workspace floats of one BN call: chunk partials (2 per channel per chunk)
// + scale/shift (forward) or the dx coefficients (backward)
KFAC_API long long kfac_bn_ws_floats(long long M, int C) {
  const Geo g = geometry(M, C);
  return 2LL * g.nchunks * C + 3LL * C;
}

KFAC_API int kfac_bn_forward(const void* x, const void* z, const float* w, const float* b,
                             float* rmean, float* rvar, long long* nbt, void* y,
                             float* save_mean, float* save_invstd, float* ws, long long M, int C,
                             float eps, float momentum, int relu, hipStream_t stream) {
  if (C % 8 || M <= 0 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15) ||
      (z && ((uintptr_t)z & 15)))
    return -2;
  const Geo g = geometry(M, C);
  float* part = ws;
  float* scale = ws + 2LL * g.nchunks * C;
  float* shift = scale + C;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(g.ncg, g.nchunks), dim3(NT), 0, stream,
                     (const uint16_t*)x, M, C, g, part);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(NT), 0, stream, part, M, C, g,
                     eps, momentum, w, b, rmean, rvar, nbt, save_mean, save_invstd, scale, shift);
  const long long nvec = M * C / 8;
  const dim3 grid(apply_grid(nvec));
  const uint16_t* X = (const uint16_t*)x;
  const uint16_t* Z = (const uint16_t*)z;
  uint16_t* Y = (uint16_t*)y;
  if (relu && z)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), grid, dim3(NT), 0, stream, X, Z, scale, shift, Y, nvec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, false>), grid, dim3(NT), 0, stream, X, Z, scale, shift, Y, nvec, C);
  else if (z)
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), grid, dim3(NT), 0, stream, X, Z, scale, shift, Y, nvec, C);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, false>), grid, dim3(NT), 0, stream, X, Z, scale, shift, Y, nvec, C);
  return (int)hipGetLastError();
}

// dz (the residual branch's gradient) is written when non-null
KFAC_API int kfac_bn_backward(const void* dy, const void* y, const void* x, const float* w,
                              const float* save_mean, const float* save_invstd, void* dx,
                              void* dz, float* dw, float* db, float* ws, long long M, int C,
                              int relu, hipStream_t stream) {
  if (C % 8 || M <= 0 || ((uintptr_t)dy & 15) || ((uintptr_t)x & 15) || ((uintptr_t)dx & 15) ||
      (relu && ((uintptr_t)y & 15)) || (dz && ((uintptr_t)dz & 15)))
    return -2;
  const Geo g = geometry(M, C);
  float* part = ws;
  float* coef = ws + 2LL * g.nchunks * C;
  const uint16_t* DY = (const uint16_t*)dy;
  const uint16_t* Y = (const uint16_t*)y;
  const uint16_t* X = (const uint16_t*)x;
  if (relu)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(g.ncg, g.nchunks), dim3(NT), 0, stream,
                       DY, Y, X, save_mean, save_invstd, M, C, g, part);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(g.ncg, g.nchunks), dim3(NT), 0, stream,
                       DY, Y, X, save_mean, save_invstd, M, C, g, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(NT), 0, stream, part, M, C,
                     g, w, save_mean, save_invstd, dw, db, coef);
  const long long nvec = M * C / 8;
  const dim3 grid(apply_grid(nvec));
  uint16_t* DX = (uint16_t*)dx;
  uint16_t* DZ = (uint16_t*)dz;
  if (relu && dz)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true>), grid, dim3(NT), 0, stream, DY, Y, X, coef, DX, DZ, nvec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false>), grid, dim3(NT), 0, stream, DY, Y, X, coef, DX, DZ, nvec, C);
  else if (dz)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true>), grid, dim3(NT), 0, stream, DY, Y, X, coef, DX, DZ, nvec, C);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false>), grid, dim3(NT), 0, stream, DY, Y, X, coef, DX, DZ, nvec, C);
  return (int)hipGetLastError();
}
