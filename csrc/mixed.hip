// Grouped dtype casts for bf16-stored model weights with fp32 master copies
// (ops/mixed.py, BF16Weights).
//
// Under torch.autocast every step casts each fp32 Conv/Linear weight to bf16
// in the forward (one elementwise launch per tensor) and each bf16 weight
// gradient back to fp32 in the backward (another launch per tensor): ~110
// launches per ResNet-50 step, ~1.4 ms of small kernels
// (profiles/r3_s2_bench_window_breakdown.txt: bfloat16_copy /
// bfloat16tofloat32_copy).  Keeping the module weights in bf16 and the fp32
// masters in the optimizer gives the same values (autocast's forward operand
// IS the RNE bf16 cast of the master; its weight gradient IS the bf16 conv
// gradient widened to fp32) with ONE launch per direction for all tensors:
//   mode 0  dst_f32[i] = float(src_bf16[i])      gradients -> masters
//   mode 1  dst_bf16[i] = bf16_rne(src_f32[i])   masters -> model weights
// Each job is a contiguous tensor; workgroups stride over 8-element chunks of
// the concatenation (16-byte bf16 / 32-byte f32 accesses), a scalar tail per
// job for numel % 8.
#include "common.h"

#include "devtable.h"

namespace {

struct CastJob {
  const void* src; void* dst; long long n;
  long long chunk_begin;    // prefix sum of ceil(n / 8)
};

constexpr int MAX_CAST = 120;   // 120 x 32 B + header < 4 KB
struct CastBatch {
  int count, mode, pad[2];
  long long chunks;
  CastJob job[MAX_CAST];
};

typedef unsigned u32x4n __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void cast_grouped_kernel(const CastBatch* __restrict__ b) {
  const int count = b->count;
  const long long chunks = b->chunks;
  for (long long c = (long long)blockIdx.x * 256 + threadIdx.x; c < chunks;
       c += (long long)gridDim.x * 256) {
    int lo = 0, hi = count - 1;        // job of chunk c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (b->job[mid].chunk_begin <= c) lo = mid; else hi = mid - 1;
    }
    const CastJob& J = b->job[lo];
    const long long e0 = (c - J.chunk_begin) * 8;
    const long long ne = J.n - e0 < 8 ? J.n - e0 : 8;
    if (MODE == 0) {
      const uint16_t* s = (const uint16_t*)J.src + e0;
      float* d = (float*)J.dst + e0;
      if (ne == 8 && ((((size_t)s) | ((size_t)d)) & 15) == 0) {
        const u32x4n v = *(const u32x4n*)s;
        fx4 lo4, hi4;
        lo4.x = bf16_bits_to_f32((uint16_t)(v.x & 0xffffu)); lo4.y = bf16_bits_to_f32((uint16_t)(v.x >> 16));
        lo4.z = bf16_bits_to_f32((uint16_t)(v.y & 0xffffu)); lo4.w = bf16_bits_to_f32((uint16_t)(v.y >> 16));
        hi4.x = bf16_bits_to_f32((uint16_t)(v.z & 0xffffu)); hi4.y = bf16_bits_to_f32((uint16_t)(v.z >> 16));
        hi4.z = bf16_bits_to_f32((uint16_t)(v.w & 0xffffu)); hi4.w = bf16_bits_to_f32((uint16_t)(v.w >> 16));
        *(fx4*)d = lo4;
        *(fx4*)(d + 4) = hi4;
      } else {
        for (int i = 0; i < ne; ++i) d[i] = bf16_bits_to_f32(s[i]);
      }
    } else {
      const float* s = (const float*)J.src + e0;
      uint16_t* d = (uint16_t*)J.dst + e0;
      if (ne == 8 && ((((size_t)s) | ((size_t)d)) & 15) == 0) {
        const fx4 a = *(const fx4*)s, z = *(const fx4*)(s + 4);
        u32x4n o;
        o.x = f32_to_bf16_bits(a.x) | ((unsigned)f32_to_bf16_bits(a.y) << 16);
        o.y = f32_to_bf16_bits(a.z) | ((unsigned)f32_to_bf16_bits(a.w) << 16);
        o.z = f32_to_bf16_bits(z.x) | ((unsigned)f32_to_bf16_bits(z.y) << 16);
        o.w = f32_to_bf16_bits(z.z) | ((unsigned)f32_to_bf16_bits(z.w) << 16);
        *(u32x4n*)d = o;
      } else {
        for (int i = 0; i < ne; ++i) d[i] = f32_to_bf16_bits(s[i]);
      }
    }
  }
}

}  // namespace

struct KfacCastRecord {
  const void* src; void* dst; long long n;
};

// Cast `count` contiguous tensors in one launch per batch of MAX_CAST
// (mode 0: bf16 -> f32, mode 1: f32 -> bf16, RNE).  The job table goes through
// the content-addressed device table cache (capturable into a hipGraph).
KFAC_API int kfac_cast_grouped(const KfacCastRecord* recs, int count, int mode,
                               hipStream_t stream) {
  if (mode != 0 && mode != 1) return -2;
  for (int base = 0; base < count; base += MAX_CAST) {
    CastBatch b;
    memset(&b, 0, sizeof(b));     // deterministic table bytes (devtable key)
    b.count = count - base < MAX_CAST ? count - base : MAX_CAST;
    b.mode = mode;
    long long chunks = 0;
    for (int k = 0; k < b.count; ++k) {
      const KfacCastRecord& r = recs[base + k];
      b.job[k].src = r.src;
      b.job[k].dst = r.dst;
      b.job[k].n = r.n;
      b.job[k].chunk_begin = chunks;
      chunks += (r.n + 7) / 8;
    }
    b.chunks = chunks;
    if (chunks == 0) continue;
    int terr = 0;
    const CastBatch* d = (const CastBatch*)kfac_devtable::get(&b, sizeof(b), stream, &terr);
    if (!d) return terr;
    long long grid = (chunks + 255) / 256;
    if (grid > 2048) grid = 2048;
    if (mode == 0)
      hipLaunchKernelGGL(cast_grouped_kernel<0>, dim3((unsigned)grid), dim3(256), 0, stream, d);
    else
      hipLaunchKernelGGL(cast_grouped_kernel<1>, dim3((unsigned)grid), dim3(256), 0, stream, d);
    const int err = (int)hipGetLastError();
    if (err) return err;
  }
  return 0;
}
