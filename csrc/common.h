// Shared helpers for the gfx950 (MI355X / CDNA4) K-FAC kernels.
// Wave size is 64 on CDNA; every block size below is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KFAC_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// dtype codes shared with the Python side (ops/_lib.py)
enum KfacDType { KDT_F32 = 0, KDT_BF16 = 1, KDT_F16 = 2, KDT_F64 = 3 };

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
  // round-to-nearest-even; NaN stays NaN through a plain cast (guide: correctness table)
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float f16_bits_to_f32(uint16_t b) {
  return (float)__builtin_bit_cast(_Float16, b);
}
__device__ __forceinline__ uint16_t f32_to_f16_bits(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

template <int DT> struct DTypeTraits;
template <> struct DTypeTraits<KDT_F32> {
  typedef float raw_t;
  static __device__ __forceinline__ float to_f32(float v) { return v; }
  static __device__ __forceinline__ float from_f32(float v) { return v; }
};
template <> struct DTypeTraits<KDT_BF16> {
  typedef uint16_t raw_t;
  static __device__ __forceinline__ float to_f32(uint16_t v) { return bf16_bits_to_f32(v); }
  static __device__ __forceinline__ uint16_t from_f32(float v) { return f32_to_bf16_bits(v); }
};
template <> struct DTypeTraits<KDT_F16> {
  typedef uint16_t raw_t;
  static __device__ __forceinline__ float to_f32(uint16_t v) { return f16_bits_to_f32(v); }
  static __device__ __forceinline__ uint16_t from_f32(float v) { return f32_to_f16_bits(v); }
};

__device__ __forceinline__ float wave_reduce_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_reduce_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Global-address-space views of pointers that come from memory (record
// tables): plain pointers loaded from a struct compile to flat_* accesses,
// which wait on lgkmcnt as well as vmcnt.  gld_if is a branch-free predicated
// load (clamped index + select): loads written as `if (ok) v = p[i]` become
// one branch per load with a full wait inside, i.e. one memory round trip
// each; these issue back to back and wait once.
#define AS1 __attribute__((address_space(1)))
typedef float fx4 __attribute__((ext_vector_type(4)));   // native vector: loads through AS1
template <class T>
__device__ __forceinline__ AS1 T* gptr(T* p) { return (AS1 T*)p; }
template <class T>
__device__ __forceinline__ const AS1 T* gptr(const T* p) { return (const AS1 T*)p; }
template <class T>
__device__ __forceinline__ T gld_if(const AS1 T* p, long long i, bool ok, T z) {
  const T v = p[ok ? i : 0];
  return ok ? v : z;
}
// 32-bit element offset: the load becomes `global_load v, v_off, s[base]` (one
// offset VGPR instead of a 64-bit address pair); callers guarantee i < 2^32
template <class T>
__device__ __forceinline__ T gld_if32(const AS1 T* p, unsigned i, bool ok, T z) {
  const T v = p[ok ? i : 0u];
  return ok ? v : z;
}

// Wave sums on the VALU (no LDS round trips): DPP quad_perm / half-mirror /
// mirror inside each 16-lane row, then the gfx950 permlane16/32 swaps across
// rows.  Every lane ends with the same value (each pairwise add is taken in
// both orders, which are equal), in a fixed order: deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float swap_sum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_sum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ double swap_sum16_d(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
__device__ __forceinline__ double swap_sum32_d(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);    // row_half_mirror
  v += dpp_f<0x140>(v);    // row_mirror
  return swap_sum32(swap_sum16(v));
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return swap_sum32_d(swap_sum16_d(v));
}

// In-register transpose-reduce of 64 values per lane over the wave: lane L
// ends with the wave sum of value L (63 shuffles, pairwise, fixed order).
template <int M>
__device__ __forceinline__ void kfac_butterfly_stage(float (&v)[64], int lane) {
  const bool up = (lane & M) != 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const float send = up ? v[i] : v[i + M];
    const float keep = up ? v[i + M] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
}
__device__ __forceinline__ float kfac_butterfly64(float (&v)[64]) {
  const int lane = threadIdx.x & 63;
  kfac_butterfly_stage<32>(v, lane);
  kfac_butterfly_stage<16>(v, lane);
  kfac_butterfly_stage<8>(v, lane);
  kfac_butterfly_stage<4>(v, lane);
  kfac_butterfly_stage<2>(v, lane);
  kfac_butterfly_stage<1>(v, lane);
  return v[0];
}

// Transposed wave sum of 16 values per lane: lanes with (lane & 15) == x end
// with the wave sum of value x (15 + 2 shuffles instead of 16 wave sums).
template <int M>
__device__ __forceinline__ void kfac_fold16(float (&v)[16], int lane) {
  const bool up = (lane & M) != 0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const float send = up ? v[i] : v[i + M];
    const float keep = up ? v[i + M] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
}
__device__ __forceinline__ float kfac_butterfly16(float (&v)[16]) {
  const int lane = threadIdx.x & 63;
  kfac_fold16<8>(v, lane);
  kfac_fold16<4>(v, lane);
  kfac_fold16<2>(v, lane);
  kfac_fold16<1>(v, lane);
  float r = v[0];
  r += __shfl_xor(r, 16, 64);
  r += __shfl_xor(r, 32, 64);
  return r;
}

// Workgroup barrier for LDS traffic only: waits for this wave's LDS
// operations (lgkmcnt) but NOT for its outstanding global loads / stores, so
// prefetches stay in flight across it (__syncthreads() is a workgroup-scope
// release + acquire, which on gfx950 also drains vmcnt).  Callers order any
// global data themselves (s_waitcnt before publishing, register dependencies
// for loaded values).
__device__ __forceinline__ void kfac_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
