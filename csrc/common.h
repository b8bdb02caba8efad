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
