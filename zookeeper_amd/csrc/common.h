// Shared helpers for the gfx950 (MI355X, CDNA4) kernels of zookeeper_amd.
//
// Conventions
//   * Every exported entry point is `extern "C"`, takes raw device pointers,
//     sizes and a hipStream_t, and returns a hipError_t as int (0 = success).
//   * Activations are NHWC bf16 (stored as uint16 bit patterns in memory,
//     converted with the native gfx950 cvt instructions via `__bf16`).
//   * Block sizes are multiples of 64 (wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZK_EXPORT extern "C" __attribute__((visibility("default")))

#define ZK_CHECK_LAUNCH() \
  do {                                       \
    hipError_t e__ = hipGetLastError();      \
    if (e__ != hipSuccess) return (int)e__;  \
  } while (0)

namespace zk {

constexpr int kWave = 64;

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// Round-to-nearest-even f32 -> bf16 through the compiler's native conversion
// (v_cvt_pk_bf16_f32 on gfx950, NaN-preserving).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// sign(v) as an e2m1 (FP4) nibble: +1 = 0x2 for v >= 0, -1 = 0xA otherwise.
// Sign images pack two channels per byte, the even channel in the low nibble
// (the operands of the MX-FP4 binary forward, igemm.hip).
__device__ __forceinline__ uint32_t fp4_sign(float v) { return v >= 0.f ? 0x2u : 0xAu; }

// splitmix64-style hash for per-example random decisions (flip, crops).
__device__ __forceinline__ uint32_t hash_u32(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(x ^ (x >> 31));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace zk
