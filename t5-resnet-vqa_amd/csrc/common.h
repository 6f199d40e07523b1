// Shared device/host helpers for libvqa_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/vqa_hip.h"

typedef unsigned short bf16_t;                                            // bf16 storage
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

#define WAVE 64

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;                                                   // v_cvt_pk_bf16_f32 (RNE, NaN-safe)
  return __builtin_bit_cast(bf16_t, b);
}

// 64-lane reductions (wave = 64 on CDNA; never 32)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); `red` must hold NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------- host side
namespace vqa {
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
}  // namespace vqa

#define VQA_REQUIRE(cond, ...) \
  do { if (!(cond)) return vqa::fail(VQA_ERR_INVALID, __VA_ARGS__); } while (0)
