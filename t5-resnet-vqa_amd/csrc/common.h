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

// N independent 64-lane sums at once (N a power of two <= 64) by a butterfly
// reduce-scatter: each exchange step halves the values a lane keeps, so the N sums
// cost N-1 + log2(64/N) shuffles instead of 6N.  Returns the sum of value index
// (lane >> (6 - log2 N)) -- every lane of that index's group holds it.
template <int N>
__device__ __forceinline__ float wave_sum_scatter(float (&v)[N]) {
  static_assert(N >= 1 && N <= 64 && (N & (N - 1)) == 0, "N must be a power of two <= 64");
  const int l = threadIdx.x & 63;
  int m = 32;
#pragma unroll
  for (int c = N; c > 1; c >>= 1, m >>= 1) {
    const bool up = (l & m) != 0;
#pragma unroll
    for (int i = 0; i < c / 2; ++i) {
      const float keep = up ? v[c / 2 + i] : v[i];
      const float send = up ? v[i] : v[c / 2 + i];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  float r = v[0];
#pragma unroll
  for (; m > 0; m >>= 1) r += __shfl_xor(r, m, 64);
  return r;
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

// ---------------------------------------------------------------- dropout
// Counter-based keep masks (include/vqa_hip.h, "dropout"): stateless, so a
// kernel regenerates exactly the forward mask in backward from (rng, site, e).
__host__ __device__ __forceinline__ uint32_t vqa_mix32(uint32_t x) {     // lowbias32 finaliser
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
struct DropK {
  uint32_t key, thresh;
  float scale;
  bool on;
};
__device__ __forceinline__ DropK drop_init(const vqa_dropout& d) {
  DropK k;
  k.on = d.p > 0.f && d.rng != nullptr && d.rng[2] != 0u;      // rng[2]: training flag (eval() clears it)
  k.key = 0; k.thresh = 0; k.scale = 1.f;
  if (k.on) {
    const uint32_t k0 = vqa_mix32(d.rng[0] + 0x9E3779B9u);
    const uint32_t k1 = vqa_mix32(k0 ^ (d.rng[1] * 0x85EBCA6Bu + 0x632BE5ABu));
    k.key = vqa_mix32(k1 ^ (d.site * 0xC2B2AE35u + 0x27D4EB2Fu));
    k.thresh = (uint32_t)((double)d.p * 4294967296.0);
    k.scale = 1.f / (1.f - d.p);
  }
  return k;
}
__device__ __forceinline__ bool drop_keep(const DropK& k, uint32_t e) {
  return vqa_mix32(e * 0x9E3779B9u + k.key) >= k.thresh;
}
// multiplier for element e: scale if kept, 0 if dropped, 1 when dropout is off
__device__ __forceinline__ float drop_mul(const DropK& k, uint32_t e) {
  return k.on ? (drop_keep(k, e) ? k.scale : 0.f) : 1.f;
}

// ---------------------------------------------------------------- host side
namespace vqa {
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
}  // namespace vqa

#define VQA_REQUIRE(cond, ...) \
  do { if (!(cond)) return vqa::fail(VQA_ERR_INVALID, __VA_ARGS__); } while (0)
