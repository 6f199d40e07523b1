// Memory-bound helpers of the step: image layout change, max-pool, column sums
// (bias gradients), T5 embedding gather / scatter-add, T5 relative-position
// bias gather / scatter, casts and zeroing.  All 16-B vectorised where the
// layout allows (cdna_hip_programming.md Guideline 13).
#include "common.h"

namespace {

// NCHW fp32 [N,3,H,W] in [0,1] (collate ToTensor, resnet_vqa_daquar_dataset.py:131-137)
// -> NHWC bf16 [N,H,W,8], channels 3..7 zero (the stem conv's K = 7*7*8).
__global__ __launch_bounds__(256) void image_to_nhwc8_kernel(const float* __restrict__ img, bf16_t* __restrict__ out,
                                                             int n, int hw) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)n * hw) return;
  const long b = i / hw, p = i - b * hw;
  const float* src = img + b * 3 * hw + p;
  uint4 u;
  u.x = (uint32_t)f2bf(src[0]) | ((uint32_t)f2bf(src[hw]) << 16);
  u.y = (uint32_t)f2bf(src[2 * hw]);
  u.z = 0; u.w = 0;
  reinterpret_cast<uint4*>(out)[i] = u;
}

// NCHW fp32 [N,3,H,W] -> the stem's space-to-depth image Z, NHWC bf16 [N,H/2+1,W/2+1,16]:
//   Z[b,u,v,(2p+q)*3+c] = img[b,c,2u+p-1,2v+q-1] (0 outside), channels 12..15 = 0.
// The 7x7 stride-2 pad-3 conv over img equals a 4x4 stride-1 pad-1 conv over Z with
// W'[o,a,e,(2p+q)*3+c] = W[o,c,2a+p,2e+q] (0 where 2a+p or 2e+q is 7): K = 256
// instead of 7*7*8 = 392, and every tap is 32 contiguous bytes.
__global__ __launch_bounds__(256) void image_to_s2d16_kernel(const float* __restrict__ img, bf16_t* __restrict__ out,
                                                             int n, int h, int w, int hz, int wz) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)n * hz * wz) return;
  const int v = (int)(i % wz);
  const long t = i / wz;
  const int u = (int)(t % hz), b = (int)(t / hz);
  const float* src = img + (long)b * 3 * h * w;
  float z[16];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int y = 2 * u + p - 1, x = 2 * v + q - 1;
      const bool ok = y >= 0 && y < h && x >= 0 && x < w;
      const long o = ok ? (long)y * w + x : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c) z[(2 * p + q) * 3 + c] = ok ? src[(long)c * h * w + o] : 0.f;
    }
#pragma unroll
  for (int c = 12; c < 16; ++c) z[c] = 0.f;
  uint4 lo, hi;
  lo.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
  lo.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
  lo.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
  lo.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
  hi.x = (uint32_t)f2bf(z[8]) | ((uint32_t)f2bf(z[9]) << 16);
  hi.y = (uint32_t)f2bf(z[10]) | ((uint32_t)f2bf(z[11]) << 16);
  hi.z = 0; hi.w = 0;
  reinterpret_cast<uint4*>(out)[2 * i] = lo;
  reinterpret_cast<uint4*>(out)[2 * i + 1] = hi;
}

// torchvision MaxPool2d(3, 2, 1) on NHWC bf16; 8 channels per thread
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int n,
                                                         int h, int w, int c, int oh, int ow) {
  const int c8 = c / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)n * oh * ow * c8) return;
  const int cc = (int)(i % c8);
  long t = i / c8;
  const int ox = (int)(t % ow); t /= ow;
  const int oy = (int)(t % oh);
  const int b = (int)(t / oh);
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
  for (int dy = 0; dy < 3; ++dy) {
    const int iy = oy * 2 - 1 + dy;
    if (iy < 0 || iy >= h) continue;
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if (ix < 0 || ix >= w) continue;
      uint4 u = reinterpret_cast<const uint4*>(x + (((long)b * h + iy) * w + ix) * c)[cc];
      const uint32_t wds[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        m[2 * j] = fmaxf(m[2 * j], bf2f((bf16_t)(wds[j] & 0xffff)));
        m[2 * j + 1] = fmaxf(m[2 * j + 1], bf2f((bf16_t)(wds[j] >> 16)));
      }
    }
  }
  uint4 o;
  o.x = (uint32_t)f2bf(m[0]) | ((uint32_t)f2bf(m[1]) << 16);
  o.y = (uint32_t)f2bf(m[2]) | ((uint32_t)f2bf(m[3]) << 16);
  o.z = (uint32_t)f2bf(m[4]) | ((uint32_t)f2bf(m[5]) << 16);
  o.w = (uint32_t)f2bf(m[6]) | ((uint32_t)f2bf(m[7]) << 16);
  reinterpret_cast<uint4*>(y)[i] = o;
}

// partial column sums of a [rows, cols] matrix: block = 256 columns x COLSUM_ROWS rows
constexpr int COLSUM_ROWS = 64;
template <bool BF16>
__global__ __launch_bounds__(256) void colsum_part_kernel(const void* __restrict__ xv, int rows, int cols, long ld,
                                                          float* __restrict__ ws) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + tx * 4;
  const int r0 = blockIdx.y * COLSUM_ROWS;
  // the thread's 16 rows are loaded unconditionally (clamped row / column, masked
  // by a multiply) before the first add: one round trip instead of 16
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int RPT = COLSUM_ROWS / 4;
  const int cl = min(c, cols - 4);
  float4 v[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = min(r0 + ty + 4 * q, rows - 1);
    if constexpr (BF16) {
      const uint2 u = *reinterpret_cast<const uint2*>((const bf16_t*)xv + (long)r * ld + cl);
      v[q] = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
    } else {
      v[q] = *reinterpret_cast<const float4*>((const float*)xv + (long)r * ld + cl);
    }
  }
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const float m = (c < cols && r0 + ty + 4 * q < rows) ? 1.f : 0.f;
    s[0] += v[q].x * m; s[1] += v[q].y * m; s[2] += v[q].z * m; s[3] += v[q].w * m;
  }
  __shared__ float red[4][256];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[ty][tx * 4 + j] = s[j];
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < cols)
    ws[(long)blockIdx.y * cols + cc] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                       red[3][threadIdx.x];
}

// h[t, :] = table[ids[t], :]  (T5Stack embed_tokens, modeling_t5.py:678)
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const long long* __restrict__ ids,
                                                            const float* __restrict__ table, float* __restrict__ out,
                                                            int tokens, int d4, int vocab, vqa_dropout drop) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)tokens * d4) return;
  const int t = (int)(i / d4), j = (int)(i - (long)t * d4);
  long long id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);     // clamp (reference raises; ids validated on host)
  float4 v = reinterpret_cast<const float4*>(table + id * (long)d4 * 4)[j];
  const DropK dk = drop_init(drop);                       // T5 embedding dropout (TF modeling_t5.py:725)
  if (dk.on) {
    const uint32_t e = (uint32_t)i * 4u;
    v.x *= drop_mul(dk, e); v.y *= drop_mul(dk, e + 1); v.z *= drop_mul(dk, e + 2); v.w *= drop_mul(dk, e + 3);
  }
  reinterpret_cast<float4*>(out)[i] = v;
}

__global__ void rng_advance_kernel(unsigned* rng) { rng[1] += 1u; }

__global__ __launch_bounds__(256) void dropout_mask_kernel(vqa_dropout d, float* __restrict__ out, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const DropK dk = drop_init(d);
  out[i] = drop_mul(dk, (uint32_t)i);
}

// Re-zero only the table rows the previous step's gradient wrote (its ids),
// instead of the whole dense [vocab, d] gradient; then remember this step's ids.
// One workgroup per token: reads its previous id before replacing it.
__global__ __launch_bounds__(256) void embedding_zero_rows_kernel(long long* __restrict__ prev,
                                                                  const long long* __restrict__ cur,
                                                                  float* __restrict__ dtable, int d, int vocab) {
  const int t = blockIdx.x;
  long long id = prev[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  float4* row = reinterpret_cast<float4*>(dtable + id * (long long)d);
  for (int c = threadIdx.x; c < d / 4; c += 256) row[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (cur && threadIdx.x == 0) prev[t] = cur[t];
}

// Deterministic dense embedding gradient (nn.Embedding sparse=False), no atomics:
//   1. one workgroup bitonic-sorts the keys (id << 16 | position), which groups
//      equal ids with their positions in token order, and finds each id-run's
//      end by a binary search of the sorted ids from the run start;
//   2. one workgroup per (run start, column slab) sums the run's dh rows in
//      that fixed order and writes the table row once.
// Bit-identical run to run (DP ranks stay in lockstep, graph replay == eager).
// ws: [0, T) sorted positions, [T, 2T) sorted ids (clamped), [2T, 3T) run end
// (valid at run starts).
// Bitonic network over n = max(pow2 >= tokens, 1024) keys, E = n/1024 per thread
// (element i = q*1024 + thread): stages with j < 64 exchange inside a wave by
// shuffles, 64 <= j < 1024 through LDS, j >= 1024 between a thread's own slots.
// Run ends by binary search of the sorted ids (one per run start).
__device__ __forceinline__ unsigned long long shfl_xor64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(unsigned)(v & 0xffffffffu), m, 64);
  const int hi = __shfl_xor((int)(unsigned)(v >> 32), m, 64);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
template <int E>
__global__ __launch_bounds__(1024) void embedding_sort_kernel(const long long* __restrict__ ids, int tokens, int vocab,
                                                              int* __restrict__ ws) {
  __shared__ unsigned long long key[E * 1024];          // E = 16: 128 KiB of the CU's 160 KiB
  constexpr int n = E * 1024;
  const int t = threadIdx.x;
  unsigned long long v[E];
#pragma unroll
  for (int q = 0; q < E; ++q) {
    const int i = q * 1024 + t;
    long long id = ids[min(i, tokens - 1)];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
    v[q] = i < tokens ? (((unsigned long long)id << 16) | (unsigned long long)i) : ~0ull;
  }
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 1024) {                                  // partner: another slot of this thread
        const int qj = j >> 10;
#pragma unroll
        for (int q = 0; q < E; ++q) {
          if (q & qj) continue;
          const int i = q * 1024 + t;
          const bool up = (i & k) == 0;
          const unsigned long long a = v[q], c = v[q | qj];
          v[q] = up ? (a < c ? a : c) : (a < c ? c : a);
          v[q | qj] = up ? (a < c ? c : a) : (a < c ? a : c);
        }
      } else if (j >= 64) {                             // partner: another wave, same slot
#pragma unroll
        for (int q = 0; q < E; ++q) key[q * 1024 + t] = v[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < E; ++q) {
          const int i = q * 1024 + t;
          const unsigned long long c = key[i ^ j];
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[q] = keep_min ? (v[q] < c ? v[q] : c) : (v[q] < c ? c : v[q]);
        }
        __syncthreads();
      } else {                                          // partner: a lane of this wave
#pragma unroll
        for (int q = 0; q < E; ++q) {
          const int i = q * 1024 + t;
          const unsigned long long c = shfl_xor64(v[q], j);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[q] = keep_min ? (v[q] < c ? v[q] : c) : (v[q] < c ? c : v[q]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < E; ++q) key[q * 1024 + t] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < E; ++q) {
    const int i = q * 1024 + t;
    if (i >= tokens) continue;
    const unsigned long long kt = v[q];
    const unsigned id = (unsigned)(kt >> 16);
    ws[i] = (int)(kt & 0xffff);
    ws[tokens + i] = (int)id;
    if (i == 0 || (unsigned)(key[i - 1] >> 16) != id) {  // run start: end = first slot with a larger id
      int lo = i + 1, hi = tokens;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((unsigned)(key[mid] >> 16) == id) lo = mid + 1; else hi = mid;
      }
      ws[2 * tokens + i] = lo;
    }
  }
}

// One workgroup per (sorted slot, 128-column slab); only the first slot of an
// id-run works, and ADDS its run's sum to the table row (the rows are zero, or
// hold the sum of an earlier token slice of the same scatter: 0 + s == s, so a
// single slice is bit-identical to a plain store).  Long runs (the pad id covers ~40% of a batch) are split over
// 16 row-lanes that each sum a fixed stride of the run; the 16 partials are
// then added in lane order through LDS, so the result is still bit-identical
// run to run.
constexpr int EMB_RL = 16, EMB_CL = 32;                // row-lanes x float4 column-lanes
__global__ __launch_bounds__(EMB_RL * EMB_CL) void embedding_bwd_kernel(const float* __restrict__ dh,
                                                                        float* __restrict__ dtable,
                                                                        const int* __restrict__ ws, int tokens,
                                                                        int d) {
  const int s0 = blockIdx.x;
  const int* pos = ws;
  const int* sid = ws + tokens;
  const int id = sid[s0];
  if (s0 > 0 && sid[s0 - 1] == id) return;           // not the first slot of its run (uniform per block)
  const int s1 = ws[2 * tokens + s0];                   // run end from the sort kernel's scan
  const int tx = threadIdx.x % EMB_CL, ty = threadIdx.x / EMB_CL;
  const int c4 = blockIdx.y * EMB_CL + tx;             // float4 column
  const bool act = c4 * 4 < d;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (act) {
    // 8 rows per batch: all position loads, then all row loads, are issued before
    // the first add, so a long run costs ~len/128 round trips, not len/16
    constexpr int U = 8;
    for (int u0 = s0 + ty; u0 < s1; u0 += EMB_RL * U) {
      // unconditional loads (index clamped into the run), the tail masked on the values:
      // a per-load branch would serialise the round trips
      int pp[U];
#pragma unroll
      for (int q = 0; q < U; ++q) pp[q] = pos[min(u0 + q * EMB_RL, s1 - 1)];
      float4 v[U];
#pragma unroll
      for (int q = 0; q < U; ++q) v[q] = reinterpret_cast<const float4*>(dh + (long)pp[q] * d)[c4];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        if (u0 + q * EMB_RL < s1) { acc.x += v[q].x; acc.y += v[q].y; acc.z += v[q].z; acc.w += v[q].w; }
      }
    }
  }
  __shared__ float4 red[EMB_RL][EMB_CL];
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && act) {
    float4 t = red[0][tx];
#pragma unroll
    for (int r = 1; r < EMB_RL; ++r) {
      const float4 v = red[r][tx];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4* dst = reinterpret_cast<float4*>(dtable + (long)id * d) + c4;
    const float4 o = *dst;
    t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
    *dst = t;
  }
}

// bias[h, i, j] = table[bucket[i*lk + j], h]   (compute_bias, modeling_t5.py:264-279)
__global__ __launch_bounds__(256) void relbias_fwd_kernel(const float* __restrict__ table,
                                                          const int* __restrict__ bucket, float* __restrict__ out,
                                                          int heads, int lqk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= heads * lqk) return;
  const int h = i / lqk, p = i - h * lqk;
  const int bk = bucket[p];
  // bucket < 0: a causally masked (query, key) pair of the T5 decoder (the extended
  // attention mask's finfo.min, TF modeling_t5 get_extended_attention_mask)
  out[i] = bk < 0 ? -3.4028234663852886e38f : table[bk * heads + h];
}

// dtable[b, h] = sum over (i, j) with bucket(i, j) == b of dbias[h, i, j]:
// one workgroup per (bucket, head), fixed-order block reduction
__global__ __launch_bounds__(256) void relbias_bwd_kernel(const float* __restrict__ dbias,
                                                          const int* __restrict__ bucket, float* __restrict__ dtable,
                                                          int heads, int lqk) {
  __shared__ float red[4];
  const int bk = blockIdx.x / heads, h = blockIdx.x - bk * heads;
  float s = 0.f;
  for (int p = threadIdx.x; p < lqk; p += 256)
    if (bucket[p] == bk) s += dbias[(long)h * lqk + p];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) dtable[bk * heads + h] = s;
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                            long n) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    float4 v = *reinterpret_cast<const float4*>(x + i);
    uint2 u;
    u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(y + i) = u;
  } else {
    for (long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}

__global__ __launch_bounds__(256) void zero_kernel(uint4* __restrict__ p, long n16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256)
    p[i] = make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(256) void copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, long n16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) dst[i] = src[i];
}

}  // namespace

extern "C" int vqa_image_to_s2d16(const float* img, void* out, int n, int h, int w, hipStream_t s) {
  VQA_REQUIRE(img && out && n > 0 && h > 1 && w > 1 && h % 2 == 0 && w % 2 == 0,
              "vqa_image_to_s2d16: bad arguments (H and W must be even)");
  const int hz = h / 2 + 1, wz = w / 2 + 1;
  const long total = (long)n * hz * wz;
  hipLaunchKernelGGL(image_to_s2d16_kernel, dim3(vqa::cdiv(total, 256)), dim3(256), 0, s, img, (bf16_t*)out, n, h, w,
                     hz, wz);
  return vqa::check_launch("vqa_image_to_s2d16");
}

extern "C" int vqa_image_to_nhwc8(const float* img, void* out, int n, int h, int w, hipStream_t s) {
  VQA_REQUIRE(img && out && n > 0 && h > 0 && w > 0, "vqa_image_to_nhwc8: bad arguments");
  const long total = (long)n * h * w;
  hipLaunchKernelGGL(image_to_nhwc8_kernel, dim3(vqa::cdiv(total, 256)), dim3(256), 0, s, img, (bf16_t*)out, n, h * w);
  return vqa::check_launch("vqa_image_to_nhwc8");
}

extern "C" int vqa_maxpool3x3s2_nhwc(const void* x, void* y, int n, int h, int w, int c, int oh, int ow,
                                     hipStream_t s) {
  VQA_REQUIRE(x && y && c % 8 == 0, "vqa_maxpool3x3s2_nhwc: bad arguments");
  const long total = (long)n * oh * ow * (c / 8);
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3(vqa::cdiv(total, 256)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n,
                     h, w, c, oh, ow);
  return vqa::check_launch("vqa_maxpool3x3s2_nhwc");
}

namespace {
// x[b, i*s, j*s, :] -> row (b, i, j) of y (row stride ldy); 8 channels (16 B) per thread
__global__ __launch_bounds__(256) void subsample_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int h,
                                                        int w, int c8, int s, int oh, int ow, long ldy8, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % c8);
  const long r = i / c8;                              // output row (b, oy, ox)
  const int ox = (int)(r % ow);
  const long t = r / ow;
  const int oy = (int)(t % oh);
  const long b = t / oh;
  y[r * ldy8 + cc] = x[((b * h + (long)oy * s) * w + (long)ox * s) * c8 + cc];
}
}  // namespace

extern "C" int vqa_subsample_nhwc(const void* x, int n, int h, int w, int c, int stride, void* y, long long ldy,
                                  hipStream_t s) {
  VQA_REQUIRE(x && y && n > 0 && h > 0 && w > 0 && stride >= 1 && c % 8 == 0 && ldy % 8 == 0 && ldy >= c &&
                  ((uintptr_t)y & 15) == 0 && ((uintptr_t)x & 15) == 0,
              "vqa_subsample_nhwc: bad arguments (c, ldy multiples of 8, 16-B aligned buffers)");
  const int oh = (h - 1) / stride + 1, ow = (w - 1) / stride + 1;
  const long total = (long)n * oh * ow * (c / 8);
  hipLaunchKernelGGL(subsample_kernel, dim3(vqa::cdiv(total, 256)), dim3(256), 0, s, (const uint4*)x, (uint4*)y, h, w,
                     c / 8, stride, oh, ow, (long)(ldy / 8), total);
  return vqa::check_launch("vqa_subsample_nhwc");
}

extern "C" int vqa_colsum_workspace_floats(int rows, int cols) { return vqa::cdiv(rows, COLSUM_ROWS) * cols; }
extern "C" int vqa_colsum_parts(int rows) { return vqa::cdiv(rows, COLSUM_ROWS); }

extern "C" int vqa_colsum(const void* x, int x_bf16, int rows, int cols, long long ld, float* out, float beta,
                          float* ws, hipStream_t s) {
  VQA_REQUIRE(x && ws && cols % 4 == 0 && ld % 4 == 0, "vqa_colsum: bad arguments");
  const int parts = vqa::cdiv(rows, COLSUM_ROWS);
  dim3 grid(vqa::cdiv(cols, 256), parts);
  if (x_bf16)
    hipLaunchKernelGGL(colsum_part_kernel<true>, grid, dim3(256), 0, s, x, rows, cols, (long)ld, ws);
  else
    hipLaunchKernelGGL(colsum_part_kernel<false>, grid, dim3(256), 0, s, x, rows, cols, (long)ld, ws);
  if (int rc = vqa::check_launch("vqa_colsum")) return rc;
  if (!out) return VQA_OK;                                   // deferred: vqa_colsum_batched reduces ws
  return vqa_colsum_partials(ws, parts, cols, cols, out, beta, s);
}

extern "C" int vqa_embedding_fwd(const long long* ids, const float* table, float* out, int tokens, int d, int vocab,
                                 const vqa_dropout* drop, hipStream_t s) {
  VQA_REQUIRE(ids && table && out && d % 4 == 0, "vqa_embedding_fwd: bad arguments");
  VQA_REQUIRE(!drop || (drop->p >= 0.f && drop->p < 1.f), "vqa_embedding_fwd: dropout p must be in [0, 1)");
  const vqa_dropout dr = drop ? *drop : vqa_dropout{0.f, 0u, nullptr};
  const long total = (long)tokens * (d / 4);
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(vqa::cdiv(total, 256)), dim3(256), 0, s, ids, table, out, tokens,
                     d / 4, vocab, dr);
  return vqa::check_launch("vqa_embedding_fwd");
}

extern "C" int vqa_rng_advance(unsigned* rng, hipStream_t s) {
  VQA_REQUIRE(rng, "vqa_rng_advance: null state");
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, s, rng);
  return vqa::check_launch("vqa_rng_advance");
}

extern "C" int vqa_dropout_mask(const vqa_dropout* d, float* out, long long n, hipStream_t s) {
  VQA_REQUIRE(d && out && n > 0 && n <= (1ll << 32), "vqa_dropout_mask: bad arguments");
  VQA_REQUIRE(d->p >= 0.f && d->p < 1.f, "vqa_dropout_mask: p must be in [0, 1)");
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(vqa::cdiv(n, 256)), dim3(256), 0, s, *d, out, (long)n);
  return vqa::check_launch("vqa_dropout_mask");
}

extern "C" int vqa_embedding_zero_rows(long long* ids_prev, const long long* ids_cur, int tokens, float* dtable,
                                       int d, int vocab, hipStream_t s) {
  VQA_REQUIRE(ids_prev && dtable && tokens > 0 && d % 4 == 0 && vocab > 0, "vqa_embedding_zero_rows: bad arguments");
  hipLaunchKernelGGL(embedding_zero_rows_kernel, dim3(tokens), dim3(256), 0, s, ids_prev, ids_cur, dtable, d, vocab);
  return vqa::check_launch("vqa_embedding_zero_rows");
}

extern "C" int vqa_embedding_bwd(const long long* ids, const float* dh, float* dtable, int tokens, int d, int vocab,
                                 int* ws, hipStream_t s) {
  // sort keys hold the position in 16 bits; one sort covers <= 16384 tokens (128 KiB of LDS).
  // Larger scatters (DP: world x B x L gathered tokens) run as consecutive slices of 16384
  // tokens in token order, each adding into the rows: deterministic, identical on every rank.
  VQA_REQUIRE(ids && dh && dtable && ws && tokens > 0 && d % 4 == 0, "vqa_embedding_bwd: bad arguments");
  constexpr int SLICE = 16384;
  for (int t0 = 0; t0 < tokens; t0 += SLICE) {
    const int n = tokens - t0 < SLICE ? tokens - t0 : SLICE;
    const long long* sid = ids + t0;
    if (n <= 1024)
      hipLaunchKernelGGL(embedding_sort_kernel<1>, dim3(1), dim3(1024), 0, s, sid, n, vocab, ws);
    else if (n <= 2048)
      hipLaunchKernelGGL(embedding_sort_kernel<2>, dim3(1), dim3(1024), 0, s, sid, n, vocab, ws);
    else if (n <= 4096)
      hipLaunchKernelGGL(embedding_sort_kernel<4>, dim3(1), dim3(1024), 0, s, sid, n, vocab, ws);
    else if (n <= 8192)
      hipLaunchKernelGGL(embedding_sort_kernel<8>, dim3(1), dim3(1024), 0, s, sid, n, vocab, ws);
    else
      hipLaunchKernelGGL(embedding_sort_kernel<16>, dim3(1), dim3(1024), 0, s, sid, n, vocab, ws);
    if (int rc = vqa::check_launch("vqa_embedding_bwd/sort")) return rc;
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(n, vqa::cdiv(d, 4 * EMB_CL)), dim3(EMB_RL * EMB_CL), 0, s,
                       dh + (long long)t0 * d, dtable, ws, n, d);
    if (int rc = vqa::check_launch("vqa_embedding_bwd")) return rc;
  }
  return VQA_OK;
}

// a batch-sum is a column sum over `batch` partial rows
extern "C" int vqa_batch_sum(const float* x, int batch, long long n, float* out, float beta, hipStream_t s) {
  VQA_REQUIRE(x && out && batch > 0 && n > 0 && n < (1ll << 31), "vqa_batch_sum: bad arguments");
  return vqa_colsum_partials(x, batch, n, (int)n, out, beta, s);
}

extern "C" int vqa_t5_relbias_fwd(const float* table, const int* bucket, float* out, int heads, int lq, int lk,
                                  hipStream_t s) {
  VQA_REQUIRE(table && bucket && out, "vqa_t5_relbias_fwd: bad arguments");
  hipLaunchKernelGGL(relbias_fwd_kernel, dim3(vqa::cdiv(heads * lq * lk, 256)), dim3(256), 0, s, table, bucket, out,
                     heads, lq * lk);
  return vqa::check_launch("vqa_t5_relbias_fwd");
}

extern "C" int vqa_t5_relbias_bwd(const float* dbias, const int* bucket, float* dtable, int heads, int lq, int lk,
                                  int nbuckets, hipStream_t s) {
  VQA_REQUIRE(dbias && bucket && dtable, "vqa_t5_relbias_bwd: bad arguments");
  hipLaunchKernelGGL(relbias_bwd_kernel, dim3(heads * nbuckets), dim3(256), 0, s, dbias, bucket, dtable, heads,
                     lq * lk);
  return vqa::check_launch("vqa_t5_relbias_bwd");
}

extern "C" int vqa_cast_f32_bf16(const float* x, void* y, long long n, hipStream_t s) {
  VQA_REQUIRE(x && y && n >= 0, "vqa_cast_f32_bf16: bad arguments");
  if (n == 0) return VQA_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(vqa::cdiv(vqa::cdiv(n, 4), 256)), dim3(256), 0, s, x, (bf16_t*)y,
                     (long)n);
  return vqa::check_launch("vqa_cast_f32_bf16");
}

// A kernel, not hipMemsetAsync: memset nodes captured into a hipGraph replayed
// garbage into the zeroed gradient buffers on the ROCm 7.0 runtime torch ships.
extern "C" int vqa_zero(void* p, long long bytes, hipStream_t s) {
  VQA_REQUIRE(p && bytes >= 0 && ((uintptr_t)p & 15) == 0 && bytes % 16 == 0,
              "vqa_zero: pointer and size must be 16-byte aligned");
  if (bytes == 0) return VQA_OK;
  const long n16 = (long)(bytes / 16);
  const int grid = (int)((n16 + 255) / 256 < 8192 ? (n16 + 255) / 256 : 8192);
  hipLaunchKernelGGL(zero_kernel, dim3(grid), dim3(256), 0, s, (uint4*)p, n16);
  return vqa::check_launch("vqa_zero");
}

// A kernel, not hipMemcpyAsync: inside a captured step a device-to-device copy would be the
// graph's only non-kernel node (a runtime blit node); the step graphs stay kernel-only.
extern "C" int vqa_copy(void* dst, const void* src, long long bytes, hipStream_t s) {
  VQA_REQUIRE(dst && src && bytes >= 0 && ((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0 && bytes % 16 == 0,
              "vqa_copy: pointers and size must be 16-byte aligned");
  if (bytes == 0) return VQA_OK;
  const long n16 = (long)(bytes / 16);
  const int grid = (int)((n16 + 255) / 256 < 8192 ? (n16 + 255) / 256 : 8192);
  hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n16);
  return vqa::check_launch("vqa_copy");
}

// Tap-shifted copies of an NHWC bf16 map (ConvTranspose2d scaler dW as a tap-batched GEMM):
// out[t][(b*h + y)*w + x][:] = in[b][y - ky + pad][x - kx + pad][:], t = ky*kw + kx, zero
// outside the map.  blockIdx.y = tap; one thread per 16-byte chunk (8 channels), 32-bit
// index math (the host bounds rows * c8 below 2^31).
__global__ __launch_bounds__(256) void tap_shift_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, int h,
                                                        int w, int c8, int kw, int pad, int per_tap) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= per_tap) return;
  const int t = blockIdx.y, ky = t / kw, kx = t - ky * kw;
  const int pos = i / c8, ch = i - pos * c8;
  const int hw = h * w, b = pos / hw, yx = pos - b * hw;
  const int y = yx / w, x = yx - y * w;
  const int sy = y - ky + pad, sx = x - kx + pad;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (sy >= 0 && sy < h && sx >= 0 && sx < w) v = in[(b * hw + sy * w + sx) * c8 + ch];
  out[(long)t * per_tap + i] = v;
}

extern "C" int vqa_tap_shift(const void* in, void* out, int n, int h, int w, int c, int kh, int kw, int pad,
                             hipStream_t s) {
  VQA_REQUIRE(in && out && n > 0 && h > 0 && w > 0 && c > 0 && kh > 0 && kw > 0 && pad >= 0 && c % 8 == 0 &&
                  ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0,
              "vqa_tap_shift: bad arguments (c a multiple of 8, 16-byte aligned maps)");
  const long per_tap = (long)n * h * w * (c / 8);
  VQA_REQUIRE(per_tap < (1l << 31) && kh * kw <= 65535, "vqa_tap_shift: map too large");
  hipLaunchKernelGGL(tap_shift_kernel, dim3((unsigned)((per_tap + 255) / 256), (unsigned)(kh * kw)), dim3(256), 0, s,
                     (const uint4*)in, (uint4*)out, h, w, c / 8, kw, pad, (int)per_tap);
  return vqa::check_launch("vqa_tap_shift");
}
