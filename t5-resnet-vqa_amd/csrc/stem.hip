// The frozen ResNet's stem convolution from an LDS input patch (r05).
//
// torchvision conv1 (7x7, stride 2, pad 3) + folded bn1 + ReLU, computed -- as the implicit
// GEMM of gemm.hip does -- as a 4x4 / stride-1 / pad-1 convolution over the space-to-depth image
// Z [n][hz][hz][16] bf16 (vqa_image_to_s2d16; weights [64][4][4][16], engine.stem_s2d_weight).
// The implicit GEMM gathers every input pixel through L2 once per tap (16x: the stem's 64-KB A
// slab per 128-pixel tile, fill-bound at 88 us for B = 64, 224^2).  Here a workgroup owns an
// 8 x 16 block of output pixels (128 = four 32-pixel MFMA row blocks) and all 64 channels: the
// 11 x 19-pixel input patch (6.7 KB) is staged in LDS once, the weights stay in registers (each
// wave's 32 channels x 256 k: 16 fragments), and the 16 taps read their A fragments from the
// patch at a per-tap pixel offset.  k = tap * 16 + c with tap = kh * 4 + kw, accumulated tap by
// tap in that order, and the epilogue is the GEMM's (acc + bias, ReLU, bf16): the output equals
// the implicit-GEMM path's bit for bit (tests/test_kernels_gpu.py).
#include "common.h"

#include <algorithm>

namespace {

typedef int i32x4s_t __attribute__((ext_vector_type(4)));

constexpr int STEM_CUS = 256;                  // MI355X compute units (the persistent grids' size)
constexpr int SR = 8, SC = 16;                 // output rows x columns per workgroup
constexpr int PR = SR + 3, PC = SC + 3;        // input patch rows x columns (4 x 4 taps, pad 1)
constexpr int PATCH_BYTES = PR * PC * 32;      // 32 B per pixel: 16 bf16 channels

// byte offset of half h (channels 8h..8h+7) of patch pixel (pr, pc); the halves of every other
// group of 8 columns are swapped, so the 16 lanes of a ds_read_b128 phase (16 consecutive
// pixels, one half) fall on distinct banks
__device__ __forceinline__ int patch_off(int pr, int pc, int h) {
  return (pr * PC + pc) * 32 + 16 * (h ^ ((pc >> 3) & 1));
}

constexpr int OUT_STRIDE = 144;                 // LDS bytes per staged output pixel (64 bf16 + 16 B pad)

__global__ __launch_bounds__(256) void stem_patch_kernel(const uint4* __restrict__ z, const bf16_t* __restrict__ w,
                                                         const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                         int hz, int oh, int ow, int ntiles) {
  __shared__ __attribute__((aligned(16))) char patch[PATCH_BYTES];
  __shared__ __attribute__((aligned(16))) char outs[SR * SC * OUT_STRIDE];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int wm = wv >> 1, wn = wv & 1;         // pixel blocks 2wm, 2wm+1; channels 32wn..32wn+31
  const int tx_n = ow / SC, per_img = tx_n * (oh / SR);

  // weights (once per workgroup: the grid is persistent): lane (n = 32wn + l%32, k half l/32)
  // holds its 8 k of every tap (16 x 16 B)
  i32x4s_t fb[16];
  {
    const bf16_t* wp = w + (long)(wn * 32 + (l & 31)) * 256 + 8 * (l >> 5);
#pragma unroll
    for (int t = 0; t < 16; ++t) fb[t] = *reinterpret_cast<const i32x4s_t*>(wp + t * 16);
  }
  // bias of the lane's 16 output channels: 8g + 4(l/32) + (0..3) of its 32-channel block
  float4 bs[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bs[g] = *reinterpret_cast<const float4*>(bias + wn * 32 + 8 * g + 4 * (l >> 5));
  int r[2], c[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = (2 * wm + i) * 32 + (l & 31);  // local pixel of this lane's A row
    r[i] = q / SC;
    c[i] = q % SC;
  }

  // XCD-contiguous tiles: workgroup b works through its XCD's range (gemm_body's split of the
  // tile ids) with the stride of that XCD's workgroups, so neighbouring 8 x 16 blocks -- whose
  // patches share rows -- are in flight together on one L2
  const int xcd = blockIdx.x & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int hi = lo + q8 + (xcd < r8 ? 1 : 0);
  const int wstride = (gridDim.x - xcd + 7) >> 3; // workgroups on this XCD
  for (int tile = lo + (blockIdx.x >> 3); tile < hi; tile += wstride) {
    const int img = tile / per_img, rem = tile - img * per_img;
    const int oy0 = (rem / tx_n) * SR, ox0 = (rem % tx_n) * SC;
    // the input patch: 11 x 19 pixels x 2 halves = 418 16-B pieces, zero outside the image
    const uint4* zi = z + (long)img * hz * hz * 2;
    __syncthreads();                             // the previous tile's patch / output reads are done
    for (int u = tid; u < PR * PC * 2; u += 256) {
      const int pr = u / (PC * 2), rr = u - pr * (PC * 2), pc = rr >> 1, h = rr & 1;
      const int iy = oy0 - 1 + pr, ix = ox0 - 1 + pc;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (iy >= 0 && iy < hz && ix >= 0 && ix < hz) v = zi[((long)iy * hz + ix) * 2 + h];
      *reinterpret_cast<uint4*>(patch + patch_off(pr, pc, h)) = v;
    }
    __syncthreads();

    f32x16_t acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int kh = t >> 2, kw = t & 3;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const i32x4s_t fa = *reinterpret_cast<const i32x4s_t*>(patch + patch_off(r[i] + kh, c[i] + kw, l >> 5));
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[t]),
                                                         __builtin_bit_cast(bf16x8_t, fa), acc[i], 0, 0, 0);
      }
    }

    // epilogue (the GEMM's: acc * 1 + bias, ReLU, bf16) staged in LDS: lane = pixel l%32 of its
    // row block, channels 8g + 4(l/32) + t; then every thread stores whole 16-B pieces of
    // 128-B pixel rows (each output row of the block is 2 KB contiguous)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      char* op = outs + ((2 * wm + i) * 32 + (l & 31)) * OUT_STRIDE + (wn * 32 + 4 * (l >> 5)) * 2;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float v0 = fmaxf(acc[i][4 * g] * 1.f + bs[g].x, 0.f), v1 = fmaxf(acc[i][4 * g + 1] * 1.f + bs[g].y, 0.f);
        const float v2 = fmaxf(acc[i][4 * g + 2] * 1.f + bs[g].z, 0.f), v3 = fmaxf(acc[i][4 * g + 3] * 1.f + bs[g].w, 0.f);
        uint2 o;
        o.x = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
        o.y = (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16);
        *reinterpret_cast<uint2*>(op + 16 * g) = o;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SR * SC * 8 / 256; ++k) {
      const int u = tid + 256 * k, px = u >> 3, j = u & 7;
      const int ry = px / SC, rx = px % SC;
      const uint4 v = *reinterpret_cast<const uint4*>(outs + px * OUT_STRIDE + 16 * j);
      *reinterpret_cast<uint4*>(y + (((long)img * oh + oy0 + ry) * ow + ox0 + rx) * 64 + 8 * j) = v;
    }
  }
}


// ---------------------------------------------------------------- stem + maxpool, fused (r05)
// torchvision conv1 + bn1 + ReLU + MaxPool2d(3, 2, 1) in one pass: a workgroup owns a 4 x 8 block
// of POOLED pixels, computes the 9 x 17 stem pixels their 3 x 3 / stride-2 windows cover (the
// 153 of five 32-pixel MFMA row blocks; a one-pixel halo recomputed by the neighbouring block)
// from a 12 x 20-pixel LDS patch, rounds them to bf16 (the stem's output precision), and writes
// only the max-pooled pixels: the 103 MB stem map (B = 64, 224^2) is never stored or re-read.
// Windows skip stem pixels outside the map (the pool's -inf padding).  The next tile's patch is
// loaded into registers while this tile computes.  Bit-identical to vqa_stem_s2d_conv followed
// by vqa_maxpool3x3s2_nhwc.
constexpr int PY = 4, PX = 8;                    // pooled rows x columns per workgroup
constexpr int FR = 2 * PY + 1, FC = 2 * PX + 1;  // stem rows x columns computed (9 x 17)
constexpr int FPR = FR + 3, FPC = FC + 3;        // input patch (12 x 20)
constexpr int FPIX = FR * FC;                    // 153 stem pixels in 5 row blocks of 32
constexpr int FSTR = 144;                        // LDS bytes per staged stem pixel (64 bf16 + 16 B pad)
constexpr int FPIECES = FPR * FPC * 2;           // 480 16-B patch pieces

__device__ __forceinline__ int fpatch_off(int pr, int pc, int h) {
  return (pr * FPC + pc) * 32 + 16 * (h ^ ((pc >> 3) & 1));
}

// IMG: the patch is built from the fp32 NCHW image itself (the space-to-depth transform of
// vqa_image_to_s2d16 applied while staging: Z[u][v][(2p+q)*3+c] = bf16(img[c][2u+p-1][2v+q-1]), 0
// outside the image, channels 12..15 zero), so the s2d image is neither written nor read
template <bool IMG>
__global__ __launch_bounds__(256) void stem_pool_kernel(const void* __restrict__ src, const bf16_t* __restrict__ w,
                                                        const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                        int hz, int oh, int ph, int ntiles) {
  const uint4* z = reinterpret_cast<const uint4*>(src);
  const float* img = reinterpret_cast<const float*>(src);
  const int H = oh * 2;                          // image height = width (IMG)
  __shared__ __attribute__((aligned(16))) char patch[FPR * FPC * 32];
  __shared__ __attribute__((aligned(16))) char stem[5 * 32 * FSTR];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int wn = wv & 1;                         // channels 32wn..32wn+31
  const int b0 = (wv >> 1) ? 3 : 0, nb = (wv >> 1) ? 2 : 3;   // stem row blocks: {0,1,2} | {3,4}
  const int tx_n = ph / PX, per_img = tx_n * (ph / PY);

  i32x4s_t fb[16];
  {
    const bf16_t* wp = w + (long)(wn * 32 + (l & 31)) * 256 + 8 * (l >> 5);
#pragma unroll
    for (int t = 0; t < 16; ++t) fb[t] = *reinterpret_cast<const i32x4s_t*>(wp + t * 16);
  }
  float4 bs[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bs[g] = *reinterpret_cast<const float4*>(bias + wn * 32 + 8 * g + 4 * (l >> 5));
  int r[3], c[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    int q = (b0 + i) * 32 + (l & 31);
    q = q < FPIX ? q : FPIX - 1;                 // padding slots read a real pixel (result unused)
    r[i] = q / FC;
    c[i] = q % FC;
  }

  const int xcd = blockIdx.x & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
  const int lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int hi = lo + q8 + (xcd < r8 ? 1 : 0);
  const int wstride = (gridDim.x - xcd + 7) >> 3;

  // this thread's patch pieces of a tile, into registers (zero outside the image):
  // Z: 16-B pieces of the s2d image; IMG: one image column of one plane, every other row
  // (thread t < 240: column cc = t % 40, plane c, row parity par) -> 12 bf16, i.e. one s2d
  // channel of one patch column over the 12 patch rows
  const int icc = tid % (2 * FPC), ic = (tid / (2 * FPC)) % 3, ipar = tid / (6 * FPC);
  const int ich = (2 * ipar + (icc & 1)) * 3 + ic;
  const int ioff = fpatch_off(0, icc >> 1, ich >> 3) + (ich & 7) * 2;
  auto load = [&](int tile, uint4 (&v)[2], float (&f)[IMG ? FPR : 1]) {
    const int im = tile / per_img, rem = tile - im * per_img;
    const int iy0 = 2 * ((rem / tx_n) * PY) - 2, ix0 = 2 * ((rem % tx_n) * PX) - 2;
    if constexpr (IMG) {
      const int C = 2 * ix0 - 1 + icc, R0 = 2 * iy0 - 1 + ipar;
      const float* ii = img + ((long)im * 3 + ic) * H * H + C;
      const bool colok = tid < 12 * FPC && C >= 0 && C < H;
#pragma unroll
      for (int j = 0; j < FPR; ++j) {            // raw: converted at the LDS store, so the
        const int R = R0 + 2 * j;                // loads stay in flight across the compute
        f[j] = (colok && R >= 0 && R < H) ? ii[(long)R * H] : 0.f;
      }
    } else {
      const uint4* zi = z + (long)im * hz * hz * 2;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int u = tid + 256 * k;
        v[k] = make_uint4(0u, 0u, 0u, 0u);
        if (u < FPIECES) {
          const int pr = u / (FPC * 2), rr = u - pr * (FPC * 2), pc = rr >> 1, h = rr & 1;
          const int iy = iy0 + pr, ix = ix0 + pc;
          if (iy >= 0 && iy < hz && ix >= 0 && ix < hz) v[k] = zi[((long)iy * hz + ix) * 2 + h];
        }
      }
    }
  };
  if constexpr (IMG) {                           // s2d channels 12..15 are zero: written once
    if (tid < FPR * FPC)
      *reinterpret_cast<uint2*>(patch + fpatch_off(tid / FPC, tid % FPC, 1) + 8) = make_uint2(0u, 0u);
  }
  uint4 pv[2];
  float pf[IMG ? FPR : 1];
  int tile = lo + (blockIdx.x >> 3);
  if (tile < hi) load(tile, pv, pf);
  for (; tile < hi; tile += wstride) {
    const int img = tile / per_img, rem = tile - img * per_img;
    const int py0 = (rem / tx_n) * PY, px0 = (rem % tx_n) * PX;
    __syncthreads();                             // the previous tile's patch / stem reads are done
    if constexpr (IMG) {
      if (tid < 12 * FPC) {
#pragma unroll
        for (int j = 0; j < FPR; ++j) *reinterpret_cast<bf16_t*>(patch + ioff + j * FPC * 32) = f2bf(pf[j]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int u = tid + 256 * k;
        if (u < FPIECES) {
          const int pr = u / (FPC * 2), rr = u - pr * (FPC * 2), pc = rr >> 1, h = rr & 1;
          *reinterpret_cast<uint4*>(patch + fpatch_off(pr, pc, h)) = pv[k];
        }
      }
    }
    __syncthreads();
    if (tile + wstride < hi) load(tile + wstride, pv, pf);   // in flight while this tile computes

    f32x16_t acc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int kh = t >> 2, kw = t & 3;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (i < nb) {
          const i32x4s_t fa = *reinterpret_cast<const i32x4s_t*>(patch + fpatch_off(r[i] + kh, c[i] + kw, l >> 5));
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[t]),
                                                           __builtin_bit_cast(bf16x8_t, fa), acc[i], 0, 0, 0);
        }
      }
    }
    // stem epilogue (acc * 1 + bias, ReLU, bf16) into the LDS stem tile
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < nb) {
        char* op = stem + ((b0 + i) * 32 + (l & 31)) * FSTR + (wn * 32 + 4 * (l >> 5)) * 2;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v0 = fmaxf(acc[i][4 * g] * 1.f + bs[g].x, 0.f), v1 = fmaxf(acc[i][4 * g + 1] * 1.f + bs[g].y, 0.f);
          const float v2 = fmaxf(acc[i][4 * g + 2] * 1.f + bs[g].z, 0.f), v3 = fmaxf(acc[i][4 * g + 3] * 1.f + bs[g].w, 0.f);
          uint2 o;
          o.x = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
          o.y = (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16);
          *reinterpret_cast<uint2*>(op + 16 * g) = o;
        }
      }
    }
    __syncthreads();
    // 3 x 3 / stride-2 max over the stem pixels inside the map: thread = (pooled pixel, 8 channels)
    {
      const int pp = tid >> 3, j = tid & 7, ly = pp / PX, lx = pp % PX;
      const int sr0 = 2 * (py0 + ly) - 1, sc0 = 2 * (px0 + lx) - 1;   // stem row / col of local (2ly, 2lx)
      float m[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        if (sr0 + dy < 0 || sr0 + dy >= oh) continue;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          if (sc0 + dx < 0 || sc0 + dx >= oh) continue;
          const uint4 u = *reinterpret_cast<const uint4*>(stem + ((2 * ly + dy) * FC + 2 * lx + dx) * FSTR + 16 * j);
          const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            m[2 * e] = fmaxf(m[2 * e], bf2f((bf16_t)(wd[e] & 0xffff)));
            m[2 * e + 1] = fmaxf(m[2 * e + 1], bf2f((bf16_t)(wd[e] >> 16)));
          }
        }
      }
      uint4 o;
      o.x = (uint32_t)f2bf(m[0]) | ((uint32_t)f2bf(m[1]) << 16);
      o.y = (uint32_t)f2bf(m[2]) | ((uint32_t)f2bf(m[3]) << 16);
      o.z = (uint32_t)f2bf(m[4]) | ((uint32_t)f2bf(m[5]) << 16);
      o.w = (uint32_t)f2bf(m[6]) | ((uint32_t)f2bf(m[7]) << 16);
      *reinterpret_cast<uint4*>(y + (((long)img * ph + py0 + ly) * ph + px0 + lx) * 64 + 8 * j) = o;
    }
  }
}

}  // namespace

extern "C" int vqa_stem_s2d_conv(const void* z, const void* w, const float* bias, void* y, int n, int hz, int oh,
                                 hipStream_t s) {
  VQA_REQUIRE(z && w && bias && y && n > 0, "vqa_stem_s2d_conv: null argument");
  VQA_REQUIRE(oh % SR == 0 && oh % SC == 0 && hz == oh + 1, "vqa_stem_s2d_conv: oh %% 16 == 0 and hz == oh + 1 needed");
  VQA_REQUIRE(((uintptr_t)z & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)bias & 15) == 0 &&
                  ((uintptr_t)y & 15) == 0,
              "vqa_stem_s2d_conv: 16-B aligned buffers needed");
  const int ntiles = n * (oh / SR) * (oh / SC);
  // persistent: two workgroups per CU of the MI355X's 256 (the kernel's occupancy: 161 VGPRs + 32
  // AGPRs), a multiple of 8 XCDs.  (No runtime query here: this launch is also captured into the
  // step graph, and a device-attribute call inside a stream capture is best avoided.)
  const int grid = std::min(ntiles, 2 * STEM_CUS) / 8 * 8 > 0 ? std::min(ntiles, 2 * STEM_CUS) / 8 * 8 : ntiles;
  hipLaunchKernelGGL(stem_patch_kernel, dim3(grid), dim3(256), 0, s, (const uint4*)z, (const bf16_t*)w, bias,
                     (bf16_t*)y, hz, oh, oh, ntiles);
  return vqa::check_launch("vqa_stem_s2d_conv");
}

extern "C" int vqa_stem_pool_s2d(const void* z, const void* w, const float* bias, void* y, int n, int hz, int oh,
                                 hipStream_t s) {
  VQA_REQUIRE(z && w && bias && y && n > 0, "vqa_stem_pool_s2d: null argument");
  const int ph = oh / 2;
  VQA_REQUIRE(oh % 2 == 0 && ph % PY == 0 && ph % PX == 0 && hz == oh + 1,
              "vqa_stem_pool_s2d: oh even, oh / 2 a multiple of 8, hz == oh + 1 needed");
  VQA_REQUIRE(((uintptr_t)z & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)bias & 15) == 0 &&
                  ((uintptr_t)y & 15) == 0,
              "vqa_stem_pool_s2d: 16-B aligned buffers needed");
  const int ntiles = n * (ph / PY) * (ph / PX);
  const int grid = std::min(ntiles, 2 * STEM_CUS) / 8 * 8 > 0 ? std::min(ntiles, 2 * STEM_CUS) / 8 * 8 : ntiles;
  hipLaunchKernelGGL(stem_pool_kernel<false>, dim3(grid), dim3(256), 0, s, z, (const bf16_t*)w, bias, (bf16_t*)y,
                     hz, oh, ph, ntiles);
  return vqa::check_launch("vqa_stem_pool_s2d");
}

extern "C" int vqa_stem_pool_img(const float* img, const void* w, const float* bias, void* y, int n, int h,
                                 hipStream_t s) {
  VQA_REQUIRE(img && w && bias && y && n > 0, "vqa_stem_pool_img: null argument");
  const int oh = h / 2, ph = oh / 2;
  VQA_REQUIRE(h % 4 == 0 && ph % PY == 0 && ph % PX == 0, "vqa_stem_pool_img: h a multiple of 32 needed");
  VQA_REQUIRE(((uintptr_t)w & 15) == 0 && ((uintptr_t)bias & 15) == 0 && ((uintptr_t)y & 15) == 0,
              "vqa_stem_pool_img: 16-B aligned weights, bias and output needed");
  const int ntiles = n * (ph / PY) * (ph / PX);
  const int grid = std::min(ntiles, 2 * STEM_CUS) / 8 * 8 > 0 ? std::min(ntiles, 2 * STEM_CUS) / 8 * 8 : ntiles;
  hipLaunchKernelGGL(stem_pool_kernel<true>, dim3(grid), dim3(256), 0, s, img, (const bf16_t*)w, bias, (bf16_t*)y,
                     oh + 1, oh, ph, ntiles);
  return vqa::check_launch("vqa_stem_pool_img");
}
