// e4m3 (OCP fp8) forward weight GEMMs of BASELINE config 5 ("fp8 MFMA weights"), and the
// per-row quantisation that feeds them.
//
//   Y = (X8 W8^T) * sx[m] * sw[n]  (+ the usual fused epilogue)
//
// X8 / W8 are row-wise e4m3 quantisations of the activation [M, K] and of the Linear weight
// [N, K] (each row scaled so its largest magnitude is 448, the e4m3 maximum); the row scales
// factor out of the K sum exactly, so the only rounding beyond the fp32 accumulation is the
// quantisation itself.  The tile body is gemm_body<..., F8> (gemm_body.h): the operands ride
// the same LDS-DMA ring as bf16 (a 128-B image row = 128 fp8 k instead of 64 bf16 k, i.e. half
// the L2 -> LDS bytes per FLOP, the k-loop's bound), and every 64-deep step is
// one v_mfma_scale_f32_32x32x64_f8f6f4 at unit block scales (2x the bf16 MFMA rate).
#include "gemm_body.h"

namespace {

template <int BM, int BN, int ST, int NWM, int NWN, int BKT = BK>
struct F8Tile {
  static int run(GemmParams& P, int batch, hipStream_t s) {
    return launch<BM, BN, ST, NWM, NWN, true, true, false, false, BKT, true>(P, batch, s);
  }
};

// e4m3 of an fp32 value already scaled into [-448, 448]: round to nearest even (the
// hardware conversion; torch.float8_e4m3fn rounds the same way)
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

// One wave per row: amax over the row, scale = amax / 448 (1 for an all-zero row),
// q = e4m3(x / scale).  x fp32 or bf16, cols % 8 == 0.
template <bool BF>
__global__ __launch_bounds__(256) void quant_rows_kernel(const void* __restrict__ x, long ldx, int rows, int cols,
                                                         uint8_t* __restrict__ q, long ldq, float* __restrict__ scale) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= rows) return;
  auto load8 = [&](int c, float (&v)[8]) {
    if constexpr (BF) {
      const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(x) + (long)row * ldx + c);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = bf2f((t & 1) ? (w[t >> 1] >> 16) : (w[t >> 1] & 0xffff));
    } else {
      const float* p = reinterpret_cast<const float*>(x) + (long)row * ldx + c;
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
  };
  float amax = 0.f;
  for (int c = l * 8; c < cols; c += 512) {
    float v[8];
    load8(c, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) amax = fmaxf(amax, fabsf(v[t]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  // correctly rounded divisions (__fdiv_rn): the compiler may not turn them into reciprocal
  // multiplies, so the scale and the quantised bytes are exactly torch's amax / 448, x / scale
  const float s = amax > 0.f ? __fdiv_rn(amax, 448.f) : 1.f;
  if (l == 0) scale[row] = s;
  for (int c = l * 8; c < cols; c += 512) {
    float v[8];
    load8(c, v);
    uint2 o;
    o.x = pack4_fp8(__fdiv_rn(v[0], s), __fdiv_rn(v[1], s), __fdiv_rn(v[2], s), __fdiv_rn(v[3], s));
    o.y = pack4_fp8(__fdiv_rn(v[4], s), __fdiv_rn(v[5], s), __fdiv_rn(v[6], s), __fdiv_rn(v[7], s));
    *reinterpret_cast<uint2*>(q + (long)row * ldq + c) = o;
  }
}

}  // namespace

// called by vqa_gemm for fp8 descriptors (gemm.hip has validated the descriptor and filled P;
// both translation units see the same GemmParams layout from gemm_common.h)
int vqa_gemm_fp8_dispatch(void* pp, int batch, int config, hipStream_t s) {
  GemmParams& P = *static_cast<GemmParams*>(pp);
  switch (config) {
    case 1: return F8Tile<128, 128, 3, 2, 2>::run(P, batch, s);
    case 2: return F8Tile<128, 64, 4, 2, 2>::run(P, batch, s);
    case 3: return F8Tile<64, 64, 4, 2, 2>::run(P, batch, s);
    case 5: return F8Tile<64, 64, 3, 2, 2>::run(P, batch, s);
    case 6: return F8Tile<128, 64, 2, 2, 2>::run(P, batch, s);
    case 7: return F8Tile<64, 128, 2, 2, 2>::run(P, batch, s);
    case 8: return F8Tile<128, 128, 2, 2, 2>::run(P, batch, s);
    case 9: return F8Tile<256, 128, 2, 4, 2>::run(P, batch, s);
    case 10: return F8Tile<128, 256, 2, 2, 4>::run(P, batch, s);
    case 12: return F8Tile<256, 128, 3, 4, 2>::run(P, batch, s);
    case 21: return F8Tile<64, 64, 2, 2, 2, 128>::run(P, batch, s);
    case 22: return F8Tile<64, 128, 2, 2, 2, 128>::run(P, batch, s);
    case 23: return F8Tile<128, 64, 2, 2, 2, 128>::run(P, batch, s);
    case 0: case 4: return F8Tile<64, 64, 2, 2, 2>::run(P, batch, s);
    default:   // 11 (256x256): its double-buffered 32-B fragments would spill; 13-20: bf16 / patch only
      return vqa::fail(VQA_ERR_INVALID, "vqa_gemm(fp8): tile config %d has no e4m3 form", config);
  }
}

extern "C" int vqa_quant_rows_fp8(const void* x, int x_bf16, long long ldx, int rows, int cols, void* q, long long ldq,
                                  float* scale, hipStream_t s) {
  VQA_REQUIRE(x && q && scale && rows > 0 && cols > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldq % 8 == 0 &&
                  ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0,
              "vqa_quant_rows_fp8: bad arguments (cols, ldx, ldq multiples of 8; aligned pointers)");
  const dim3 grid(vqa::cdiv(rows, 4));
  if (x_bf16)
    hipLaunchKernelGGL(quant_rows_kernel<true>, grid, dim3(256), 0, s, x, (long)ldx, rows, cols, (uint8_t*)q, (long)ldq,
                       scale);
  else
    hipLaunchKernelGGL(quant_rows_kernel<false>, grid, dim3(256), 0, s, x, (long)ldx, rows, cols, (uint8_t*)q,
                       (long)ldq, scale);
  return vqa::check_launch("vqa_quant_rows_fp8");
}
