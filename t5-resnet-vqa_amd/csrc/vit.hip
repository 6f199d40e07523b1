// Data-movement kernels of BASELINE config 4, the ViT-base + T5 encoder-decoder path
// (model/vit_vqa_model.py:127-227, `VitVQAModel`): the patch embedding's im2col, row
// gathers / scatters (CLS rows, the concat of the fusing layer, the answer-token gather)
// and the T5 decoder's cross-attention over its single encoder token.  All HBM-bound
// and small next to the GEMMs; one thread per 16-byte piece or per output column.
#include "common.h"

namespace {

// out[(b*np + py*nx + px)][c*P*P + ky*P + kx] = bf16(img[b][c][py*P + ky][px*P + kx]):
// Conv2d(3, 768, 16, stride 16) weights [768][3][16][16] flatten in exactly this K order.
// One thread per 8 consecutive k (8 pixels of one image row).
__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ img, bf16_t* __restrict__ out,
                                                       int n, int h, int w, int P) {
  const int nx = w / P, ny = h / P, K = 3 * P * P, per = K / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)n * ny * nx * per;
  if (idx >= total) return;
  const long row = idx / per;
  const int k0 = (int)(idx - row * per) * 8;
  const int b = (int)(row / (ny * nx)), pp = (int)(row - (long)b * ny * nx);
  const int py = pp / nx, px = pp - py * nx;
  const int c = k0 / (P * P), rem = k0 - c * P * P, ky = rem / P, kx = rem - ky * P;
  const float* src = img + (((long)b * 3 + c) * h + py * P + ky) * w + px * P + kx;
  const float4 a = *reinterpret_cast<const float4*>(src);
  const float4 d = *reinterpret_cast<const float4*>(src + 4);
  uint4 u;
  u.x = (uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16);
  u.y = (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16);
  u.z = (uint32_t)f2bf(d.x) | ((uint32_t)f2bf(d.y) << 16);
  u.w = (uint32_t)f2bf(d.z) | ((uint32_t)f2bf(d.w) << 16);
  *reinterpret_cast<uint4*>(out + row * K + k0) = u;
}

// dst row r <-> src row (idx ? idx[r] : offset + r*stride), 16 B per thread;
// scatter = 0: dst[r] = src[row(r)]; scatter = 1: dst[row(r)] = src[r]
__global__ __launch_bounds__(256) void rows_kernel(const char* __restrict__ src, long lds, const long long* idx,
                                                   long stride, long offset, char* __restrict__ dst, long ldd,
                                                   int rows, int chunks, int scatter) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * chunks) return;
  const int r = (int)(i / chunks), c = (int)(i - (long)r * chunks);
  const long other = idx ? idx[r] : offset + (long)r * stride;
  const long sr = scatter ? r : other, dr = scatter ? other : r;
  *reinterpret_cast<uint4*>(dst + dr * ldd + c * 16) = *reinterpret_cast<const uint4*>(src + sr * lds + c * 16);
}

// out[b] = b*len + max{j : mask[b][j] == 1} (0 when none): the answer-token row of
// vit_vqa_model.py:208-209 (torch.max over where(mask == 1, arange, 0))
__global__ __launch_bounds__(256) void last_index_kernel(const long long* __restrict__ mask, int batch, int len,
                                                         long long* __restrict__ out) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= batch) return;
  int last = 0;
  for (int j = 0; j < len; ++j)
    if (mask[(long)b * len + j] == 1) last = j;
  out[b] = (long long)b * len + last;
}

// T5 EncDecAttention over ONE encoder token (vit_vqa_model.py:199-205: the fused embedding
// unsqueezed to [B, 1, 768]): softmax over a single key is 1, so the context of query i,
// head h is drop(1) * v[b, h] (TF modeling_t5 T5Attention dropout on the weights, element
// index ((b*H + h)*len + i) of the [B, H, len, 1] weights; no gradient reaches q or k).
__global__ __launch_bounds__(256) void xattn1_fwd_kernel(const bf16_t* __restrict__ v, long ldv,
                                                         bf16_t* __restrict__ out, long ldo, int batch, int len,
                                                         int heads, int dh, vqa_dropout drop) {
  const int D = heads * dh;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;         // one thread per 8 columns of one row
  const int per = D / 8;
  if (i >= (long)batch * len * per) return;
  const long row = i / per;
  const int c0 = (int)(i - row * per) * 8;
  const int b = (int)(row / len), q = (int)(row - (long)b * len), h = c0 / dh;
  const DropK dk = drop_init(drop);
  const float m = dk.on ? drop_mul(dk, (uint32_t)(((long)b * heads + h) * len + q)) : 1.f;
  uint4 u = *reinterpret_cast<const uint4*>(v + (long)b * ldv + c0);
  if (m != 1.f) {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      w[t] = (uint32_t)f2bf(bf2f(w[t] & 0xffff) * m) | ((uint32_t)f2bf(bf2f(w[t] >> 16) * m) << 16);
    u = make_uint4(w[0], w[1], w[2], w[3]);
  }
  *reinterpret_cast<uint4*>(out + row * ldo + c0) = u;
}

// dv[b][c] = sum_i drop(b, h(c), i) * dctx[b*len + i][c], in query order (deterministic)
__global__ __launch_bounds__(256) void xattn1_bwd_kernel(const bf16_t* __restrict__ dctx, long ldd,
                                                         float* __restrict__ dv32, bf16_t* __restrict__ dv16,
                                                         long lddv, int batch, int len, int heads, int dh,
                                                         vqa_dropout drop) {
  const int D = heads * dh;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)batch * D) return;
  const int b = (int)(i / D), c = (int)(i - (long)b * D), h = c / dh;
  const DropK dk = drop_init(drop);
  float s = 0.f;
  for (int q = 0; q < len; ++q) {
    const float m = dk.on ? drop_mul(dk, (uint32_t)(((long)b * heads + h) * len + q)) : 1.f;
    s += m * bf2f(dctx[((long)b * len + q) * ldd + c]);
  }
  if (dv32) dv32[(long)b * lddv + c] = s;
  if (dv16) dv16[(long)b * lddv + c] = f2bf(s);
}

}  // namespace

extern "C" int vqa_vit_patchify(const float* img, void* out, int n, int h, int w, int patch, hipStream_t s) {
  VQA_REQUIRE(img && out && n > 0 && patch > 0 && patch % 8 == 0 && h % patch == 0 && w % patch == 0 &&
                  ((uintptr_t)img & 15) == 0 && ((uintptr_t)out & 15) == 0,
              "vqa_vit_patchify: bad arguments (patch %% 8, H and W multiples of the patch, 16-B aligned)");
  const long total = (long)n * (h / patch) * (w / patch) * (3 * patch * patch / 8);
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)vqa::cdiv(total, 256)), dim3(256), 0, s, img, (bf16_t*)out, n,
                     h, w, patch);
  return vqa::check_launch("vqa_vit_patchify");
}

static int rows_common(const void* src, long long lds, const long long* idx, long long stride, long long offset,
                       void* dst, long long ldd, int rows, int cols, int esz, int scatter, hipStream_t s,
                       const char* name) {
  VQA_REQUIRE(src && dst && rows >= 0 && cols > 0 && (esz == 2 || esz == 4) && (cols * esz) % 16 == 0 &&
                  (lds * esz) % 16 == 0 && (ldd * esz) % 16 == 0 && ((uintptr_t)src & 15) == 0 &&
                  ((uintptr_t)dst & 15) == 0,
              "%s: bad arguments (16-byte rows and strides)", name);
  if (rows == 0) return VQA_OK;
  const int chunks = cols * esz / 16;
  hipLaunchKernelGGL(rows_kernel, dim3((unsigned)vqa::cdiv((long)rows * chunks, 256)), dim3(256), 0, s,
                     (const char*)src, (long)(lds * esz), idx, (long)stride, (long)offset, (char*)dst,
                     (long)(ldd * esz), rows, chunks, scatter);
  return vqa::check_launch(name);
}

extern "C" int vqa_gather_rows(const void* src, long long lds, const long long* idx, long long stride,
                               long long offset, void* dst, long long ldd, int rows, int cols, int esz,
                               hipStream_t s) {
  return rows_common(src, lds, idx, stride, offset, dst, ldd, rows, cols, esz, 0, s, "vqa_gather_rows");
}

extern "C" int vqa_scatter_rows(const void* src, long long lds, const long long* idx, long long stride,
                                long long offset, void* dst, long long ldd, int rows, int cols, int esz,
                                hipStream_t s) {
  return rows_common(src, lds, idx, stride, offset, dst, ldd, rows, cols, esz, 1, s, "vqa_scatter_rows");
}

extern "C" int vqa_last_index(const long long* mask, int batch, int len, long long* out, hipStream_t s) {
  VQA_REQUIRE(mask && out && batch > 0 && len > 0, "vqa_last_index: bad arguments");
  hipLaunchKernelGGL(last_index_kernel, dim3(vqa::cdiv(batch, 256)), dim3(256), 0, s, mask, batch, len, out);
  return vqa::check_launch("vqa_last_index");
}

extern "C" int vqa_xattn1_fwd(const void* v, long long ldv, void* out, long long ldo, int batch, int len,
                              int heads, int dh, const vqa_dropout* drop, hipStream_t s) {
  VQA_REQUIRE(v && out && batch > 0 && len > 0 && heads > 0 && dh % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0,
              "vqa_xattn1_fwd: bad arguments");
  vqa_dropout d = drop ? *drop : vqa_dropout{0.f, 0u, nullptr};
  const long total = (long)batch * len * heads * dh / 8;
  hipLaunchKernelGGL(xattn1_fwd_kernel, dim3((unsigned)vqa::cdiv(total, 256)), dim3(256), 0, s, (const bf16_t*)v,
                     (long)ldv, (bf16_t*)out, (long)ldo, batch, len, heads, dh, d);
  return vqa::check_launch("vqa_xattn1_fwd");
}

extern "C" int vqa_xattn1_bwd(const void* dctx, long long ldd, float* dv32, void* dv16, long long lddv, int batch,
                              int len, int heads, int dh, const vqa_dropout* drop, hipStream_t s) {
  VQA_REQUIRE(dctx && (dv32 || dv16) && batch > 0 && len > 0 && heads > 0 && dh > 0 && lddv >= heads * dh,
              "vqa_xattn1_bwd: bad arguments");
  vqa_dropout d = drop ? *drop : vqa_dropout{0.f, 0u, nullptr};
  const long total = (long)batch * heads * dh;
  hipLaunchKernelGGL(xattn1_bwd_kernel, dim3((unsigned)vqa::cdiv(total, 256)), dim3(256), 0, s,
                     (const bf16_t*)dctx, (long)ldd, dv32, (bf16_t*)dv16, (long)lddv, batch, len, heads, dh, d);
  return vqa::check_launch("vqa_xattn1_bwd");
}
