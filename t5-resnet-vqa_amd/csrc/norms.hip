// Row normalisations over D = 768-wide rows (any D % 256 == 0 up to 1024), one
// wave per row, fp32 math, fused residual-gradient and bf16 copies.
//   T5LayerNorm (RMS, eps 1e-6)      TF/models/t5/modeling_t5.py:50-72
//   nn.LayerNorm(768) (eps 1e-5)     multi_head_vision_text_attn.py:120-126
// Backward kernels also emit per-block partial column sums (dgamma/dbeta) into
// a workspace [gridDim.x][D] that vqa_colsum_partials() reduces
// deterministically (no atomics).
#include "common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;       // 4 waves, one row each
constexpr int MAXV = 4;                 // up to 4 float4 per lane -> D <= 1024

template <int NV>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&x)[NV][4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float4 v = reinterpret_cast<const float4*>(p)[i * 64 + l];
    x[i][0] = v.x; x[i][1] = v.y; x[i][2] = v.z; x[i][3] = v.w;
  }
}
template <int NV>
__device__ __forceinline__ void store_row32(float* __restrict__ p, const float (&x)[NV][4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    reinterpret_cast<float4*>(p)[i * 64 + l] = make_float4(x[i][0], x[i][1], x[i][2], x[i][3]);
}
template <int NV>
__device__ __forceinline__ void store_row16(bf16_t* __restrict__ p, const float (&x)[NV][4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    uint2 u;
    u.x = (uint32_t)f2bf(x[i][0]) | ((uint32_t)f2bf(x[i][1]) << 16);
    u.y = (uint32_t)f2bf(x[i][2]) | ((uint32_t)f2bf(x[i][3]) << 16);
    reinterpret_cast<uint2*>(p)[i * 64 + l] = u;
  }
}
template <int NV>
__device__ __forceinline__ void load_vec(const float* __restrict__ p, float (&x)[NV][4]) { load_row<NV>(p, x); }

// multiply a row held as [NV][4] per lane by the dropout factors of row `row`
template <int NV>
__device__ __forceinline__ void drop_row(const DropK& k, int row, float (&x)[NV][4]) {
  if (!k.on) return;
  const int l = threadIdx.x & 63;
  const uint32_t base = (uint32_t)row * (uint32_t)(NV * 256);
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) x[i][j] *= drop_mul(k, base + (uint32_t)((i * 64 + l) * 4 + j));
}
template <int NV>
__device__ __forceinline__ void store_row16_drop(bf16_t* __restrict__ p, const DropK& k, int row,
                                                 const float (&x)[NV][4]) {
  if (!k.on) { store_row16<NV>(p, x); return; }
  float y[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) y[i][j] = x[i][j];
  drop_row<NV>(k, row, y);
  store_row16<NV>(p, y);
}
template <int NV>
__device__ __forceinline__ void store_row32_drop(float* __restrict__ p, const DropK& k, int row,
                                                 const float (&x)[NV][4]) {
  if (!k.on) { store_row32<NV>(p, x); return; }
  float y[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) y[i][j] = x[i][j];
  drop_row<NV>(k, row, y);
  store_row32<NV>(p, y);
}

// ------------------------------------------------------------------ RMSNorm
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          float* __restrict__ y32, bf16_t* __restrict__ y16,
                                                          float* __restrict__ rstd, int rows, float eps,
                                                          vqa_dropout drop) {
  const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = NV * 256;
  const DropK dk = drop_init(drop);
  float v[NV][4], g[NV][4];
  load_row<NV>(x + (long)row * D, v);
  load_vec<NV>(w, g);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) ss += v[i][j] * v[i][j];
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i][j] = g[i][j] * (v[i][j] * r);
  drop_row<NV>(dk, row, v);
  if (y32) store_row32<NV>(y32 + (long)row * D, v);
  if (y16) store_row16<NV>(y16 + (long)row * D, v);
  if (rstd && (threadIdx.x & 63) == 0) rstd[row] = r;
}

// dx = r*g - (r^3/D) * x * sum(g*x),  g = w*dy ;  dw partial = sum_rows dy*x*r
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          const float* __restrict__ rstd, const float* __restrict__ w,
                                                          const float* __restrict__ dres, float* __restrict__ dx32,
                                                          bf16_t* __restrict__ dx16, float* __restrict__ dw_ws,
                                                          int rows, int rows_per_block, vqa_dropout drop_dy,
                                                          vqa_dropout drop_dx32, vqa_dropout drop_dx16) {
  constexpr int D = NV * 256;
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const DropK kdy = drop_init(drop_dy), k32 = drop_init(drop_dx32), k16 = drop_init(drop_dx16);
  float g[NV][4];
  load_vec<NV>(w, g);
  float dwacc[NV][4] = {};
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  // a wave's rows two at a time, both rows' loads issued before either is used: one memory
  // round trip per pair instead of per row (the per-row arithmetic and order are unchanged)
  for (int row0 = r0 + wv; row0 < r1; row0 += 2 * ROWS_PER_BLOCK) {
    float d[2][NV][4], v[2][NV][4], o[2][NV][4], r[2];
    const int nr = row0 + ROWS_PER_BLOCK < r1 ? 2 : 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h < nr) {
        const int row = row0 + h * ROWS_PER_BLOCK;
        load_row<NV>(dy + (long)row * D, d[h]);
        load_row<NV>(x + (long)row * D, v[h]);
        if (dres) load_row<NV>(dres + (long)row * D, o[h]);
        r[h] = rstd[row];
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h >= nr) break;
      const int row = row0 + h * ROWS_PER_BLOCK;
      drop_row<NV>(kdy, row, d[h]);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s += g[i][j] * d[h][i][j] * v[h][i][j];
          dwacc[i][j] += d[h][i][j] * v[h][i][j] * r[h];
        }
      s = wave_sum(s);
      const float c = r[h] * r[h] * r[h] * s / D;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = r[h] * g[i][j] * d[h][i][j] - c * v[h][i][j];
          o[h][i][j] = dres ? o[h][i][j] + t : t;
        }
      if (dx32) store_row32_drop<NV>(dx32 + (long)row * D, k32, row, o[h]);
      if (dx16) store_row16_drop<NV>(dx16 + (long)row * D, k16, row, o[h]);
    }
  }
  // reduce the 4 waves' dw partials through LDS, write one row per block
  __shared__ float red[ROWS_PER_BLOCK][NV * 256];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wv][(i * 64 + l) * 4 + j] = dwacc[i][j];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    dw_ws[(long)blockIdx.x * D + c] = t;
  }
}

// ------------------------------------------------------------------ LayerNorm
template <int NV>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gam,
                                                            const float* __restrict__ bet, float* __restrict__ y32,
                                                            bf16_t* __restrict__ y16, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, int rows, float eps) {
  const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = NV * 256;
  float v[NV][4], g[NV][4], b[NV][4];
  load_row<NV>(x + (long)row * D, v);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[i][j];
  const float mu = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { float t = v[i][j] - mu; ss += t * t; }
  const float r = rsqrtf(wave_sum(ss) / D + eps);
  load_vec<NV>(gam, g);
  load_vec<NV>(bet, b);
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i][j] = (v[i][j] - mu) * r * g[i][j] + b[i][j];
  if (y32) store_row32<NV>(y32 + (long)row * D, v);
  if (y16) store_row16<NV>(y16 + (long)row * D, v);
  if ((threadIdx.x & 63) == 0) { mean_out[row] = mu; rstd_out[row] = r; }
}

// xh = (x-mu)*r ; g = gam*dy ; dx = r*(g - mean(g) - xh*mean(g*xh)) (+dres)
// partials: dgamma = sum dy*xh -> ws[0..D), dbeta = sum dy -> ws[D..2D)
template <int NV>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                            const float* __restrict__ mean, const float* __restrict__ rstd,
                                                            const float* __restrict__ gam, const float* __restrict__ dres,
                                                            float* __restrict__ dx32, bf16_t* __restrict__ dx16,
                                                            float* __restrict__ ws, int rows, int rows_per_block,
                                                            vqa_dropout drop_dx16, int with_dsum) {
  constexpr int D = NV * 256;
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const DropK k16 = drop_init(drop_dx16);
  float g[NV][4];
  load_vec<NV>(gam, g);
  float dga[NV][4] = {}, dba[NV][4] = {}, dsa[NV][4] = {};
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  // two rows per iteration, both rows' loads issued first (as in rmsnorm_bwd_kernel)
  for (int row0 = r0 + wv; row0 < r1; row0 += 2 * ROWS_PER_BLOCK) {
    float d[2][NV][4], v[2][NV][4], rr[2][NV][4], mu[2], r[2];
    const int nr = row0 + ROWS_PER_BLOCK < r1 ? 2 : 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h < nr) {
        const int row = row0 + h * ROWS_PER_BLOCK;
        load_row<NV>(dy + (long)row * D, d[h]);
        load_row<NV>(x + (long)row * D, v[h]);
        if (dres) load_row<NV>(dres + (long)row * D, rr[h]);
        mu[h] = mean[row];
        r[h] = rstd[row];
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h >= nr) break;
      const int row = row0 + h * ROWS_PER_BLOCK;
      float o[NV][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[h][i][j] = (v[h][i][j] - mu[h]) * r[h];        // xhat
          const float gd = g[i][j] * d[h][i][j];
          s1 += gd;
          s2 += gd * v[h][i][j];
          dga[i][j] += d[h][i][j] * v[h][i][j];
          dba[i][j] += d[h][i][j];
        }
      s1 = wave_sum(s1) / D;
      s2 = wave_sum(s2) / D;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[i][j] = r[h] * (g[i][j] * d[h][i][j] - s1 - v[h][i][j] * s2);
          if (dres) rr[h][i][j] += o[i][j];
        }
      // post-LN: dres is an accumulator that only the fp32 output carries; the branch
      // gradient (dx16, dsum) is the LayerNorm input gradient alone
      if (dx32) store_row32<NV>(dx32 + (long)row * D, dres ? rr[h] : o);
      if (dx16 || with_dsum) {
        drop_row<NV>(k16, row, o);                         // the branch gradient (masked)
        if (dx16) store_row16<NV>(dx16 + (long)row * D, o);
#pragma unroll
        for (int i = 0; i < NV; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) dsa[i][j] += o[i][j];
      }
    }
  }
  __shared__ float red[ROWS_PER_BLOCK][NV * 256];
  const int npass = with_dsum ? 3 : 2;
  for (int pass = 0; pass < npass; ++pass) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        red[wv][(i * 64 + l) * 4 + j] = pass == 0 ? dga[i][j] : (pass == 1 ? dba[i][j] : dsa[i][j]);
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256)
      ws[((long)blockIdx.x * 3 + pass) * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    __syncthreads();
  }
}

// out[c] = beta*out[c] + sum_p ws[p*stride + c]  (fixed order -> deterministic).
// 1024 threads = 64 columns x 16 part-groups, so the partial reads are spread
// over 16 waves instead of one long dependent chain per column.
__global__ __launch_bounds__(1024) void colsum_partials_kernel(const float* __restrict__ ws, int parts, long stride,
                                                               int cols, float* __restrict__ out, float beta) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 4
    for (int p = ty; p < parts; p += 16) s += ws[(long)p * stride + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][tx];
    out[c] = beta != 0.f ? beta * out[c] + t : t;
  }
}

// the LayerNorm backward's up to three column sums in one launch: blockIdx.y picks
// the output (0 dgamma, 1 dbeta, 2 branch-gradient sum) from ws[p][3][cols]
__global__ __launch_bounds__(1024) void colsum3_partials_kernel(const float* __restrict__ ws, int parts, long stride,
                                                                int cols, float* __restrict__ o0,
                                                                float* __restrict__ o1, float* __restrict__ o2) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx, which = blockIdx.y;
  const float* w = ws + (long)which * cols;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 4
    for (int p = ty; p < parts; p += 16) s += w[(long)p * stride + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][tx];
    (which == 0 ? o0 : (which == 1 ? o1 : o2))[c] = t;
  }
}

// Any number of deferred partial-row reductions in one launch: block b serves job
// j (scalar scan, first_block ascending), 64 columns x 16 part-groups as above.
__global__ __launch_bounds__(1024) void colsum_batched_kernel(const vqa_colsum_job* __restrict__ jobs, int njobs) {
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].first_block <= (int)blockIdx.x) ++j;
  const vqa_colsum_job J = jobs[j];
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x - J.first_block) * 64 + tx;
  float s = 0.f;
  if (c < J.cols) {
#pragma unroll 4
    for (int p = ty; p < J.parts; p += 16) s += J.ws[(long)p * J.stride + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < J.cols) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][tx];
    J.out[c] = J.beta != 0.f ? J.beta * J.out[c] + t : t;
  }
}

constexpr int NORM_BWD_ROWS = 8;       // rows per block in the backward kernels (256 blocks at 2048 rows)

vqa_dropout dr(const vqa_dropout* d) {
  vqa_dropout o{0.f, 0u, nullptr};
  return d ? *d : o;
}
bool dr_ok(const vqa_dropout* d) { return !d || (d->p >= 0.f && d->p < 1.f); }

}  // namespace

#define DISPATCH_NV(D, ...)                                          \
  switch ((D) / 256) {                                               \
    case 1: { constexpr int NV = 1; __VA_ARGS__; break; }            \
    case 2: { constexpr int NV = 2; __VA_ARGS__; break; }            \
    case 3: { constexpr int NV = 3; __VA_ARGS__; break; }            \
    case 4: { constexpr int NV = 4; __VA_ARGS__; break; }            \
    default: return vqa::fail(VQA_ERR_INVALID, "norm: D=%d unsupported (D %% 256 == 0, <= 1024)", (D)); \
  }

extern "C" int vqa_rmsnorm_fwd(const float* x, const float* w, float* y32, void* y16, float* rstd, int rows, int d,
                               float eps, const vqa_dropout* drop, hipStream_t s) {
  VQA_REQUIRE(x && w && (y32 || y16) && rows > 0 && d % 256 == 0, "vqa_rmsnorm_fwd: bad arguments");
  VQA_REQUIRE(dr_ok(drop), "vqa_rmsnorm_fwd: dropout p must be in [0, 1)");
  dim3 grid(vqa::cdiv(rows, ROWS_PER_BLOCK));
  DISPATCH_NV(d, hipLaunchKernelGGL(rmsnorm_fwd_kernel<NV>, grid, dim3(256), 0, s, x, w, y32, (bf16_t*)y16, rstd,
                                    rows, eps, dr(drop)));
  return vqa::check_launch("vqa_rmsnorm_fwd");
}

extern "C" int vqa_norm_bwd_parts(int rows) { return vqa::cdiv(rows, NORM_BWD_ROWS); }
extern "C" int vqa_norm_bwd_workspace_floats(int rows, int d) { return 3 * vqa_norm_bwd_parts(rows) * d; }

extern "C" int vqa_rmsnorm_bwd(const float* dy, const float* x, const float* rstd, const float* w, const float* dres,
                               float* dx32, void* dx16, float* dw, float dw_beta, float* ws, int rows, int d,
                               const vqa_dropout* drop_dy, const vqa_dropout* drop_dx32, const vqa_dropout* drop_dx16,
                               hipStream_t s) {
  VQA_REQUIRE(dy && x && rstd && w && ws && (dx32 || dx16) && d % 256 == 0, "vqa_rmsnorm_bwd: bad arguments");
  VQA_REQUIRE(dr_ok(drop_dy) && dr_ok(drop_dx32) && dr_ok(drop_dx16), "vqa_rmsnorm_bwd: dropout p must be in [0, 1)");
  const int parts = vqa_norm_bwd_parts(rows);
  DISPATCH_NV(d, hipLaunchKernelGGL(rmsnorm_bwd_kernel<NV>, dim3(parts), dim3(256), 0, s, dy, x, rstd, w, dres, dx32,
                                    (bf16_t*)dx16, ws, rows, NORM_BWD_ROWS, dr(drop_dy), dr(drop_dx32),
                                    dr(drop_dx16)));
  if (int rc = vqa::check_launch("vqa_rmsnorm_bwd")) return rc;
  if (!dw) return VQA_OK;                                    // deferred: vqa_colsum_batched reduces ws
  hipLaunchKernelGGL(colsum_partials_kernel, dim3(vqa::cdiv(d, 64)), dim3(1024), 0, s, ws, parts, (long)d, d, dw,
                     dw_beta);
  return vqa::check_launch("vqa_rmsnorm_bwd/colsum");
}

extern "C" int vqa_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y32, void* y16,
                                 float* mean, float* rstd, int rows, int d, float eps, hipStream_t s) {
  VQA_REQUIRE(x && gamma && beta && mean && rstd && (y32 || y16) && d % 256 == 0, "vqa_layernorm_fwd: bad arguments");
  dim3 grid(vqa::cdiv(rows, ROWS_PER_BLOCK));
  DISPATCH_NV(d, hipLaunchKernelGGL(layernorm_fwd_kernel<NV>, grid, dim3(256), 0, s, x, gamma, beta, y32,
                                    (bf16_t*)y16, mean, rstd, rows, eps));
  return vqa::check_launch("vqa_layernorm_fwd");
}

extern "C" int vqa_layernorm_bwd(const float* dy, const float* x, const float* mean, const float* rstd,
                                 const float* gamma, const float* dres, float* dx32, void* dx16, float* dgamma,
                                 float* dbeta, float* ws, int rows, int d, const vqa_dropout* drop_dx16,
                                 float* dsum, hipStream_t s) {
  VQA_REQUIRE(dy && x && mean && rstd && gamma && ws && (dx32 || dx16) && d % 256 == 0 && !dgamma == !dbeta,
              "vqa_layernorm_bwd: bad arguments");
  VQA_REQUIRE(dr_ok(drop_dx16), "vqa_layernorm_bwd: dropout p must be in [0, 1)");
  const int parts = vqa_norm_bwd_parts(rows);
  DISPATCH_NV(d, hipLaunchKernelGGL(layernorm_bwd_kernel<NV>, dim3(parts), dim3(256), 0, s, dy, x, mean, rstd, gamma,
                                    dres, dx32, (bf16_t*)dx16, ws, rows, NORM_BWD_ROWS, dr(drop_dx16),
                                    dsum != nullptr ? 1 : 0));
  if (int rc = vqa::check_launch("vqa_layernorm_bwd")) return rc;
  if (!dgamma) return VQA_OK;                                // deferred: vqa_colsum_batched reduces ws
  hipLaunchKernelGGL(colsum3_partials_kernel, dim3(vqa::cdiv(d, 64), dsum ? 3 : 2), dim3(1024), 0, s, ws, parts,
                     (long)3 * d, d, dgamma, dbeta, dsum);
  return vqa::check_launch("vqa_layernorm_bwd/colsum");
}

extern "C" int vqa_colsum_partials(const float* ws, int parts, long long stride, int cols, float* out, float beta,
                                   hipStream_t s) {
  VQA_REQUIRE(ws && out && parts > 0 && cols > 0, "vqa_colsum_partials: bad arguments");
  hipLaunchKernelGGL(colsum_partials_kernel, dim3(vqa::cdiv(cols, 64)), dim3(1024), 0, s, ws, parts, (long)stride, cols,
                     out, beta);
  return vqa::check_launch("vqa_colsum_partials");
}

extern "C" int vqa_colsum_batched(const vqa_colsum_job* jobs, int njobs, int nblocks, hipStream_t s) {
  VQA_REQUIRE(jobs && njobs > 0 && nblocks > 0, "vqa_colsum_batched: bad arguments");
  hipLaunchKernelGGL(colsum_batched_kernel, dim3(nblocks), dim3(1024), 0, s, jobs, njobs);
  return vqa::check_launch("vqa_colsum_batched");
}
