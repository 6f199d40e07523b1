// Optimiser tail of train_one_step (faster_rcnn_vqa_trainer.py:399-404):
//   clip_grad_norm_(params, 1.0)  ->  AdamW(wd=0.1, amsgrad=True) over the
//   trainer's param groups (:231-267)  ->  get_linear_schedule_with_warmup
//   (:279-287, TF/optimization.py:101-107).
// Everything stays on the device so the whole step can be one hipGraph:
//   1. vqa_grad_sqnorm    grid-stride partial sums of g^2 (fp64 accumulators)
//   2. vqa_optim_finalize one thread: norm, clip coefficient, LR multiplier
//                         lambda(step), bias corrections; advances `step`
//   3. vqa_adamw_amsgrad  one fused HBM pass over p, g, m, v, vmax -> p, m, v,
//                         vmax and the bf16 shadow copy used by the GEMMs.
// The DP average (1/world) enters as grad_scale in steps 2 and 3.
#include "adamw.h"

namespace {

__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ g, long n4, double* __restrict__ ws) {
  // Four grid-stride loads issued before their (in-order) accumulation: the sum is the
  // same as the one-load loop's, bit for bit, with 4x the loads in flight per wave.
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const long st = (long)gridDim.x * 256;
  double s = 0.0;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n4; i += 4 * st) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = g4[i + u * st];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      s += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y + (double)v[u].z * v[u].z + (double)v[u].w * v[u].w;
  }
  for (; i < n4; i += st) {
    const float4 v = g4[i];
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// the LR multiplier lambda(step) and the bias corrections of the update at step counter `step`
// (get_linear_schedule_with_warmup, TF/optimization.py:101-107; torch AdamW's 1 - beta^t): one
// function for vqa_optim_finalize and the embedding rows' early update, so both round alike
__device__ __forceinline__ void schedule_at(double step, int warmup, int total, float beta1, float beta2,
                                            float& lam_f, float& bc1, float& bc2s) {
  double lam;
  if (step < warmup) lam = step / (double)(warmup > 1 ? warmup : 1);
  else lam = fmax(0.0, (double)(total - step) / (double)((total - warmup) > 1 ? (total - warmup) : 1));
  const double t = step + 1.0;
  lam_f = (float)lam;
  bc1 = (float)(1.0 - pow((double)beta1, t));
  bc2s = (float)sqrt(1.0 - pow((double)beta2, t));
}

__global__ void finalize_kernel(const double* __restrict__ ws, int parts, float grad_scale, float max_norm,
                                int warmup, int total, float beta1, float beta2, float* __restrict__ st) {
  // fixed-order two-level sum of the partials by one workgroup
  __shared__ double red[256];
  double part = 0.0;
  for (int i = threadIdx.x; i < parts; i += 256) part += ws[i];
  red[threadIdx.x] = part;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double ss = 0.0;
  for (int i = 0; i < 256; ++i) ss += red[i];
  const float norm = (float)(sqrt(ss) * (double)grad_scale);
  float coef = 1.f;
  if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
  const double step = (double)st[VQA_ST_STEP];
  float lam, bc1, bc2s;
  schedule_at(step, warmup, total, beta1, beta2, lam, bc1, bc2s);
  st[VQA_ST_GRAD_NORM] = norm;
  st[VQA_ST_CLIP_COEF] = coef;
  st[VQA_ST_LR_SCALE] = lam;
  st[VQA_ST_BC1] = bc1;
  st[VQA_ST_BC2_SQRT] = bc2s;
  st[VQA_ST_STEP] = (float)(step + 1.0);
  st[VQA_ST_PENDING] = 1.f;
}

// The embedding table's update split by rows.  mark[id] = the step counter for every id of the
// step's tokens (embed_mark_kernel, before the step's finalize).  A row no token touched has an
// exactly zero gradient, so its AdamW update needs neither the gradient nor the clip coefficient
// (g * gscale * coef = +0 for any finite coef) -- only the schedule of the coming finalize: MODE 0
// applies it to those rows, beside the backward, before finalize.  MODE 1 (after finalize, which
// advanced the counter) applies the full update to the marked rows.  Every row gets the same
// arithmetic as the dense pass (adamw_update4_with), so the table ends bit-identical to it; a row
// marked but not touched (a warm-up's ids) gets g = 0 in MODE 1, the same result as in MODE 0.
__global__ __launch_bounds__(256) void embed_mark_kernel(const long long* __restrict__ ids, int n, int rows,
                                                         int* __restrict__ mark, const float* __restrict__ st) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long id = ids[i];
  if (id >= 0 && id < rows) mark[id] = (int)st[VQA_ST_STEP];
}

// one block per row, or (rows_per_block > 1) a grid of rows / rows_per_block blocks striding over
// the rows: the untouched rows' pass runs beside the latency-bound backward chain, where a
// 32k-block grid would hold CU slots the chain's launches wait for
template <int MODE>
__global__ __launch_bounds__(192) void adamw_rows_kernel(AdamArgs A, const int* __restrict__ mark, int rows, int d4,
                                                         int warmup, int total) {
  const int step = (int)A.st[VQA_ST_STEP];
  float coef, lam, bc1, bc2s;
  if (MODE == 0) {
    coef = 1.f;
    schedule_at((double)A.st[VQA_ST_STEP], warmup, total, A.b1, A.b2, lam, bc1, bc2s);
  } else {
    if (A.st[VQA_ST_PENDING] == 0.f) return;
    coef = A.st[VQA_ST_CLIP_COEF];
    lam = A.st[VQA_ST_LR_SCALE];
    bc1 = A.st[VQA_ST_BC1];
    bc2s = A.st[VQA_ST_BC2_SQRT];
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
  const bool touched = mark[row] == (MODE == 0 ? step : step - 1);
  if (MODE == 0 ? touched : !touched) continue;
  for (int c = threadIdx.x; c < d4; c += 192) {
    const long i = (long)row * d4 + c;
    f32x4_t p = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.p) + i);
    f32x4_t g4 = {0.f, 0.f, 0.f, 0.f};
    if (MODE == 1) g4 = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.g) + i);
    f32x4_t m = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.m) + i);
    f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.v) + i);
    f32x4_t vm = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.vm) + i);
    adamw_update4_with(A, i, p, g4, m, v, vm, coef, lam, bc1, bc2s);
    __builtin_nontemporal_store(p, reinterpret_cast<f32x4_t*>(A.p) + i);
    __builtin_nontemporal_store(m, reinterpret_cast<f32x4_t*>(A.m) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t*>(A.v) + i);
    __builtin_nontemporal_store(vm, reinterpret_cast<f32x4_t*>(A.vm) + i);
    if (A.p16) {
      uint2 u;
      u.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
      u.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
      reinterpret_cast<uint2*>(A.p16)[i] = u;
    }
  }
  }
}

// One float4 of every stream per thread, no grid-stride loop: 138k blocks of
// 256 keep ~2k threads x 5 x 16 B of loads in flight per CU.  Every stream is
// touched once per step (5.4 GB >> the 256 MiB Infinity Cache), so loads and
// stores are non-temporal.
__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs A) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= A.n4 || A.st[VQA_ST_PENDING] == 0.f) return;   // nothing to apply (see VQA_ST_PENDING)
  f32x4_t p = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.p) + i);
  const f32x4_t g4 = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.g) + i);
  f32x4_t m = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.m) + i);
  f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.v) + i);
  f32x4_t vm = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(A.vm) + i);
  adamw_update4(A, i, p, g4, m, v, vm);
  __builtin_nontemporal_store(p, reinterpret_cast<f32x4_t*>(A.p) + i);
  __builtin_nontemporal_store(m, reinterpret_cast<f32x4_t*>(A.m) + i);
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t*>(A.v) + i);
  __builtin_nontemporal_store(vm, reinterpret_cast<f32x4_t*>(A.vm) + i);
  if (A.p16) {
    uint2 u;
    u.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
    u.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
    reinterpret_cast<uint2*>(A.p16)[i] = u;            // the next forward reads it: keep it cacheable
  }
}

int grid_for(long n4) {
  long b = (n4 + 255) / 256;
  return (int)(b < 4096 ? b : 4096);
}

}  // namespace

extern "C" int vqa_grad_sqnorm(const float* g, long long n, double* ws, int parts, hipStream_t s) {
  VQA_REQUIRE(g && ws && n % 4 == 0 && parts > 0, "vqa_grad_sqnorm: bad arguments (n %% 4 == 0)");
  hipLaunchKernelGGL(sqnorm_kernel, dim3(parts), dim3(256), 0, s, g, (long)(n / 4), ws);
  return vqa::check_launch("vqa_grad_sqnorm");
}

extern "C" int vqa_optim_finalize(const double* ws, int parts, float grad_scale, float max_norm, int warmup, int total,
                                  float beta1, float beta2, float* state, hipStream_t s) {
  VQA_REQUIRE(ws && state && parts > 0, "vqa_optim_finalize: bad arguments");
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, ws, parts, grad_scale, max_norm, warmup, total, beta1,
                     beta2, state);
  return vqa::check_launch("vqa_optim_finalize");
}

extern "C" int vqa_adamw_amsgrad(const vqa_adamw_desc* d, hipStream_t s) {
  AdamArgs A;
  if (int rc = adam_args(d, A)) return rc;
  hipLaunchKernelGGL(adamw_kernel, dim3(vqa::cdiv(A.n4, 256)), dim3(256), 0, s, A);
  return vqa::check_launch("vqa_adamw_amsgrad");
}

extern "C" int vqa_embed_mark(const long long* ids, int n, int rows, int* mark, const float* state, hipStream_t s) {
  VQA_REQUIRE(ids && mark && state && n > 0 && rows > 0, "vqa_embed_mark: bad arguments");
  hipLaunchKernelGGL(embed_mark_kernel, dim3(vqa::cdiv(n, 256)), dim3(256), 0, s, ids, n, rows, mark, state);
  return vqa::check_launch("vqa_embed_mark");
}

extern "C" int vqa_adamw_rows(const vqa_adamw_desc* d, const int* mark, int rows, int cols, int touched, int warmup,
                              int total, hipStream_t s) {
  AdamArgs A;
  if (int rc = adam_args(d, A)) return rc;
  VQA_REQUIRE(mark && rows > 0 && cols > 0 && cols % 4 == 0 && (long long)rows * cols == d->n,
              "vqa_adamw_rows: rows x cols must be the descriptor's n (cols %% 4 == 0)");
  // touched > 1 (the untouched-rows pass only): a grid of `touched` blocks striding over the rows
  const int grid = touched > 1 && touched < rows ? touched : rows;
  if (touched == 1)
    hipLaunchKernelGGL(adamw_rows_kernel<1>, dim3(rows), dim3(192), 0, s, A, mark, rows, cols / 4, warmup, total);
  else
    hipLaunchKernelGGL(adamw_rows_kernel<0>, dim3(grid), dim3(192), 0, s, A, mark, rows, cols / 4, warmup, total);
  return vqa::check_launch("vqa_adamw_rows");
}
