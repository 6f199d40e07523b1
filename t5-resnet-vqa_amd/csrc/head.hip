// Answer head: AttentionPooler (resnet_vqa_model.py:14-26) + classification
// Linear(768, A) + log_softmax + NLLLoss(mean) (resnet_vqa_model.py:152-160),
// forward and backward, fp32 end to end (straight from the fp32 masters).
//   pooler kernels: one workgroup per sample, each thread keeps its D/256
//     columns of all L rows in registers, so scores, softmax, pooling and the
//     pooler backward need a single read of the sample;
//   classifier: logits fused into the forward kernel; dpooled and dWc by an
//     LDS-tiled fp32 GEMM;
//   every reduction runs in a fixed order (bit-reproducible).
#include <type_traits>

#include "common.h"

namespace {

constexpr int MAXA = 1024;

// ------------------------------------------------------------ small fp32 GEMM
// C[m, n] = sum_k A(m, k) B(k, n) (+ bias[n]);  A(m,k) = a[m*sam + k*sak], B(k,n) = b[k*sbk + n*sbn]
constexpr int SG_T = 32, SG_K = 32;
__global__ __launch_bounds__(256) void sgemm_kernel(int M, int N, int K, const float* __restrict__ a, long sam, long sak,
                                                    const float* __restrict__ b, long sbk, long sbn,
                                                    float* __restrict__ c, long ldc, const float* __restrict__ bias) {
  __shared__ float As[SG_K][SG_T + 1], Bs[SG_K][SG_T + 1];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;          // 32 x 8 threads, 4 rows each
  const int m0 = blockIdx.y * SG_T, n0 = blockIdx.x * SG_T;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += SG_K) {
    for (int i = threadIdx.x; i < SG_T * SG_K; i += 256) {
      const int r = i / SG_K, kk = i - r * SG_K;                    // A tile: row r, k kk
      const int m = m0 + r, k = k0 + kk;
      As[kk][r] = (m < M && k < K) ? a[(long)m * sam + (long)k * sak] : 0.f;
      const int kb = i / SG_T, nn = i - kb * SG_T;                 // B tile: k kb, col nn
      const int kg = k0 + kb, n = n0 + nn;
      Bs[kb][nn] = (kg < K && n < N) ? b[(long)kg * sbk + (long)n * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < SG_K; ++kk) {
      const float bv = Bs[kk][tx];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = fmaf(As[kk][ty * 4 + r], bv, acc[r]);
    }
    __syncthreads();
  }
  const int n = n0 + tx;
  if (n >= N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + ty * 4 + r;
    if (m < M) c[(long)m * ldc + n] = acc[r] + (bias ? bias[n] : 0.f);
  }
}

int sgemm(hipStream_t s, int M, int N, int K, const float* a, long sam, long sak, const float* b, long sbk, long sbn,
          float* c, long ldc, const float* bias) {
  dim3 grid(vqa::cdiv(N, SG_T), vqa::cdiv(M, SG_T));
  hipLaunchKernelGGL(sgemm_kernel, grid, dim3(256), 0, s, M, N, K, a, sam, sak, b, sbk, sbn, c, ldc, bias);
  return vqa::check_launch("head/sgemm");
}

// ------------------------------------------------------------ pooler
// block-wide reduction of NV per-thread vectors of length L (one value per row t)
template <int LMAX>
__device__ __forceinline__ void block_row_sums(float (&part)[LMAX], int L, float* red /*[4][LMAX]*/,
                                               float* out /*[LMAX]*/) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < LMAX; ++t) {
    if (t < L) {
      const float v = wave_sum(part[t]);
      if (l == 0) red[wv * LMAX + t] = v;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < L; t += 256) out[t] = red[t] + red[LMAX + t] + red[2 * LMAX + t] + red[3 * LMAX + t];
  __syncthreads();
}

// The whole forward head of one sample in one workgroup (resnet_vqa_model.py:152-160):
// pooler (scores, softmax over L, weighted sum) -> pooled row in LDS -> 170 logits, one wave per
// answer at a time, lanes striding the D-long dot so the Wc row read is one
// coalesced 256-B access per step -> log_softmax over the answers in LDS -> NLL.
// Replaces a K=768 LDS-tiled sgemm whose 12 workgroups walked K serially (~33 us).
template <int LMAX>
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wp,
                                                       const float* __restrict__ bp, const float* __restrict__ wc,
                                                       const float* __restrict__ bc, const long long* __restrict__ tgt,
                                                       float* __restrict__ att, float* __restrict__ pooled,
                                                       float* __restrict__ logp, float* __restrict__ nll, int L, int D,
                                                       int A) {
  constexpr int NC = 3;
  __shared__ float red[4 * LMAX], sc[LMAX], pr[768], lg[MAXA], r4[4];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const float* xb = x + (long)b * L * D;
  float xr[LMAX][NC], part[LMAX];
  float w[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) w[j] = (tid + 256 * j < D) ? wp[tid + 256 * j] : 0.f;
#pragma unroll
  for (int t = 0; t < LMAX; ++t) {
    part[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      xr[t][j] = (t < L && d < D) ? xb[(long)t * D + d] : 0.f;
      part[t] = fmaf(xr[t][j], w[j], part[t]);
    }
  }
  block_row_sums<LMAX>(part, L, red, sc);
  if (tid < 64) {                                     // softmax over the sequence (Softmax(dim=1))
    const float s = tid < L ? sc[tid] + bp[0] : -INFINITY;
    const float m = wave_max(s);
    const float e = tid < L ? __expf(s - m) : 0.f;
    const float z = wave_sum(e);
    if (tid < L) { sc[tid] = e / z; att[(long)b * L + tid] = e / z; }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int d = tid + 256 * j;
    if (d >= D) continue;
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < LMAX; ++t)
      if (t < L) p = fmaf(sc[t], xr[t][j], p);
    pooled[(long)b * D + d] = p;
    pr[d] = p;
  }
  __syncthreads();
  for (int a = wv; a < A; a += 4) {                   // logits = pooled Wc^T + bc
    const float* wr = wc + (long)a * D;
    float s = 0.f;
    for (int k = l; k < D; k += 64) s = fmaf(pr[k], wr[k], s);
    s = wave_sum(s);
    if (l == 0) lg[a] = s + bc[a];
  }
  __syncthreads();
  float m = -INFINITY;
  for (int c = tid; c < A; c += 256) m = fmaxf(m, lg[c]);
  m = wave_max(m);
  if (l == 0) r4[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(r4[0], r4[1]), fmaxf(r4[2], r4[3]));
  __syncthreads();
  float z = 0.f;
  for (int c = tid; c < A; c += 256) z += __expf(lg[c] - m);
  z = wave_sum(z);
  if (l == 0) r4[wv] = z;
  __syncthreads();
  const float lse = m + __logf(r4[0] + r4[1] + r4[2] + r4[3]);
  for (int c = tid; c < A; c += 256) logp[(long)b * A + c] = lg[c] - lse;
  if (tid == 0 && tgt) nll[b] = -(lg[tgt[b]] - lse);
}

// fixed-order mean / sum of n values by one workgroup
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ v, int n, float scale,
                                                     float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// dlogits = (softmax - onehot) / B
__global__ __launch_bounds__(256) void dlogits_kernel(const float* __restrict__ logp, const long long* __restrict__ tgt,
                                                      float* __restrict__ dl, int A, float inv_b) {
  const int b = blockIdx.x;
  const long long t = tgt[b];
  for (int c = threadIdx.x; c < A; c += 256)
    dl[(long)b * A + c] = (__expf(logp[(long)b * A + c]) - (c == t ? 1.f : 0.f)) * inv_b;
}

// pooler backward for one sample: da = x dpooled ; dscore = a (da - sum a da) ;
// dx = a dpooled^T + dscore wp^T
template <int LMAX>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ att,
                                                       const float* __restrict__ dpooled,
                                                       const float* __restrict__ wp, float* __restrict__ dx32,
                                                       bf16_t* __restrict__ dx16, float* __restrict__ dscore, int L,
                                                       int D) {
  constexpr int NC = 3;
  __shared__ float red[4 * LMAX], da[LMAX], a[LMAX];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* xb = x + (long)b * L * D;
  float xr[LMAX][NC], part[LMAX], dp[NC], w[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int d = tid + 256 * j;
    dp[j] = d < D ? dpooled[(long)b * D + d] : 0.f;
    w[j] = d < D ? wp[d] : 0.f;
  }
#pragma unroll
  for (int t = 0; t < LMAX; ++t) {
    part[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      xr[t][j] = (t < L && d < D) ? xb[(long)t * D + d] : 0.f;
      part[t] = fmaf(xr[t][j], dp[j], part[t]);
    }
  }
  for (int t = tid; t < L; t += 256) a[t] = att[(long)b * L + t];
  block_row_sums<LMAX>(part, L, red, da);
  if (tid < 64) {
    const float ai = tid < L ? a[tid] : 0.f, dai = tid < L ? da[tid] : 0.f;
    const float s = wave_sum(ai * dai);
    if (tid < L) {
      const float ds = ai * (dai - s);
      da[tid] = ds;
      dscore[(long)b * L + tid] = ds;
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < LMAX; ++t) {
    if (t >= L) continue;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      if (d >= D) continue;
      const float g = a[t] * dp[j] + da[t] * w[j];
      dx32[((long)b * L + t) * D + d] = g;
      if (dx16) dx16[((long)b * L + t) * D + d] = f2bf(g);
    }
  }
}

// partial dWp[d] = sum_rows dscore[row] x[row][d] over 64-row chunks
__global__ __launch_bounds__(256) void wpool_part_kernel(const float* __restrict__ x, const float* __restrict__ ds,
                                                         float* __restrict__ ws, int rows, int D) {
  const int r0 = blockIdx.y * 64;
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= D) return;
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < min(rows, r0 + 64); ++r) s = fmaf(ds[r], x[(long)r * D + d], s);
  ws[(long)blockIdx.y * D + d] = s;
}

template <typename F>
int with_lmax(int L, F f) {
  if (L <= 16) return f(std::integral_constant<int, 16>());
  if (L <= 32) return f(std::integral_constant<int, 32>());
  return f(std::integral_constant<int, 64>());
}

}  // namespace

extern "C" int vqa_head_workspace_floats(int batch, int seq, int d, int answers) {
  return 2 * batch * answers + batch * d + batch * seq + vqa::cdiv(batch * seq, 64) * d;
}

// ws layout: logits | dlogits [B*A] each, dpooled [B*D], dscore [B*L], dWp partials
extern "C" int vqa_head_fwd(const float* x, const float* wp, const float* bp, const float* wc, const float* bc,
                            const long long* targets, float* att, float* pooled, float* logp, float* nll, float* loss,
                            int batch, int seq, int d, int answers, hipStream_t s) {
  VQA_REQUIRE(x && wp && bp && wc && bc && att && pooled && logp, "vqa_head_fwd: null argument");
  VQA_REQUIRE(seq <= 64 && d <= 768 && answers <= MAXA, "vqa_head_fwd: shape out of range (L<=64, D<=768)");
  VQA_REQUIRE(!targets || (nll && loss), "vqa_head_fwd: targets need nll and loss outputs");
  int rc = with_lmax(seq, [&](auto lm) {
    hipLaunchKernelGGL(head_fwd_kernel<decltype(lm)::value>, dim3(batch), dim3(256), 0, s, x, wp, bp, wc, bc, targets,
                       att, pooled, logp, nll, seq, d, answers);
    return vqa::check_launch("vqa_head_fwd");
  });
  if (rc) return rc;
  if (targets) {
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(256), 0, s, nll, batch, 1.0f / batch, loss);
    return vqa::check_launch("vqa_head_fwd/mean");
  }
  return VQA_OK;
}

extern "C" int vqa_head_bwd(const float* x, const float* att, const float* pooled, const float* logp,
                            const long long* targets, const float* wp, const float* wc, float* dx32, void* dx16,
                            float* dwp, float* dbp, float* dwc, float* dbc, float* ws, int batch, int seq, int d,
                            int answers, hipStream_t s) {
  VQA_REQUIRE(x && att && pooled && logp && targets && wp && wc && dx32 && dwp && dbp && dwc && dbc && ws,
              "vqa_head_bwd: null argument");
  VQA_REQUIRE(seq <= 64 && d <= 768 && answers <= MAXA, "vqa_head_bwd: shape out of range");
  float* dl = ws + batch * answers;
  float* dpool = dl + batch * answers;
  float* dsc = dpool + batch * d;
  float* part = dsc + batch * seq;
  hipLaunchKernelGGL(dlogits_kernel, dim3(batch), dim3(256), 0, s, logp, targets, dl, answers, 1.0f / batch);
  int rc = vqa::check_launch("vqa_head_bwd/dlogits");
  if (rc) return rc;
  // dpooled[b, :] = dlogits[b, :] Wc
  if ((rc = sgemm(s, batch, d, answers, dl, answers, 1, wc, d, 1, dpool, d, nullptr))) return rc;
  rc = with_lmax(seq, [&](auto lm) {
    hipLaunchKernelGGL(pool_bwd_kernel<decltype(lm)::value>, dim3(batch), dim3(256), 0, s, x, att, dpool, wp, dx32,
                       (bf16_t*)dx16, dsc, seq, d);
    return vqa::check_launch("vqa_head_bwd/pool");
  });
  if (rc) return rc;
  // dWc = dlogits^T pooled ; dbc = column sums of dlogits
  if ((rc = sgemm(s, answers, d, batch, dl, 1, answers, pooled, d, 1, dwc, d, nullptr))) return rc;
  if ((rc = vqa_colsum_partials(dl, batch, answers, answers, dbc, 0.f, s))) return rc;
  const int rows = batch * seq, parts = vqa::cdiv(rows, 64);
  hipLaunchKernelGGL(wpool_part_kernel, dim3(vqa::cdiv(d, 256), parts), dim3(256), 0, s, x, dsc, part, rows, d);
  if ((rc = vqa::check_launch("vqa_head_bwd/wpool"))) return rc;
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(256), 0, s, dsc, rows, 1.0f, dbp);
  if ((rc = vqa::check_launch("vqa_head_bwd/dbp"))) return rc;
  return vqa_colsum_partials(part, parts, d, d, dwp, 0.f, s);
}
