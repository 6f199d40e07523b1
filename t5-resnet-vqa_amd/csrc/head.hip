// Answer head: AttentionPooler (resnet_vqa_model.py:14-26) + classification
// Linear(768, A) + log_softmax + NLLLoss(mean) (resnet_vqa_model.py:152-160),
// forward and backward.  Tiny (B x 170 x 768): fp32 throughout, straight from
// the fp32 master weights; one workgroup per sample plus deterministic
// reductions for the weight gradients.
#include "common.h"

namespace {

constexpr int MAXL = 64;
constexpr int MAXA = 1024;

__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wp,
                                                       const float* __restrict__ bp, const float* __restrict__ wc,
                                                       const float* __restrict__ bc,
                                                       const long long* __restrict__ targets, float* __restrict__ att,
                                                       float* __restrict__ pooled, float* __restrict__ logp,
                                                       float* __restrict__ nll, int L, int D, int A) {
  __shared__ float sc[MAXL];
  __shared__ float pl[1024];
  __shared__ float lg[MAXA];
  __shared__ float red[4];
  const int b = blockIdx.x, wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float* xb = x + (long)b * L * D;
  // scores[t] = x[t]·wp + bp
  for (int t = wv; t < L; t += 4) {
    float s = 0.f;
    for (int d = l; d < D; d += 64) s += xb[(long)t * D + d] * wp[d];
    s = wave_sum(s);
    if (l == 0) sc[t] = s + bp[0];
  }
  __syncthreads();
  if (wv == 0) {                                      // softmax over the sequence (Softmax(dim=1))
    const float s = l < L ? sc[l] : -INFINITY;
    const float m = wave_max(s);
    const float e = l < L ? __expf(s - m) : 0.f;
    const float z = wave_sum(e);
    if (l < L) { sc[l] = e / z; att[(long)b * L + l] = e / z; }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256) {        // pooled = a^T x
    float s = 0.f;
    for (int t = 0; t < L; ++t) s += sc[t] * xb[(long)t * D + d];
    pl[d] = s;
    pooled[(long)b * D + d] = s;
  }
  __syncthreads();
  for (int c = wv; c < A; c += 4) {                   // logits = pooled Wc^T + bc
    float s = 0.f;
    for (int d = l; d < D; d += 64) s += pl[d] * wc[(long)c * D + d];
    s = wave_sum(s);
    if (l == 0) lg[c] = s + bc[c];
  }
  __syncthreads();
  float m = -INFINITY;
  for (int c = threadIdx.x; c < A; c += 256) m = fmaxf(m, lg[c]);
  m = wave_max(m);
  if (l == 0) red[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float z = 0.f;
  for (int c = threadIdx.x; c < A; c += 256) z += __expf(lg[c] - m);
  z = wave_sum(z);
  if (l == 0) red[wv] = z;
  __syncthreads();
  const float lse = m + __logf(red[0] + red[1] + red[2] + red[3]);
  for (int c = threadIdx.x; c < A; c += 256) logp[(long)b * A + c] = lg[c] - lse;
  if (threadIdx.x == 0 && targets) nll[b] = -(lg[targets[b]] - lse);
}

__global__ void mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += v[i];
    out[0] = s / n;
  }
}

// per-sample backward: dlogits, dpooled, pooler backward -> dx; saves dlogits / dscore
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ x, const float* __restrict__ att,
                                                       const float* __restrict__ logp,
                                                       const long long* __restrict__ targets,
                                                       const float* __restrict__ wp, const float* __restrict__ wc,
                                                       float* __restrict__ dx32, bf16_t* __restrict__ dx16,
                                                       float* __restrict__ dlogits, float* __restrict__ dscore, int L,
                                                       int D, int A, float inv_b) {
  __shared__ float dl[MAXA];
  __shared__ float dp[1024];
  __shared__ float a[MAXL], da[MAXL];
  const int b = blockIdx.x, wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float* xb = x + (long)b * L * D;
  const long long t = targets[b];
  for (int c = threadIdx.x; c < A; c += 256) {
    const float g = (__expf(logp[(long)b * A + c]) - (c == t ? 1.f : 0.f)) * inv_b;
    dl[c] = g;
    dlogits[(long)b * A + c] = g;
  }
  for (int i = threadIdx.x; i < L; i += 256) a[i] = att[(long)b * L + i];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256) {
    float s = 0.f;
    for (int c = 0; c < A; ++c) s += dl[c] * wc[(long)c * D + d];
    dp[d] = s;
  }
  __syncthreads();
  for (int i = wv; i < L; i += 4) {
    float s = 0.f;
    for (int d = l; d < D; d += 64) s += dp[d] * xb[(long)i * D + d];
    s = wave_sum(s);
    if (l == 0) da[i] = s;
  }
  __syncthreads();
  if (wv == 0) {
    const float ai = l < L ? a[l] : 0.f, dai = l < L ? da[l] : 0.f;
    const float sum = wave_sum(ai * dai);
    if (l < L) {
      const float ds = ai * (dai - sum);
      da[l] = ds;
      dscore[(long)b * L + l] = ds;
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < L * D; idx += 256) {
    const int i = idx / D, d = idx - i * D;
    const float g = a[i] * dp[d] + da[i] * wp[d];
    dx32[(long)b * L * D + idx] = g;
    if (dx16) dx16[(long)b * L * D + idx] = f2bf(g);
  }
}

// dWc[c][d] = sum_b dlogits[b][c] pooled[b][d] ; dbc[c] = sum_b dlogits[b][c]
__global__ __launch_bounds__(256) void head_wgrad_cls_kernel(const float* __restrict__ dlogits,
                                                             const float* __restrict__ pooled, float* __restrict__ dwc,
                                                             float* __restrict__ dbc, int B, int D, int A) {
  const int c = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += 256) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlogits[(long)b * A + c] * pooled[(long)b * D + d];
    dwc[(long)c * D + d] = s;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlogits[(long)b * A + c];
    dbc[c] = s;
  }
}

// partials of dWp[d] = sum_rows dscore[row] x[row][d]  over 64-row chunks
__global__ __launch_bounds__(256) void head_wgrad_pool_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dscore, float* __restrict__ ws,
                                                              int rows, int D) {
  const int r0 = blockIdx.y * 64;
  for (int d = blockIdx.x * 256 + threadIdx.x; d < D; d += gridDim.x * 256) {
    float s = 0.f;
    for (int r = r0; r < min(rows, r0 + 64); ++r) s += dscore[r] * x[(long)r * D + d];
    ws[(long)blockIdx.y * D + d] = s;
  }
}

__global__ void sum_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += v[i];
    out[0] = s;
  }
}

}  // namespace

extern "C" int vqa_head_fwd(const float* x, const float* wp, const float* bp, const float* wc, const float* bc,
                            const long long* targets, float* att, float* pooled, float* logp, float* nll, float* loss,
                            int batch, int seq, int d, int answers, hipStream_t s) {
  VQA_REQUIRE(x && wp && bp && wc && bc && att && pooled && logp, "vqa_head_fwd: null argument");
  VQA_REQUIRE(seq <= MAXL && d <= 1024 && answers <= MAXA, "vqa_head_fwd: shape out of range");
  VQA_REQUIRE(!targets || (nll && loss), "vqa_head_fwd: targets need nll and loss outputs");
  hipLaunchKernelGGL(head_fwd_kernel, dim3(batch), dim3(256), 0, s, x, wp, bp, wc, bc, targets, att, pooled, logp, nll,
                     seq, d, answers);
  if (int rc = vqa::check_launch("vqa_head_fwd")) return rc;
  if (targets) {
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(64), 0, s, nll, batch, loss);
    return vqa::check_launch("vqa_head_fwd/mean");
  }
  return VQA_OK;
}

extern "C" int vqa_head_workspace_floats(int batch, int seq, int d, int answers) {
  return batch * answers + batch * seq + vqa::cdiv(batch * seq, 64) * d;
}

extern "C" int vqa_head_bwd(const float* x, const float* att, const float* pooled, const float* logp,
                            const long long* targets, const float* wp, const float* wc, float* dx32, void* dx16,
                            float* dwp, float* dbp, float* dwc, float* dbc, float* ws, int batch, int seq, int d,
                            int answers, hipStream_t s) {
  VQA_REQUIRE(x && att && pooled && logp && targets && wp && wc && dx32 && dwp && dbp && dwc && dbc && ws,
              "vqa_head_bwd: null argument");
  VQA_REQUIRE(seq <= MAXL && d <= 1024 && answers <= MAXA, "vqa_head_bwd: shape out of range");
  float* dlogits = ws;
  float* dscore = ws + batch * answers;
  float* part = dscore + batch * seq;
  hipLaunchKernelGGL(head_bwd_kernel, dim3(batch), dim3(256), 0, s, x, att, logp, targets, wp, wc, dx32, (bf16_t*)dx16,
                     dlogits, dscore, seq, d, answers, 1.0f / batch);
  if (int rc = vqa::check_launch("vqa_head_bwd")) return rc;
  hipLaunchKernelGGL(head_wgrad_cls_kernel, dim3(answers), dim3(256), 0, s, dlogits, pooled, dwc, dbc, batch, d,
                     answers);
  const int rows = batch * seq, parts = vqa::cdiv(rows, 64);
  hipLaunchKernelGGL(head_wgrad_pool_kernel, dim3(vqa::cdiv(d, 256), parts), dim3(256), 0, s, x, dscore, part, rows, d);
  if (int rc = vqa::check_launch("vqa_head_bwd/wgrad")) return rc;
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, s, dscore, rows, dbp);
  return vqa_colsum_partials(part, parts, d, d, dwp, 0.f, s);
}
