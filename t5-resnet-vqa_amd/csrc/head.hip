// Answer head: AttentionPooler (resnet_vqa_model.py:14-26) + classification
// Linear(768, A) + log_softmax + NLLLoss(mean) (resnet_vqa_model.py:152-160),
// forward and backward, fp32 end to end (straight from the fp32 masters).
//   pooler kernels: one workgroup per sample, each thread keeps its D/256
//     columns of all L rows in registers, so scores, softmax, pooling and the
//     pooler backward need a single read of the sample;
//   classifier: logits fused into the forward kernel, dpooled into the
//     per-sample backward kernel, dWc/dbc and the pooler weight partials in one
//     two-role launch;
//   every reduction runs in a fixed order (bit-reproducible).
#include <type_traits>

#include "common.h"

namespace {

constexpr int MAXA = 1024;

// ------------------------------------------------------------ pooler
// block-wide reduction of NV per-thread vectors of length L (one value per row t)
template <int LMAX>
__device__ __forceinline__ void block_row_sums(float (&part)[LMAX], int L, float* red /*[4][LMAX]*/,
                                               float* out /*[LMAX]*/) {
  constexpr int SH = LMAX == 16 ? 2 : (LMAX == 32 ? 1 : 0);     // lane >> SH = row index after the scatter
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float v = wave_sum_scatter<LMAX>(part);
  if ((l & ((1 << SH) - 1)) == 0) red[wv * LMAX + (l >> SH)] = v;
  __syncthreads();
  for (int t = threadIdx.x; t < L; t += 256) out[t] = red[t] + red[LMAX + t] + red[2 * LMAX + t] + red[3 * LMAX + t];
  __syncthreads();
}

// Loads whose row/column may fall outside the tensor are issued UNconditionally
// at a clamped index and masked by a multiply: a "cond ? load : 0" (or a select
// of a loaded value, which hipcc sinks back into a branch) makes every load its
// own branch + vmcnt(0) wait (one L2 round trip per element,
// cdna_hip_programming.md §5 'Three .s-level traps' (c)).
//
// The whole forward head of one sample in one workgroup (resnet_vqa_model.py:152-160):
// pooler (scores, softmax over L, weighted sum) -> pooled row in LDS -> 170 logits, one wave per
// answer at a time, lanes striding the D-long dot so the Wc row read is one
// coalesced 256-B access per step -> log_softmax over the answers in LDS -> NLL.
template <int LMAX>
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wp,
                                                       const float* __restrict__ bp, const float* __restrict__ wc,
                                                       const float* __restrict__ bc, const long long* __restrict__ tgt,
                                                       float* __restrict__ att, float* __restrict__ pooled,
                                                       float* __restrict__ logp, float* __restrict__ nll, int L, int D,
                                                       int A) {
  constexpr int NC = 3;
  __shared__ float red[4 * LMAX], sc[LMAX], lg[MAXA], r4[4];
  __shared__ __attribute__((aligned(16))) float pr[768];
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
      const float v = xb[(long)min(t, L - 1) * D + min(d, D - 1)];   // unconditional load, masked value
      xr[t][j] = v * ((t < L && d < D) ? 1.f : 0.f);
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
  // logits = pooled Wc^T + bc: each wave takes 8 answers per pass; a lane holds 12
  // pooled values (float4 columns lane, lane+64, lane+128) and issues its 24 Wc float4
  // loads before the first FMA, so a pass costs one L2 round trip (D <= 768)
  {
    float4 pv[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int k = 4 * (l + 64 * j);
      pv[j] = k < D ? *reinterpret_cast<const float4*>(pr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int a0 = 8 * wv; a0 < A; a0 += 32) {
      float4 wr[8][3];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int k = 4 * (l + 64 * j), a = a0 + u;
          const float4 t = *reinterpret_cast<const float4*>(wc + (long)min(a, A - 1) * D + min(k, D - 4));
          const float m = (a < A && k < D) ? 1.f : 0.f;
          wr[u][j] = make_float4(t.x * m, t.y * m, t.z * m, t.w * m);
        }
      float sv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j)
          s += pv[j].x * wr[u][j].x + pv[j].y * wr[u][j].y + pv[j].z * wr[u][j].z + pv[j].w * wr[u][j].w;
        sv[u] = s;
      }
      const float s = wave_sum_scatter<8>(sv);          // lane group l>>3 holds answer a0 + (l>>3)
      const int a = a0 + (l >> 3);
      if ((l & 7) == 0 && a < A) lg[a] = s + bc[a];
    }
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

// Backward of one sample in one workgroup: dlogits = (softmax - onehot)/B (kept
// for the classifier weight gradient), dpooled = dlogits Wc (each thread its
// D/256 columns, Wc rows read coalesced), then the pooler backward:
// da = x dpooled ; dscore = a (da - sum a da) ; dx = a dpooled^T + dscore wp^T.
template <int LMAX>
__global__ __launch_bounds__(256) void head_bwd_sample_kernel(
    const float* __restrict__ x, const float* __restrict__ att, const float* __restrict__ logp,
    const long long* __restrict__ tgt, const float* __restrict__ wc, const float* __restrict__ wp,
    float* __restrict__ dl_out, float* __restrict__ dx32, bf16_t* __restrict__ dx16, float* __restrict__ dscore, int L,
    int D, int A, float inv_b) {
  constexpr int NC = 3;
  __shared__ float red[4 * LMAX], da[LMAX], a[LMAX], dl[MAXA];
  const int b = blockIdx.x, tid = threadIdx.x;
  const long long t = tgt[b];
  for (int c = tid; c < A; c += 256) {
    const float g = (__expf(logp[(long)b * A + c]) - (c == t ? 1.f : 0.f)) * inv_b;
    dl[c] = g;
    dl_out[(long)b * A + c] = g;
  }
  for (int s = tid; s < L; s += 256) a[s] = att[(long)b * L + s];
  __syncthreads();
  // dpooled: 16 answers x 3 columns of Wc in flight per thread (coalesced rows)
  float dp[NC] = {0.f, 0.f, 0.f}, w[NC];
  for (int c0 = 0; c0 < A; c0 += 16) {
    float wv[16][NC];
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int d = tid + 256 * j;
        const float v = wc[(long)min(c0 + u, A - 1) * D + min(d, D - 1)];
        wv[u][j] = v * ((c0 + u < A && d < D) ? 1.f : 0.f);
      }
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int j = 0; j < NC; ++j) dp[j] = fmaf(c0 + u < A ? dl[c0 + u] : 0.f, wv[u][j], dp[j]);
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) w[j] = tid + 256 * j < D ? wp[tid + 256 * j] : 0.f;
  const float* xb = x + (long)b * L * D;
  float xr[LMAX][NC], part[LMAX];
#pragma unroll
  for (int s = 0; s < LMAX; ++s) {
    part[s] = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      const float v = xb[(long)min(s, L - 1) * D + min(d, D - 1)];   // unconditional load, masked value
      xr[s][j] = v * ((s < L && d < D) ? 1.f : 0.f);
      part[s] = fmaf(xr[s][j], dp[j], part[s]);
    }
  }
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
  for (int s = 0; s < LMAX; ++s) {
    if (s >= L) continue;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      if (d >= D) continue;
      const float g = a[s] * dp[j] + da[s] * w[j];
      dx32[((long)b * L + s) * D + d] = g;
      if (dx16) dx16[((long)b * L + s) * D + d] = f2bf(g);
    }
  }
}

// Weight gradients of the head, two workgroup roles in one launch:
//   blocks [0, A): classifier row a: dWc[a, :] = sum_b dl[b, a] pooled[b, :], dbc[a] = sum_b dl[b, a]
//   blocks [A, A + parts): pooler partials over a 64-row chunk p:
//     part[p, :] = sum_rows dscore[row] x[row, :], pbp[p] = sum_rows dscore[row]
// (fixed-order sums; the partials are reduced by head_pool_final_kernel)
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ dl, const float* __restrict__ pooled,
                                                         const float* __restrict__ x, const float* __restrict__ ds,
                                                         float* __restrict__ dwc, float* __restrict__ dbc,
                                                         float* __restrict__ part, float* __restrict__ pbp, int B,
                                                         int A, int rows, int D) {
  // both roles: out[d] = sum_{r in [r0, r1)} coef[r] * src[r, d] for the thread's 3
  // columns, 16 rows x 3 columns of loads in flight per thread (fixed row order)
  const int blk = blockIdx.x, tid = threadIdx.x;
  __shared__ float cf[64];
  const bool cls = blk < A;
  const int r0 = cls ? 0 : (blk - A) * 64, r1 = cls ? B : min(rows, r0 + 64);
  const float* srcm = cls ? pooled : x;
  float acc[3] = {0.f, 0.f, 0.f}, csum = 0.f;
  for (int c0 = r0; c0 < r1; c0 += 64) {             // coefficient chunks of 64 rows
    const int cn = min(64, r1 - c0);
    __syncthreads();
    for (int r = tid; r < cn; r += 256) cf[r] = cls ? dl[(long)(c0 + r) * A + blk] : ds[c0 + r];
    __syncthreads();
    for (int q0 = 0; q0 < cn; q0 += 16) {
      float v[16][3];
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int d = tid + 256 * j;
          const float t = srcm[(long)(c0 + min(q0 + u, cn - 1)) * D + min(d, D - 1)];
          v[u][j] = t * ((q0 + u < cn && d < D) ? 1.f : 0.f);
        }
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = fmaf(q0 + u < cn ? cf[q0 + u] : 0.f, v[u][j], acc[j]);
    }
    if (tid == 0)
      for (int r = 0; r < cn; ++r) csum += cf[r];
  }
  float* out = cls ? dwc + (long)blk * D : part + (long)(blk - A) * D;
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (tid + 256 * j < D) out[tid + 256 * j] = acc[j];
  if (tid == 0) {
    if (cls) dbc[blk] = csum; else pbp[blk - A] = csum;
  }
}

// dWp[d] = sum_p part[p, d], dbp = sum_p pbp[p]   (fixed order)
__global__ __launch_bounds__(256) void head_pool_final_kernel(const float* __restrict__ part,
                                                              const float* __restrict__ pbp, int parts, int D,
                                                              float* __restrict__ dwp, float* __restrict__ dbp) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d < D) {
    float s = 0.f;
    for (int p = 0; p < parts; ++p) s += part[(long)p * D + d];
    dwp[d] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int p = 0; p < parts; ++p) s += pbp[p];
    dbp[0] = s;
  }
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
  VQA_REQUIRE(seq <= 64 && d <= 768 && d % 4 == 0 && answers <= MAXA,
              "vqa_head_fwd: shape out of range (L<=64, D<=768, D%4==0)");
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
  const int rows = batch * seq, parts = vqa::cdiv(rows, 64);
  float* pbp = ws;                                   // [parts] (parts <= batch*answers)
  float* dl = ws + batch * answers;                  // [B, A]
  float* dsc = dl + batch * answers + batch * d;     // [B*L]
  float* part = dsc + batch * seq;                   // [parts, D]
  int rc = with_lmax(seq, [&](auto lm) {
    hipLaunchKernelGGL(head_bwd_sample_kernel<decltype(lm)::value>, dim3(batch), dim3(256), 0, s, x, att, logp,
                       targets, wc, wp, dl, dx32, (bf16_t*)dx16, dsc, seq, d, answers, 1.0f / batch);
    return vqa::check_launch("vqa_head_bwd/sample");
  });
  if (rc) return rc;
  hipLaunchKernelGGL(head_wgrad_kernel, dim3(answers + parts), dim3(256), 0, s, dl, pooled, x, dsc, dwc, dbc, part, pbp,
                     batch, answers, rows, d);
  if ((rc = vqa::check_launch("vqa_head_bwd/wgrad"))) return rc;
  hipLaunchKernelGGL(head_pool_final_kernel, dim3(vqa::cdiv(d, 256)), dim3(256), 0, s, part, pbp, parts, d, dwp, dbp);
  return vqa::check_launch("vqa_head_bwd/final");
}
