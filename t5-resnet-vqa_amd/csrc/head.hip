// Answer head: AttentionPooler (resnet_vqa_model.py:14-26) + classification
// Linear(768, A) (D up to 1024 for T5-large widths) + log_softmax + NLLLoss(mean) (resnet_vqa_model.py:152-160),
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

// Loads whose row/column may fall outside the tensor are issued UNconditionally
// at a clamped index and masked by a multiply: a "cond ? load : 0" (or a select
// of a loaded value, which hipcc sinks back into a branch) makes every load its
// own branch + vmcnt(0) wait (one L2 round trip per element,
// cdna_hip_programming.md §5 'Three .s-level traps' (c)).
//
// Forward, three launches (resnet_vqa_model.py:152-160):
//   head_pool_fwd      one workgroup per sample: scores, softmax over L, pooled row
//   head_logits        (8 answers) x (16 samples) per workgroup: logits = pooled Wc^T + bc
//   head_lse           one workgroup: log_softmax over the answers, NLL, mean loss over the B' rows
//                      whose target is >= 0 (nn.NLLLoss ignore_index: a short final batch padded to B)
// Backward, three launches:
//   head_dpooled       dlogits = (softmax - onehot)/B' and dpooled = dlogits Wc, 64 columns x
//                      16 samples per workgroup, the answer sum split over the 4 waves
//   head_pool_bwd      one workgroup per sample: pooler backward -> dx, and the sample's
//                      pooler-weight partial sum_l dscore_l x_l (the thread owns its columns)
//   head_wgrad         classifier dWc / dbc tiles (16 answers x 256 columns) and the fixed-order
//                      sum of the per-sample pooler partials, in one two-role launch
// Pooler kernels: 4 * PC4 threads = 4 row groups x PC4 float4 columns, PC4 = 192 for
// D <= 768 (T5-base) and 256 for D <= 1024 (T5-large), D % 4 == 0; a thread holds
// RPG = LMAX/4 rows of one float4 column in registers, so each sample is read once with
// 16-B loads and the 12 (16) waves of the workgroup share the instruction stream (one wave
// per SIMD spent ~4x longer issuing the scalar-load form).  Row sums: a reduce-scatter
// inside each wave, then the WPG = PC4/64 waves of the row group in a fixed order.
// (At 1024 threads the register cap is 128: the L > 32, D > 768 variants spill ~80 B/lane.)
template <int RPG, int WPG>
__device__ __forceinline__ void pool_row_sums(float (&part)[RPG], float* red /*[4*WPG][RPG]*/, float* out, int L) {
  constexpr int SH = RPG == 4 ? 4 : (RPG == 8 ? 3 : 2);   // lane >> SH = row index after the scatter
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float v = wave_sum_scatter<RPG>(part);
  if ((l & ((1 << SH) - 1)) == 0) red[wv * RPG + (l >> SH)] = v;
  __syncthreads();
  if (threadIdx.x < 4 * RPG) {                          // row r = group * RPG + i: waves WPG*g .. WPG*g+WPG-1
    const int g = threadIdx.x / RPG, i = threadIdx.x - g * RPG;
    if (g * RPG + i < L) {
      float t = red[(WPG * g) * RPG + i];
#pragma unroll
      for (int j = 1; j < WPG; ++j) t += red[(WPG * g + j) * RPG + i];
      out[g * RPG + i] = t;
    }
  }
  __syncthreads();
}

template <int LMAX, int PC4>
__global__ __launch_bounds__(4 * PC4) void head_pool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wp,
                                                            const float* __restrict__ bp, float* __restrict__ att,
                                                            float* __restrict__ pooled, int L, int D) {
  constexpr int RPG = LMAX / 4;
  constexpr int WPG = PC4 / 64;
  __shared__ float red[4 * WPG * RPG], sc[LMAX];
  __shared__ __attribute__((aligned(16))) float4 pr[4][PC4];
  const int b = blockIdx.x, tid = threadIdx.x, g = tid / PC4, c4 = tid - g * PC4, C4 = D / 4;
  const float cm = c4 < C4 ? 1.f : 0.f;
  const float4* xb = reinterpret_cast<const float4*>(x + (long)b * L * D) + min(c4, C4 - 1);
  const float4 w = reinterpret_cast<const float4*>(wp)[min(c4, C4 - 1)];
  float4 xr[RPG];
  float part[RPG];
#pragma unroll
  for (int i = 0; i < RPG; ++i) {
    const int r = g * RPG + i;
    const float4 v = xb[(long)min(r, L - 1) * C4];       // unconditional load, masked value
    const float m = (r < L) ? cm : 0.f;
    xr[i] = make_float4(v.x * m, v.y * m, v.z * m, v.w * m);
    part[i] = xr[i].x * w.x + xr[i].y * w.y + xr[i].z * w.z + xr[i].w * w.w;
  }
  pool_row_sums<RPG, WPG>(part, red, sc, L);
  if (tid < 64) {                                     // softmax over the sequence (Softmax(dim=1))
    const float s = tid < L ? sc[tid] + bp[0] : -INFINITY;
    const float m = wave_max(s);
    const float e = tid < L ? __expf(s - m) : 0.f;
    const float z = wave_sum(e);
    if (tid < L) { sc[tid] = e / z; att[(long)b * L + tid] = e / z; }
  }
  __syncthreads();
  float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RPG; ++i) {
    const float a = g * RPG + i < L ? sc[g * RPG + i] : 0.f;
    p.x = fmaf(a, xr[i].x, p.x); p.y = fmaf(a, xr[i].y, p.y); p.z = fmaf(a, xr[i].z, p.z); p.w = fmaf(a, xr[i].w, p.w);
  }
  pr[g][c4] = p;
  __syncthreads();
  if (g == 0 && c4 < C4) {                            // fixed order over the 4 row groups
    float4 o = pr[0][c4];
#pragma unroll
    for (int q = 1; q < 4; ++q) { o.x += pr[q][c4].x; o.y += pr[q][c4].y; o.z += pr[q][c4].z; o.w += pr[q][c4].w; }
    reinterpret_cast<float4*>(pooled + (long)b * D)[c4] = o;
  }
}

// logits[b, a] = pooled[b, :] . Wc[a, :] + bc[a] for 8 answers x 16 samples per workgroup:
// a lane holds float4 columns (lane, lane+64, ..., lane+64(NJ-1)) of the 8 Wc rows, each wave
// takes 4 samples; one wave_sum_scatter<8> per sample finishes 8 dots at once
// (D <= 256 NJ, D % 4 == 0: NJ = 3 for D <= 768, 4 for D <= 1024)
template <int NJ>
__global__ __launch_bounds__(256) void head_logits_kernel(const float* __restrict__ pooled,
                                                          const float* __restrict__ wc, const float* __restrict__ bc,
                                                          float* __restrict__ logits, int B, int D, int A) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int a0 = blockIdx.x * 8, s0 = blockIdx.y * 16 + wv * 4;
  float4 wr[8][NJ];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = 4 * (l + 64 * j), a = a0 + u;
      const float4 t = *reinterpret_cast<const float4*>(wc + (long)min(a, A - 1) * D + min(k, D - 4));
      const float m = (a < A && k < D) ? 1.f : 0.f;
      wr[u][j] = make_float4(t.x * m, t.y * m, t.z * m, t.w * m);
    }
  float4 pv[4][NJ];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = 4 * (l + 64 * j);
      const float4 t = *reinterpret_cast<const float4*>(pooled + (long)min(s0 + q, B - 1) * D + min(k, D - 4));
      const float m = k < D ? 1.f : 0.f;
      pv[q][j] = make_float4(t.x * m, t.y * m, t.z * m, t.w * m);
    }
  const int a = a0 + (l >> 3);
  const float bias = bc[min(a, A - 1)];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float sv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        s += pv[q][j].x * wr[u][j].x + pv[q][j].y * wr[u][j].y + pv[q][j].z * wr[u][j].z + pv[q][j].w * wr[u][j].w;
      sv[u] = s;
    }
    const float s = wave_sum_scatter<8>(sv);          // lane group l>>3 holds answer a0 + (l>>3)
    if ((l & 7) == 0 && a < A && s0 + q < B) logits[(long)(s0 + q) * A + a] = s + bias;
  }
}

// log_softmax over the answers (in place: logits -> log-probs), NLL of the target and the
// mean loss, one 1024-thread workgroup: wave w takes samples w, w+16, ... (A <= 1024)
template <int NI>                                      // answers per lane: A <= 64 * NI
__global__ __launch_bounds__(1024) void head_lse_kernel(float* __restrict__ lp, const long long* __restrict__ tgt,
                                                        float* __restrict__ nll, float* __restrict__ loss, int B,
                                                        int A) {
  __shared__ float nl[1024];
  __shared__ int nv[1024];                             // row b has a target >= 0 (not ignored)
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int b0 = wv * 4; b0 < B; b0 += 64) {            // 4 samples per wave and pass, all loads first
    float v[4][NI];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < NI; ++i) v[q][i] = lp[(long)min(b0 + q, B - 1) * A + min(l + 64 * i, A - 1)];
    int t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = tgt ? (int)tgt[min(b0 + q, B - 1)] : -1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int b = b0 + q;
      float m = -INFINITY;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        if (l + 64 * i < A) m = fmaxf(m, v[q][i]);
      m = wave_max(m);
      float z = 0.f, vt = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (l + 64 * i < A) z += __expf(v[q][i] - m);
        if (l + 64 * i == t[q]) vt = v[q][i];
      }
      const float lse = m + __logf(wave_sum(z));
      vt = wave_sum(vt);                                // the one lane holding the target
      if (b < B) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (l + 64 * i < A) lp[(long)b * A + l + 64 * i] = v[q][i] - lse;
        if (tgt && l == 0) {                            // ignore_index rows: nll 0, not in the mean
          const float v = t[q] >= 0 ? -(vt - lse) : 0.f;
          nl[b & 1023] = v;
          nv[b & 1023] = t[q] >= 0;
          nll[b] = v;
        }
      }
    }
  }
  if (!tgt) return;
  __syncthreads();
  if (threadIdx.x == 0) {                             // fixed-order mean (NLLLoss reduction='mean')
    float s = 0.f;
    int n = 0;
    for (int b = 0; b < B; ++b) { s += nl[b]; n += nv[b]; }
    loss[0] = s / (float)n;                           // n = B for a full batch: s / B as before
  }
}

// dlogits (kept for the classifier weight gradient) and dpooled = dlogits Wc.
// Workgroup = 64 columns x 16 samples; the answers go in chunks of 4 * AQ = 192 (one chunk
// for DAQUAR's 170): in each chunk wave w sums answers [c + w*AQ, c + (w+1)*AQ) with all of
// its Wc loads in flight, carrying its partial from chunk to chunk; the four wave partials
// are then added in a fixed order through LDS.
constexpr int DP_AQ = 48;                             // answers per wave and chunk
template <bool CHUNKED>                               // false: A <= 192, one chunk (straight-line code)
__global__ __launch_bounds__(256) void head_dpooled_kernel(const float* __restrict__ lp,
                                                           const long long* __restrict__ tgt,
                                                           const float* __restrict__ wc, float* __restrict__ dl_out,
                                                           float* __restrict__ dpooled, int B, int D, int A,
                                                           const float* __restrict__ nll, float* __restrict__ loss,
                                                           const float* __restrict__ row_total, float row_scale) {
  constexpr int AP = 4 * DP_AQ;                       // padded answer row in LDS
  __shared__ __attribute__((aligned(16))) float dl[16][AP];
  __shared__ float red[4][16][64];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int c = blockIdx.x * 64 + l, s0 = blockIdx.y * 16;
  constexpr int FI = 16 * AP / 256;                   // fill elements per thread (all loads first)
  // the NLL mean's divisor: rows with a target >= 0 (ignore_index rows get no gradient); a full
  // batch gives 1 / B exactly as the host-computed factor did
  // Data parallel (row_total set): the divisor is the valid-row count summed over the ranks,
  // row_total[0], over row_scale = the world size, so that the ranks' gradients, summed and
  // scaled by 1/world in the update, are the global batch's NLL mean whatever each rank's rows
  // (a rank with no valid row contributes zero).  The rank's loss is rewritten the same way:
  // sum(nll) * world / total, whose mean over the ranks is the global batch's loss.
  float inv_b;
  if (row_total) {
    inv_b = row_scale / row_total[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
      float s = 0.f;                                    // the forward's fixed order (head_lse)
      for (int b = 0; b < B; ++b) s += nll[b];
      loss[0] = (s * row_scale) / row_total[0];
    }
  } else {
    int nvalid = 0;
    for (int b0 = 0; b0 < B; b0 += 256) nvalid += __syncthreads_count(b0 + tid < B && tgt[min(b0 + tid, B - 1)] >= 0);
    inv_b = 1.0f / (float)nvalid;
  }
  float acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  for (int c0 = 0; c0 < (CHUNKED ? A : 1); c0 += AP) {
    float ev[FI];
    int tv[FI];
#pragma unroll
    for (int k = 0; k < FI; ++k) {
      const int i = tid + 256 * k, q = i / AP, a = c0 + i - q * AP, b = min(s0 + q, B - 1);
      ev[k] = lp[(long)b * A + min(a, A - 1)];
      tv[k] = (int)tgt[b];
    }
    if (c0) __syncthreads();                          // the previous chunk's dl has been read
#pragma unroll
    for (int k = 0; k < FI; ++k) {
      const int i = tid + 256 * k, q = i / AP, j = i - q * AP, a = c0 + j, b = s0 + q;
      const float g = (b < B && a < A && tv[k] >= 0) ? (__expf(ev[k]) - (a == tv[k] ? 1.f : 0.f)) * inv_b : 0.f;
      dl[q][j] = g;
      if (blockIdx.x == 0 && b < B && a < A) dl_out[(long)b * A + a] = g;
    }
    float w[DP_AQ];
#pragma unroll
    for (int i = 0; i < DP_AQ; ++i)
      w[i] = wc[(long)min(c0 + wv * DP_AQ + i, A - 1) * D + min(c, D - 1)];   // masked through dl = 0 past A
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float s = acc[q];                                 // 0 in the first chunk: A <= 192 sums as before
#pragma unroll
      for (int i = 0; i < DP_AQ; i += 4) {
        const float4 g = *reinterpret_cast<const float4*>(&dl[q][wv * DP_AQ + i]);
        s = fmaf(g.x, w[i], s);
        s = fmaf(g.y, w[i + 1], s);
        s = fmaf(g.z, w[i + 2], s);
        s = fmaf(g.w, w[i + 3], s);
      }
      acc[q] = s;
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) red[wv][q][l] = acc[q];
  __syncthreads();
  for (int i = tid; i < 16 * 64; i += 256) {
    const int q = i >> 6, cl = i & 63, b = s0 + q, cc = blockIdx.x * 64 + cl;
    const float v = ((red[0][q][cl] + red[1][q][cl]) + red[2][q][cl]) + red[3][q][cl];
    if (b < B && cc < D) dpooled[(long)b * D + cc] = v;
  }
}

// Pooler backward of one sample: da = x dpooled ; dscore = a (da - sum a da) ;
// dx = a dpooled^T + dscore wp^T ; and the sample's pooler weight / bias partials
// part[b, d] = sum_l dscore_l x[l, d], pbp[b] = sum_l dscore_l (summed over b by head_wgrad).
// Same 4 row groups x PC4 float4 columns layout as head_pool_fwd_kernel.
template <int LMAX, int PC4>
__global__ __launch_bounds__(4 * PC4) void head_pool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ att,
                                                            const float* __restrict__ dpooled,
                                                            const float* __restrict__ wp, float* __restrict__ dx32,
                                                            bf16_t* __restrict__ dx16, float* __restrict__ part,
                                                            float* __restrict__ pbp, int L, int D) {
  constexpr int RPG = LMAX / 4;
  constexpr int WPG = PC4 / 64;
  __shared__ float red[4 * WPG * RPG], da[LMAX], a[LMAX];
  __shared__ __attribute__((aligned(16))) float4 pr[4][PC4];
  const int b = blockIdx.x, tid = threadIdx.x, g = tid / PC4, c4 = tid - g * PC4, C4 = D / 4;
  const float cm = c4 < C4 ? 1.f : 0.f;
  if (tid < L) a[tid] = att[(long)b * L + tid];
  const float4* xb = reinterpret_cast<const float4*>(x + (long)b * L * D) + min(c4, C4 - 1);
  const float4 w = reinterpret_cast<const float4*>(wp)[min(c4, C4 - 1)];
  float4 dp = reinterpret_cast<const float4*>(dpooled + (long)b * D)[min(c4, C4 - 1)];
  dp = make_float4(dp.x * cm, dp.y * cm, dp.z * cm, dp.w * cm);
  float4 xr[RPG];
  float pt[RPG];
#pragma unroll
  for (int i = 0; i < RPG; ++i) {
    const int r = g * RPG + i;
    const float4 v = xb[(long)min(r, L - 1) * C4];       // unconditional load, masked value
    const float m = (r < L) ? cm : 0.f;
    xr[i] = make_float4(v.x * m, v.y * m, v.z * m, v.w * m);
    pt[i] = xr[i].x * dp.x + xr[i].y * dp.y + xr[i].z * dp.z + xr[i].w * dp.w;
  }
  pool_row_sums<RPG, WPG>(pt, red, da, L);
  if (tid < 64) {
    const float ai = tid < L ? a[tid] : 0.f, dai = tid < L ? da[tid] : 0.f;
    const float s = wave_sum(ai * dai);
    const float ds = tid < L ? ai * (dai - s) : 0.f;
    if (tid < L) da[tid] = ds;
    const float tot = wave_sum(ds);
    if (tid == 0) pbp[b] = tot;
  }
  __syncthreads();
  float4 pw = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RPG; ++i) {
    const int r = g * RPG + i;
    if (r >= L) continue;
    const float ar = a[r], dr = da[r];
    pw.x = fmaf(dr, xr[i].x, pw.x); pw.y = fmaf(dr, xr[i].y, pw.y);
    pw.z = fmaf(dr, xr[i].z, pw.z); pw.w = fmaf(dr, xr[i].w, pw.w);
    if (c4 >= C4) continue;
    const float4 o = make_float4(ar * dp.x + dr * w.x, ar * dp.y + dr * w.y, ar * dp.z + dr * w.z,
                                 ar * dp.w + dr * w.w);
    const long e = ((long)b * L + r) * D + 4 * c4;
    *reinterpret_cast<float4*>(dx32 + e) = o;
    if (dx16) {
      uint2 u;
      u.x = (uint32_t)f2bf(o.x) | ((uint32_t)f2bf(o.y) << 16);
      u.y = (uint32_t)f2bf(o.z) | ((uint32_t)f2bf(o.w) << 16);
      *reinterpret_cast<uint2*>(dx16 + e) = u;
    }
  }
  pr[g][c4] = pw;
  __syncthreads();
  if (g == 0 && c4 < C4) {                            // fixed order over the 4 row groups
    float4 o = pr[0][c4];
#pragma unroll
    for (int q = 1; q < 4; ++q) { o.x += pr[q][c4].x; o.y += pr[q][c4].y; o.z += pr[q][c4].z; o.w += pr[q][c4].w; }
    reinterpret_cast<float4*>(part + (long)b * D)[c4] = o;
  }
}

// Two roles, fixed-order sums over the B samples:
//   blocks [0, nca * ncd): dWc[a, c] = sum_b dl[b, a] pooled[b, c] for 16 answers x 256 columns
//     (thread = column, 16 accumulators), dbc[a] = sum_b dl[b, a] (column block 0)
//   blocks [nca * ncd, + ncd): dWp[c] = sum_b part[b, c], dbp = sum_b pbp[b]
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ dl, const float* __restrict__ pooled,
                                                         const float* __restrict__ part, const float* __restrict__ pbp,
                                                         float* __restrict__ dwc, float* __restrict__ dbc,
                                                         float* __restrict__ dwp, float* __restrict__ dbp, int B, int A,
                                                         int D) {
  __shared__ __attribute__((aligned(16))) float cf[64][16];
  const int tid = threadIdx.x, ncd = (D + 255) / 256, nca = (A + 15) / 16;
  const int blk = blockIdx.x;
  if (blk < nca * ncd) {
    const int a0 = (blk / ncd) * 16, c = (blk % ncd) * 256 + tid;
    float acc[16], csum = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc[u] = 0.f;
    for (int b0 = 0; b0 < B; b0 += 64) {
      const int bn = min(64, B - b0);
      __syncthreads();
      for (int i = tid; i < 64 * 16; i += 256) {
        const int q = i >> 4, u = i & 15;
        const float v = dl[(long)(b0 + min(q, bn - 1)) * A + min(a0 + u, A - 1)];
        cf[q][u] = (q < bn && a0 + u < A) ? v : 0.f;
      }
      __syncthreads();
      if (tid < 16)                                     // dbc: the staged coefficients, fixed order
        for (int q = 0; q < 64; ++q) csum += cf[q][tid];
      float pv[64];
#pragma unroll
      for (int q = 0; q < 64; ++q) pv[q] = pooled[(long)(b0 + min(q, bn - 1)) * D + min(c, D - 1)];
#pragma unroll
      for (int q = 0; q < 64; ++q) {
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
          const float4 g = *reinterpret_cast<const float4*>(&cf[q][u]);   // zero past bn / A
          acc[u] = fmaf(g.x, pv[q], acc[u]);
          acc[u + 1] = fmaf(g.y, pv[q], acc[u + 1]);
          acc[u + 2] = fmaf(g.z, pv[q], acc[u + 2]);
          acc[u + 3] = fmaf(g.w, pv[q], acc[u + 3]);
        }
      }
    }
    if (c < D)
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (a0 + u < A) dwc[(long)(a0 + u) * D + c] = acc[u];
    if (blk % ncd == 0 && tid < 16 && a0 + tid < A) dbc[a0 + tid] = csum;
  } else {
    const int c = (blk - nca * ncd) * 256 + tid;
    float s = 0.f;
    for (int b0 = 0; b0 < B; b0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = part[(long)min(b0 + u, B - 1) * D + min(c, D - 1)];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (b0 + u < B) s += v[u];
    }
    if (c < D) dwp[c] = s;
    if (blk == nca * ncd) {                           // dbp: stage pbp in LDS, one thread sums in order
      for (int b0 = 0; b0 < B; b0 += 256) {
        __syncthreads();
        if (b0 + tid < B) cf[tid >> 4][tid & 15] = pbp[b0 + tid];
        __syncthreads();
        if (tid == 0) {
          float t = b0 ? dbp[0] : 0.f;
          for (int q = 0; q < min(256, B - b0); ++q) t += cf[q >> 4][q & 15];
          dbp[0] = t;
        }
      }
    }
  }
}

template <typename F>
int with_lmax(int L, F f) {
  if (L <= 16) return f(std::integral_constant<int, 16>());
  if (L <= 32) return f(std::integral_constant<int, 32>());
  return f(std::integral_constant<int, 64>());
}

// float4 columns per pooler row group: 192 up to D = 768 (unchanged T5-base kernels), 256 up to 1024
template <typename F>
int with_pc4(int D, F f) {
  if (D <= 768) return f(std::integral_constant<int, 192>());
  return f(std::integral_constant<int, 256>());
}

}  // namespace

extern "C" int vqa_head_workspace_floats(int batch, int seq, int d, int answers) {
  (void)seq;
  return batch + batch * answers + 2 * batch * d;
}

// logits go through `logp` (head_logits writes them, head_lse turns them into log-probs in place)
extern "C" int vqa_head_fwd(const float* x, const float* wp, const float* bp, const float* wc, const float* bc,
                            const long long* targets, float* att, float* pooled, float* logp, float* nll, float* loss,
                            int batch, int seq, int d, int answers, hipStream_t s) {
  VQA_REQUIRE(x && wp && bp && wc && bc && att && pooled && logp, "vqa_head_fwd: null argument");
  VQA_REQUIRE(seq >= 1 && seq <= 64 && d >= 4 && d <= 1024 && d % 4 == 0 && answers >= 1 && answers <= MAXA &&
                  batch >= 1 && batch <= 1024,
              "vqa_head_fwd: shape out of range (1<=L<=64, 4<=D<=1024, D%4==0, 1<=A<=1024, 1<=B<=1024)");
  VQA_REQUIRE(!targets || (nll && loss), "vqa_head_fwd: targets need nll and loss outputs");
  int rc = with_lmax(seq, [&](auto lm) {
    return with_pc4(d, [&](auto pc) {
      hipLaunchKernelGGL((head_pool_fwd_kernel<decltype(lm)::value, decltype(pc)::value>), dim3(batch),
                         dim3(4 * decltype(pc)::value), 0, s, x, wp, bp, att, pooled, seq, d);
      return vqa::check_launch("vqa_head_fwd/pool");
    });
  });
  if (rc) return rc;
  const dim3 lg(vqa::cdiv(answers, 8), vqa::cdiv(batch, 16));
  if (d <= 768)
    hipLaunchKernelGGL(head_logits_kernel<3>, lg, dim3(256), 0, s, pooled, wc, bc, logp, batch, d, answers);
  else
    hipLaunchKernelGGL(head_logits_kernel<4>, lg, dim3(256), 0, s, pooled, wc, bc, logp, batch, d, answers);
  if ((rc = vqa::check_launch("vqa_head_fwd/logits"))) return rc;
  if (answers <= 256)
    hipLaunchKernelGGL(head_lse_kernel<4>, dim3(1), dim3(1024), 0, s, logp, targets, nll, loss, batch, answers);
  else
    hipLaunchKernelGGL(head_lse_kernel<16>, dim3(1), dim3(1024), 0, s, logp, targets, nll, loss, batch, answers);
  return vqa::check_launch("vqa_head_fwd/lse");
}

// ws layout: pbp [B] | dlogits [B*A] | dpooled [B*D] | pooler partials [B*D]
extern "C" int vqa_head_bwd(const float* x, const float* att, const float* pooled, const float* logp,
                            const long long* targets, const float* wp, const float* wc, float* dx32, void* dx16,
                            float* dwp, float* dbp, float* dwc, float* dbc, float* ws, int batch, int seq, int d,
                            int answers, const float* nll, float* loss, const float* row_total, float row_scale,
                            hipStream_t s) {
  VQA_REQUIRE(x && att && pooled && logp && targets && wp && wc && dx32 && dwp && dbp && dwc && dbc && ws,
              "vqa_head_bwd: null argument");
  VQA_REQUIRE(!row_total || (nll && loss && row_scale > 0.f),
              "vqa_head_bwd: a global row total needs nll, loss and row_scale > 0");
  VQA_REQUIRE(seq >= 1 && seq <= 64 && d >= 4 && d <= 1024 && d % 4 == 0 && answers >= 1 && answers <= MAXA &&
                  batch >= 1 && batch <= 1024,
              "vqa_head_bwd: shape out of range (1<=L<=64, 4<=D<=1024, D%4==0, 1<=A<=1024, 1<=B<=1024)");
  float* pbp = ws;
  float* dl = pbp + batch;
  float* dpool = dl + batch * answers;
  float* part = dpool + batch * d;
  const dim3 dg(vqa::cdiv(d, 64), vqa::cdiv(batch, 16));
  if (answers <= 4 * DP_AQ)
    hipLaunchKernelGGL(head_dpooled_kernel<false>, dg, dim3(256), 0, s, logp, targets, wc, dl, dpool, batch, d, answers,
                       nll, loss, row_total, row_scale);
  else
    hipLaunchKernelGGL(head_dpooled_kernel<true>, dg, dim3(256), 0, s, logp, targets, wc, dl, dpool, batch, d, answers,
                       nll, loss, row_total, row_scale);
  int rc = vqa::check_launch("vqa_head_bwd/dpooled");
  if (rc) return rc;
  rc = with_lmax(seq, [&](auto lm) {
    return with_pc4(d, [&](auto pc) {
      hipLaunchKernelGGL((head_pool_bwd_kernel<decltype(lm)::value, decltype(pc)::value>), dim3(batch),
                         dim3(4 * decltype(pc)::value), 0, s, x, att, dpool, wp, dx32, (bf16_t*)dx16, part, pbp, seq,
                         d);
      return vqa::check_launch("vqa_head_bwd/pool");
    });
  });
  if (rc) return rc;
  const int ncd = vqa::cdiv(d, 256), nca = vqa::cdiv(answers, 16);
  hipLaunchKernelGGL(head_wgrad_kernel, dim3(nca * ncd + ncd), dim3(256), 0, s, dl, pooled, part, pbp, dwc, dbc, dwp, dbp,
                     batch, answers, d);
  return vqa::check_launch("vqa_head_bwd/wgrad");
}

// Valid rows of a batch (targets >= 0, i.e. not ignore_index) as a float, one workgroup: the
// data-parallel step all-reduces it into vqa_head_bwd's row_total before the backward.
namespace {
__global__ __launch_bounds__(256) void count_targets_kernel(const long long* __restrict__ tgt, int B,
                                                            float* __restrict__ out) {
  const int tid = threadIdx.x;
  int n = 0;
  for (int b0 = 0; b0 < B; b0 += 256) n += __syncthreads_count(b0 + tid < B && tgt[min(b0 + tid, B - 1)] >= 0);
  if (tid == 0) out[0] = (float)n;
}
}  // namespace

extern "C" int vqa_count_targets(const long long* targets, int batch, float* out, hipStream_t s) {
  VQA_REQUIRE(targets && out && batch >= 1 && batch <= 1024, "vqa_count_targets: null argument or batch out of 1..1024");
  hipLaunchKernelGGL(count_targets_kernel, dim3(1), dim3(256), 0, s, targets, batch, out);
  return vqa::check_launch("vqa_count_targets");
}
