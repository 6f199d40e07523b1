// Stand-alone timing of the answer-head kernels (includes head.hip directly):
// per-kernel HIP-event times at B=64, L=32, D=768, A=170, so a change to one
// kernel can be judged in isolation.   hipcc --offload-arch=gfx950 -O3 -I../../include
#include "../../t5-resnet-vqa_amd/csrc/head.hip"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)


// phase-truncated copy of head_fwd_kernel: STOP = 1 after the x loads, 2 after the
// row sums, 3 after pooling, 4 after the logits, 5 = whole kernel
template <int LMAX, int STOP>
__global__ __launch_bounds__(256) void head_probe(const float* __restrict__ x, const float* __restrict__ wp,
                                                  const float* __restrict__ bp, const float* __restrict__ wc,
                                                  const float* __restrict__ bc, float* __restrict__ out, int L, int D,
                                                  int A) {
  constexpr int NC = 3;
  __shared__ float red[4 * LMAX], sc[LMAX], lg[MAXA];
  __shared__ __attribute__((aligned(16))) float pr[768];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const float* xb = x + (long)b * L * D;
  float xr[LMAX][NC], part[LMAX];
  float w[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) w[j] = wp[tid + 256 * j];
#pragma unroll
  for (int t = 0; t < LMAX; ++t) {
    part[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int d = tid + 256 * j;
      xr[t][j] = xb[(long)t * D + d];
      part[t] = fmaf(xr[t][j], w[j], part[t]);
    }
  }
  if (STOP == 1) { float s = 0; for (int t = 0; t < LMAX; ++t) s += part[t]; out[b * 256 + tid] = s; return; }
  block_row_sums<LMAX>(part, L, red, sc);
  if (STOP == 2) { out[b * 256 + tid] = sc[tid & (LMAX - 1)] + xr[3][1]; return; }
  if (tid < 64) {
    const float s = tid < L ? sc[tid] + bp[0] : -INFINITY;
    const float m = wave_max(s);
    const float e = tid < L ? __expf(s - m) : 0.f;
    const float z = wave_sum(e);
    if (tid < L) sc[tid] = e / z;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int d = tid + 256 * j;
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < LMAX; ++t) p = fmaf(sc[t], xr[t][j], p);
    pr[d] = p;
  }
  __syncthreads();
  if (STOP == 3) { out[b * 256 + tid] = pr[tid]; return; }
  {
    float4 pv[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pv[j] = *reinterpret_cast<const float4*>(pr + 4 * (l + 64 * j));
    for (int a0 = 8 * wv; a0 < A; a0 += 32) {
      float4 wr[8][3];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) wr[u][j] = *reinterpret_cast<const float4*>(wc + (long)min(a0 + u, A - 1) * D + 4 * (l + 64 * j));
      float sv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) s += pv[j].x * wr[u][j].x + pv[j].y * wr[u][j].y + pv[j].z * wr[u][j].z + pv[j].w * wr[u][j].w;
        sv[u] = s;
      }
      const float s = wave_sum_scatter<8>(sv);
      const int a = a0 + (l >> 3);
      if ((l & 7) == 0 && a < A) lg[a] = s + bc[a];
    }
  }
  __syncthreads();
  out[b * 256 + tid] = lg[tid % A];
}

int main() {
  const int B = 64, L = 32, D = 768, A = 170;
  std::vector<float> hx(B * L * D), hw(A * D), hwp(D);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = ((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = ((i * 40503u) % 1000) / 10000.f - 0.05f;
  for (int i = 0; i < D; ++i) hwp[i] = ((i * 7919) % 100) / 1000.f - 0.05f;
  std::vector<long long> ht(B);
  for (int b = 0; b < B; ++b) ht[b] = (b * 37) % A;
  float *x, *wp, *bp, *wc, *bc, *att, *pooled, *logp, *nll, *loss, *ws, *dx32, *dwp, *dbp, *dwc, *dbc;
  long long* tgt;
  CK(hipMalloc(&x, hx.size() * 4)); CK(hipMalloc(&wp, D * 4)); CK(hipMalloc(&bp, 4)); CK(hipMalloc(&wc, A * D * 4));
  CK(hipMalloc(&bc, A * 4)); CK(hipMalloc(&att, B * L * 4)); CK(hipMalloc(&pooled, B * D * 4));
  CK(hipMalloc(&logp, B * A * 4)); CK(hipMalloc(&nll, B * 4)); CK(hipMalloc(&loss, 4)); CK(hipMalloc(&tgt, B * 8));
  CK(hipMalloc(&ws, vqa_head_workspace_floats(B, L, D, A) * 4)); CK(hipMalloc(&dx32, hx.size() * 4));
  CK(hipMalloc(&dwp, D * 4)); CK(hipMalloc(&dbp, 4)); CK(hipMalloc(&dwc, A * D * 4)); CK(hipMalloc(&dbc, A * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wc, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wp, hwp.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bp, 0, 4)); CK(hipMemset(bc, 0, A * 4));
  CK(hipMemcpy(tgt, ht.data(), B * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    hipEventRecord(e0, 0);
    for (int i = 0; i < 50; ++i) fn();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us\n", name, ms * 1000 / 50);
  };
  timeit("vqa_head_fwd", [&] { vqa_head_fwd(x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A, 0); });
  timeit("head_fwd_kernel<32> only", [&] {
    hipLaunchKernelGGL(head_fwd_kernel<32>, dim3(B), dim3(256), 0, 0, x, wp, bp, wc, bc, tgt, att, pooled, logp, nll,
                       L, D, A);
  });
  timeit("vqa_head_bwd", [&] {
    vqa_head_bwd(x, att, pooled, logp, tgt, wp, wc, dx32, nullptr, dwp, dbp, dwc, dbc, ws, B, L, D, A, 0);
  });
  float* dl = ws + B * A;
  float* dsc = dl + B * A + B * D;
  timeit("head_bwd_sample<32> only", [&] {
    hipLaunchKernelGGL(head_bwd_sample_kernel<32>, dim3(B), dim3(256), 0, 0, x, att, logp, tgt, wc, wp, dl, dx32,
                       (bf16_t*)nullptr, dsc, L, D, A, 1.0f / B);
  });
  float* pout;
  CK(hipMalloc(&pout, B * 256 * 4));
#define PROBE(S) timeit("probe stop " #S, [&] { hipLaunchKernelGGL((head_probe<32, S>), dim3(B), dim3(256), 0, 0, x, wp, bp, wc, bc, pout, L, D, A); });
  PROBE(1) PROBE(2) PROBE(3) PROBE(4)
  timeit("empty launch (reduce 1 blk)", [&] { hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(256), 0, 0, nll, 1, 1.f, loss); });
  CK(hipDeviceSynchronize());
  return 0;
}
