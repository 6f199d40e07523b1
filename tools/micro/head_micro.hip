// Stand-alone timing of the answer-head kernels (includes head.hip directly):
// per-kernel HIP-event times at B=64, L=32, D=768, A=170, so a change to one
// kernel can be judged in isolation.
//   hipcc --offload-arch=gfx950 -O3 -I../../include head_micro.hip -o head_micro \
//     -L../../t5-resnet-vqa_amd/lib -lvqa_hip -Wl,-rpath,'$ORIGIN/../../t5-resnet-vqa_amd/lib'
#include "../../t5-resnet-vqa_amd/csrc/head.hip"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
float timeit(F f, int reps = 50) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int B = 64, L = 32, D = 768, A = 170;
  std::vector<float> h((size_t)B * L * D);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  float *x, *wp, *bp, *wc, *bc, *att, *pooled, *logp, *nll, *loss, *dx, *dwp, *dbp, *dwc, *dbc, *ws;
  long long* tgt;
  CK(hipMalloc(&x, h.size() * 4));
  CK(hipMemcpy(x, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&wp, D * 4)); CK(hipMemcpy(wp, h.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bp, 4)); CK(hipMemset(bp, 0, 4));
  CK(hipMalloc(&wc, A * D * 4)); CK(hipMemcpy(wc, h.data() + 5, A * D * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bc, A * 4)); CK(hipMemset(bc, 0, A * 4));
  std::vector<long long> ht(B);
  for (int i = 0; i < B; ++i) ht[i] = (i * 37) % A;
  CK(hipMalloc(&tgt, B * 8)); CK(hipMemcpy(tgt, ht.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&att, B * L * 4)); CK(hipMalloc(&pooled, B * D * 4)); CK(hipMalloc(&logp, B * A * 4));
  CK(hipMalloc(&nll, B * 4)); CK(hipMalloc(&loss, 4)); CK(hipMalloc(&dx, (size_t)B * L * D * 4));
  CK(hipMalloc(&dwp, D * 4)); CK(hipMalloc(&dbp, 4)); CK(hipMalloc(&dwc, A * D * 4)); CK(hipMalloc(&dbc, A * 4));
  CK(hipMalloc(&ws, (size_t)vqa_head_workspace_floats(B, L, D, A) * 4));
  float* pbp = ws; float* dl = pbp + B; float* dpool = dl + B * A; float* part = dpool + B * D;
  hipStream_t s = 0;
  vqa_head_fwd(x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A, s);
  vqa_head_bwd(x, att, pooled, logp, tgt, wp, wc, dx, nullptr, dwp, dbp, dwc, dbc, ws, B, L, D, A, s);
  CK(hipDeviceSynchronize());
  printf("pool_fwd   %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_pool_fwd_kernel<32>, dim3(B), dim3(768), 0, s, x, wp, bp, att, pooled, L, D); }));
  printf("logits     %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_logits_kernel, dim3((A + 7) / 8, B / 16), dim3(256), 0, s, pooled, wc, bc, logp, B, D, A); }));
  printf("lse        %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_lse_kernel<4>, dim3(1), dim3(1024), 0, s, logp, tgt, nll, loss, B, A); }));
  vqa_head_fwd(x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A, s);
  printf("dpooled    %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_dpooled_kernel, dim3(D / 64, B / 16), dim3(256), 0, s, logp, tgt, wc, dl, dpool, B, D, A, 1.f / B); }));
  printf("pool_bwd   %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_pool_bwd_kernel<32>, dim3(B), dim3(768), 0, s, x, att, dpool, wp, dx, (bf16_t*)nullptr, part, pbp, L, D); }));
  printf("wgrad      %7.2f us\n", timeit([&] { hipLaunchKernelGGL(head_wgrad_kernel, dim3(11 * 3 + 3), dim3(256), 0, s, dl, pooled, part, pbp, dwc, dbc, dwp, dbp, B, A, D); }));
  printf("head_fwd   %7.2f us (API, 3 launches)\n", timeit([&] { vqa_head_fwd(x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A, s); }));
  printf("head_bwd   %7.2f us (API, 3 launches)\n", timeit([&] { vqa_head_bwd(x, att, pooled, logp, tgt, wp, wc, dx, nullptr, dwp, dbp, dwc, dbc, ws, B, L, D, A, s); }));
  CK(hipDeviceSynchronize());
  return 0;
}
