// Stand-alone timing of the answer-head kernels (includes head.hip directly):
// per-kernel HIP-event times at B=64, L=32, D=768, A=170, so a change to one
// kernel can be judged in isolation.   hipcc --offload-arch=gfx950 -O3 -I../../include
#include "../../t5-resnet-vqa_amd/csrc/head.hip"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

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
  timeit("empty launch (reduce 1 blk)", [&] { hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(256), 0, 0, nll, 1, 1.f, loss); });
  CK(hipDeviceSynchronize());
  return 0;
}
