// Stand-alone timing of the attention kernels through the C ABI (links the built
// attention objects): T5 (B=64, 12 x 64, L=32, rel-bias + key mask) and SGA
// (8 x 96, Lk = 32 / 49) forward and backward, HIP events, 100 launches each.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../include/vqa_hip.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static void* dalloc(size_t bytes, float fill_scale = 0.f) {
  void* p;
  (void)hipMalloc(&p, bytes);
  std::vector<unsigned short> h(bytes / 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = fill_scale == 0.f ? 0 : (unsigned short)(0x3c00 + (i * 2654435761u >> 20) % 512);
  (void)hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice);
  return p;
}

int main() {
  const int B = 64, L = 32;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 5; ++i) fn();
    hipEventRecord(e0, 0);
    for (int i = 0; i < 100; ++i) fn();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-26s %8.2f us\n", name, ms * 1000 / 100);
  };
  for (int t5 = 1; t5 >= 0; --t5) {
    for (int lk : {32, 49}) {
      if (t5 && lk != 32) continue;
      const int H = t5 ? 12 : 8, DH = t5 ? 64 : 96, D = 768;
      void* qkv = dalloc((size_t)B * 64 * 3 * D * 2, 1.f);
      void* o = dalloc((size_t)B * L * D * 2);
      float* p = (float*)dalloc((size_t)B * H * L * 64 * 4);
      float* bias = (float*)dalloc((size_t)H * L * L * 4);
      long long* mask;
      CK(hipMalloc(&mask, B * L * 8));
      std::vector<long long> hm(B * L);
      for (int i = 0; i < B * L; ++i) hm[i] = (i % L) < 20 + (i / L) % 12;
      CK(hipMemcpy(mask, hm.data(), B * L * 8, hipMemcpyHostToDevice));
      void* dout = dalloc((size_t)B * L * D * 2, 1.f);
      void* dqkv = dalloc((size_t)B * 64 * 3 * D * 2);
      float* dsb = (float*)dalloc((size_t)B * H * L * L * 4);
      unsigned rng[4] = {1, 2, 1, 0};
      unsigned* drng;
      CK(hipMalloc(&drng, 16));
      CK(hipMemcpy(drng, rng, 16, hipMemcpyHostToDevice));
      vqa_attn_desc d;
      memset(&d, 0, sizeof(d));
      d.q = qkv; d.ldq = 3 * D;
      d.k = (char*)qkv + D * 2; d.ldk = 3 * D;
      d.v = (char*)qkv + 2 * D * 2; d.ldv = 3 * D;
      d.o = o; d.ldo = D; d.p = p;
      d.bias = t5 ? bias : nullptr; d.key_mask = t5 ? mask : nullptr;
      d.batch = B; d.heads = H; d.lq = L; d.lk = lk; d.dh = DH; d.scale = t5 ? 1.f : 0.1020621f;
      d.dout = dout; d.lddo = D;
      d.dq = dqkv; d.lddq = 3 * D; d.dk = (char*)dqkv + D * 2; d.lddk = 3 * D; d.dv = (char*)dqkv + 2 * D * 2;
      d.lddv = 3 * D; d.dbias = t5 ? dsb : nullptr;
      d.drop.p = 0.1f; d.drop.site = 3; d.drop.rng = drng;
      char nm[64];
      snprintf(nm, sizeof nm, "%s fwd lk=%d", t5 ? "T5 " : "SGA", lk);
      timeit(nm, [&] { vqa_attn_fwd(&d, 0); });
      snprintf(nm, sizeof nm, "%s bwd lk=%d", t5 ? "T5 " : "SGA", lk);
      timeit(nm, [&] { vqa_attn_bwd(&d, 0); });
      d.drop.p = 0.f;
      snprintf(nm, sizeof nm, "%s fwd lk=%d nodrop", t5 ? "T5 " : "SGA", lk);
      timeit(nm, [&] { vqa_attn_fwd(&d, 0); });
      CK(hipDeviceSynchronize());
    }
  }
  printf("last error: %s\n", vqa_last_error());
  return 0;
}
