// Wave-grid / ring-depth variants of the LDS-patch 3x3 convolution (csrc/conv_patch.inl) on the
// frozen ResNet-50's stride-1 3x3 geometries at B = 64: event-timed back-to-back launches and a
// bitwise check against the library's dispatch (every variant sums the same k-tiles in the same
// chunk-major order, so the outputs must be identical).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include conv_patch_micro.hip ../../t5-resnet-vqa_amd/csrc/api.hip \
//     -o conv_patch_micro
#include <hip/hip_runtime.h>
#define VQA_GEMM_MICRO 1
#include "../../t5-resnet-vqa_amd/csrc/gemm.hip"
#include "../../t5-resnet-vqa_amd/csrc/conv_patch.inl"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_rand(bf16_t* p, long n, unsigned seed) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = f2bf(((x & 0xffff) / 65536.f - 0.5f) * 0.25f);
  }
}

float timeit(const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < 8; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) v.push_back(ms * 1e3f / 20);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct Conv {
  int n, h, c, co;
  bf16_t *x, *w;
  bf16_t* out;
  float* b;
  std::vector<float> ref;
  GemmParams P;
  vqa_gemm_desc d;
};

Conv make(int n, int h, int c, int co) {
  Conv v{n, h, c, co};
  CK(hipMalloc(&v.x, (size_t)n * h * h * c * 2));
  CK(hipMalloc(&v.w, (size_t)co * 9 * c * 2));
  CK(hipMalloc(&v.out, (size_t)n * h * h * co * 2));
  CK(hipMalloc(&v.b, (size_t)co * 4));
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, v.x, (long)n * h * h * c, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, v.w, (long)co * 9 * c, 2u);
  CK(hipMemset(v.b, 0, co * 4));
  vqa_gemm_desc& d = v.d;
  d = vqa_gemm_desc{};
  d.a = v.x; d.b = v.w; d.m = n * h * h; d.n = co; d.k = 9 * c; d.lda = 9 * c; d.ldb = 9 * c;
  d.c16 = v.out; d.ldc16 = co; d.bias = v.b; d.alpha = 1.f; d.relu = 1; d.batch = 1;
  d.a_conv = 2;
  d.ga = vqa_conv_geom{n, h, h, c, h, h, 3, 3, 1, 1};
  if (prepare(&d, v.P)) { printf("prepare: %s\n", vqa_last_error()); exit(1); }
  CK(hipDeviceSynchronize());
  return v;
}

PatchGeom geom(const vqa_conv_geom& g, int bm) {
  PatchGeom G;
  G.R = bm / g.w < g.h ? bm / g.w : g.h;
  G.rbs = vqa::cdiv(g.h, G.R);
  G.npix = (G.R + 2) * (g.w + 2);
  G.pins = vqa::cdiv(G.npix, 8);
  G.chunks = g.c / 64;
  G.ppart = vqa::cdiv(G.pins, 10 - 3);
  return G;
}

std::vector<float> fetch(Conv& v) {
  std::vector<unsigned short> o((size_t)v.d.m * v.co);
  CK(hipMemcpy(o.data(), v.out, o.size() * 2, hipMemcpyDeviceToHost));
  std::vector<float> f(o.size());
  for (size_t i = 0; i < o.size(); ++i) f[i] = (float)o[i];
  return f;
}

void lib(const char* tag, Conv& v, int cfg) {
  vqa_gemm_desc d = v.d;
  d.config = cfg;
  GemmParams P = v.P;
  auto f = [&]() { GemmParams Q = P; conv_patch_dispatch(Q, cfg, 0); };
  f();
  CK(hipDeviceSynchronize());
  v.ref = fetch(v);
  const float us = timeit(f);
  const double tf = 2.0 * d.m * d.n * d.k / us * 1e-6;
  printf("%-4s %2dx%2dx%3d->%3d lib cfg %d                       %7.2f us %6.1f TF/s %.3f\n", tag, v.h, v.h, v.c, v.co,
         cfg, us, tf, tf / 2517.0);
  fflush(stdout);
}

template <int BM, int BN, int NWM, int NWN, int S>
void var(const char* tag, Conv& v) {
  const vqa_conv_geom& g = v.P.ga;
  const PatchGeom G = geom(g, BM);
  const bool db = G.chunks > 1;
  const int pmax = db ? PMAX_DB : PMAX_SB;
  if (G.npix > pmax) { printf("%-4s %3dx%3d %dx%d s%d: patch %d px > %d, skipped\n", tag, BM, BN, NWM, NWN, S, G.npix, pmax); return; }
  GemmParams P = v.P;
  P.tiles_m = g.n * G.rbs;
  P.tiles_n = vqa::cdiv(P.n, BN);
  CK(hipMemset(v.out, 0xff, (size_t)v.d.m * v.co * 2));
  auto f = [&]() {
    if (db)
      hipLaunchKernelGGL((conv_patch_kernel<BM, BN, NWM, NWN, PMAX_DB, true, S>), dim3(P.tiles_m * P.tiles_n),
                         dim3(64 * NWM * NWN), 0, 0, P, G);
    else
      hipLaunchKernelGGL((conv_patch_kernel<BM, BN, NWM, NWN, PMAX_SB, false, S>), dim3(P.tiles_m * P.tiles_n),
                         dim3(64 * NWM * NWN), 0, 0, P, G);
  };
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> o = fetch(v);
  long bad = 0;
  for (size_t i = 0; i < o.size(); ++i) bad += o[i] != v.ref[i];
  const float us = timeit(f);
  const double tf = 2.0 * v.d.m * v.d.n * v.d.k / us * 1e-6;
  printf("%-4s %2dx%2dx%3d->%3d var %3dx%3d %dx%d s%d tiles %5d %7.2f us %6.1f TF/s %.3f %s\n", tag, v.h, v.h, v.c, v.co,
         BM, BN, NWM, NWN, S, P.tiles_m * P.tiles_n, us, tf, tf / 2517.0, bad ? "MISMATCH" : "bitwise==lib");
  fflush(stdout);
}

int main() {
  {
    Conv v = make(64, 56, 64, 64);                   // layer1 conv2 (single chunk)
    lib("l1", v, 17);
    var<128, 64, 2, 2, 2>("l1", v);
    var<128, 64, 4, 2, 2>("l1", v);
    var<128, 64, 2, 2, 3>("l1", v);
    var<64, 64, 2, 2, 2>("l1", v);
  }
  {
    Conv v = make(64, 28, 128, 128);                 // layer2 conv2
    lib("l2", v, 17);
    lib("l2", v, 18);
    var<128, 64, 2, 2, 3>("l2", v);
    var<128, 64, 4, 2, 3>("l2", v);
    var<128, 64, 2, 2, 2>("l2", v);
    var<128, 64, 2, 2, 4>("l2", v);
    var<128, 128, 2, 4, 3>("l2", v);
    var<128, 128, 4, 2, 3>("l2", v);
    var<64, 128, 2, 4, 3>("l2", v);
  }
  {
    Conv v = make(64, 14, 256, 256);                 // layer3 conv2
    lib("l3", v, 17);
    var<128, 64, 2, 2, 3>("l3", v);
    var<128, 64, 4, 2, 3>("l3", v);
    var<128, 64, 2, 2, 4>("l3", v);
    var<128, 128, 2, 4, 3>("l3", v);
    var<128, 128, 4, 2, 3>("l3", v);
    var<64, 128, 2, 4, 3>("l3", v);
    var<64, 64, 2, 2, 3>("l3", v);
  }
  {
    Conv v = make(64, 7, 512, 512);                  // layer4 conv2
    lib("l4", v, 19);
    lib("l4", v, 20);
    var<64, 64, 2, 2, 3>("l4", v);
    var<64, 128, 2, 4, 3>("l4", v);
    var<64, 128, 2, 2, 3>("l4", v);
    var<64, 64, 2, 2, 4>("l4", v);
  }
  return 0;
}
