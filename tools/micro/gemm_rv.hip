// Register-direct GEMM tiles (csrc/gemm_rv.h) against the library's barrier-ring tiles
// (gemm_body.h) on the step's GEMM shapes: event-timed back-to-back launches (the way
// bench.py's time_kernel and the step's graph run them) and a bitwise check of the output
// against the library kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include gemm_rv.hip ../../t5-resnet-vqa_amd/csrc/api.hip \
//     -o gemm_rv
#include <hip/hip_runtime.h>
#define VQA_GEMM_MICRO 1
#include "../../t5-resnet-vqa_amd/csrc/gemm.hip"
#include "gemm_rv.h"
#include "gemm_vs.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Prob {
  int M, N, K;
  bool bt;              // B m/n-contig ([K][N]: the dX form)
  bool res;
  bf16_t *a, *b;
  float *c32, *r32, *ref;
};

__global__ void fill_rand(bf16_t* p, long n, unsigned seed) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffff) / 65536.f - 0.5f) * 0.25f;
    p[i] = f2bf(f);
  }
}

Prob make(int M, int N, int K, bool bt, bool res) {
  Prob p{M, N, K, bt, res};
  CK(hipMalloc(&p.a, (size_t)M * K * 2));
  CK(hipMalloc(&p.b, (size_t)N * K * 2));
  CK(hipMalloc(&p.c32, (size_t)M * N * 4));
  CK(hipMalloc(&p.r32, (size_t)M * N * 4));
  CK(hipMalloc(&p.ref, (size_t)M * N * 4));
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, p.a, (long)M * K, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, p.b, (long)N * K, 2u);
  CK(hipMemset(p.r32, 0, (size_t)M * N * 4));
  CK(hipDeviceSynchronize());
  return p;
}

GemmParams params(const Prob& p) {
  vqa_gemm_desc d{};
  d.a = p.a; d.lda = p.K; d.b = p.b; d.ldb = p.bt ? p.N : p.K; d.m = p.M; d.n = p.N; d.k = p.K;
  d.b_trans = p.bt;
  d.c32 = p.c32; d.ldc32 = p.N; d.alpha = 1.f; d.batch = 1;
  if (p.res) { d.res32 = p.r32; d.ldres = p.N; }
  GemmParams P;
  if (prepare(&d, P)) { printf("prepare failed: %s\n", vqa_last_error()); exit(1); }
  return P;
}

// median over 7 samples of (20 back-to-back launches between two events) / 20
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

template <int BM, int BN, int S, int NWM, int NWN, int BKT = 64>
void lib(const char* tag, Prob& p) {
  GemmParams P = params(p);
  auto f = [&]() {
    GemmParams Q = P;
    if (p.bt) launch<BM, BN, S, NWM, NWN, true, false, false, false, BKT>(Q, 1, 0);
    else launch<BM, BN, S, NWM, NWN, true, true, false, false, BKT>(Q, 1, 0);
  };
  const float us = timeit(f);
  f();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(p.ref, p.c32, (size_t)p.M * p.N * 4, hipMemcpyDeviceToDevice));
  const double tf = 2.0 * p.M * p.N * p.K / us * 1e-6;
  printf("%-6s %5dx%5dx%5d %s lib %3dx%3d s%d %dx%d bk%3d            %8.2f us %7.1f TF/s %.3f\n", tag, p.M, p.N, p.K,
         p.bt ? "NT" : "NN", BM, BN, S, NWM, NWN, BKT, us, tf, tf / 2517.0);
  fflush(stdout);
}

template <int BM, int BN, int NWM, int NWN, bool DB, int BKT, int PD>
void rv(const char* tag, Prob& p) {
  GemmParams P = params(p);
  constexpr bool LKC = DB ? true : false;       // DB: A k-contig in LDS; !DB: B n-contig in LDS
  if (DB && p.bt) return;
  CK(hipMemset(p.c32, 0xff, (size_t)p.M * p.N * 4));
  auto f = [&]() {
    GemmParams Q = P;
    launch_rv<BM, BN, NWM, NWN, DB, LKC, BKT, PD>(Q, 1, 0);
  };
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> x((size_t)p.M * p.N), y((size_t)p.M * p.N);
  CK(hipMemcpy(x.data(), p.c32, x.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), p.ref, y.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (size_t i = 0; i < x.size(); ++i) bad += memcmp(&x[i], &y[i], 4) != 0;
  const float us = timeit(f);
  const double tf = 2.0 * p.M * p.N * p.K / us * 1e-6;
  printf("%-6s %5dx%5dx%5d %s rv  %3dx%3d %dx%d %s bk%3d pd%d %8.2f us %7.1f TF/s %.3f %s\n", tag, p.M, p.N, p.K,
         p.bt ? "NT" : "NN", BM, BN, NWM, NWN, DB ? "B-direct" : "A-direct", BKT, PD, us, tf, tf / 2517.0,
         bad ? "MISMATCH" : "bitwise==lib");
  if (bad) printf("   %ld of %zu elements differ (x[0]=%g ref=%g)\n", bad, x.size(), x[0], y[0]);
  fflush(stdout);
}

template <int BM, int BN, int NWM, int NWN, int BKT>
void vs(const char* tag, Prob& p) {
  GemmParams P = params(p);
  CK(hipMemset(p.c32, 0xff, (size_t)p.M * p.N * 4));
  auto f = [&]() {
    GemmParams Q = P;
    if (p.bt) launch_vs<BM, BN, NWM, NWN, true, false, BKT>(Q, 1, 0);
    else launch_vs<BM, BN, NWM, NWN, true, true, BKT>(Q, 1, 0);
  };
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> x((size_t)p.M * p.N), y((size_t)p.M * p.N);
  CK(hipMemcpy(x.data(), p.c32, x.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), p.ref, y.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (size_t i = 0; i < x.size(); ++i) bad += memcmp(&x[i], &y[i], 4) != 0;
  const float us = timeit(f);
  const double tf = 2.0 * p.M * p.N * p.K / us * 1e-6;
  printf("%-6s %5dx%5dx%5d %s vs  %3dx%3d %dx%d vgpr-staged bk%3d %8.2f us %7.1f TF/s %.3f %s\n", tag, p.M, p.N, p.K,
         p.bt ? "NT" : "NN", BM, BN, NWM, NWN, BKT, us, tf, tf / 2517.0, bad ? "MISMATCH" : "bitwise==lib");
  if (bad) printf("   %ld of %zu elements differ (x[0]=%g ref=%g)\n", bad, x.size(), x[0], y[0]);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  if (which == 0 || which == 1) {                 // SGA / T5 o-projection, forward
    Prob p = make(2048, 768, 768, false, true);
    lib<64, 64, 2, 2, 2, 128>("o", p);
    lib<64, 64, 2, 2, 2>("o", p);
    vs<64, 64, 2, 2, 64>("o", p);
    vs<64, 64, 2, 2, 128>("o", p);
    vs<128, 64, 2, 2, 64>("o", p);
    vs<64, 128, 2, 2, 64>("o", p);
    vs<128, 128, 2, 2, 64>("o", p);
  }
  if (which == 0 || which == 2) {                 // T5 q|k|v
    Prob p = make(2048, 2304, 768, false, false);
    lib<128, 64, 2, 2, 2>("qkv", p);
    vs<128, 64, 2, 2, 64>("qkv", p);
    vs<128, 64, 2, 2, 128>("qkv", p);
    vs<64, 128, 2, 2, 64>("qkv", p);
    vs<128, 128, 2, 2, 64>("qkv", p);
  }
  if (which == 0 || which == 3) {                 // T5 wo (K = 3072)
    Prob p = make(2048, 768, 3072, false, true);
    lib<64, 64, 3, 2, 2>("wo", p);
    vs<64, 64, 2, 2, 64>("wo", p);
    vs<64, 64, 2, 2, 128>("wo", p);
    vs<128, 64, 2, 2, 64>("wo", p);
    vs<128, 128, 2, 2, 64>("wo", p);
  }
  if (which == 0 || which == 4) {                 // input gradient dX = dY W (B n-contig)
    Prob p = make(2048, 768, 768, true, false);
    lib<64, 64, 2, 2, 2, 128>("dx", p);
    vs<64, 64, 2, 2, 64>("dx", p);
    vs<64, 64, 2, 2, 128>("dx", p);
    vs<128, 64, 2, 2, 64>("dx", p);
  }
  if (which == 0 || which == 5) {                 // conv-like long K (plain operands as a proxy)
    Prob p = make(12544, 256, 2304, false, false);
    lib<64, 128, 2, 2, 2>("c3", p);
    lib<128, 128, 2, 2, 2>("c3", p);
    vs<64, 128, 2, 2, 64>("c3", p);
    vs<128, 128, 2, 2, 64>("c3", p);
    vs<128, 256, 2, 4, 64>("c3", p);
    vs<256, 128, 4, 2, 64>("c3", p);
  }
  return 0;
}
