// Where a 2048-row projection GEMM's time goes, phase by phase: every workgroup stamps the
// 100 MHz wall clock at entry, after its prologue DMAs are issued, when its first k-tile has
// landed, after the k-loop and after the epilogue (gemm.hip VQA_GEMM_STAMP hooks).  Prints,
// per shape x tile config: the event-timed launch, the span from the first entry to the
// last exit, the entry skew, and the median phase durations.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include gemm_stamps.hip ../../t5-resnet-vqa_amd/csrc/api.hip \
//     -o gemm_stamps
#include <hip/hip_runtime.h>
__device__ unsigned long long g_st[16384 * 8];
#define VQA_GEMM_STAMP(i)                                                                       \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.z == 0) g_st[blockIdx.x * 8 + (i)] = wall_clock64();      \
  } while (0)
#define VQA_GEMM_MICRO 1
#include "../../t5-resnet-vqa_amd/csrc/gemm.hip"
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// r05: `c16` runs the frozen ResNet's 1x1-convolution form instead: bf16 output, bias, ReLU and
// (res) a bf16 residual -- the epilogue of the bottleneck's expand / reduce GEMMs
template <int BM, int BN, int S, int NWM = 2, int NWN = 2, int BKT = 64>
void run(const char* tag, int M, int N, int K, bool res, int splitk = 0, bool c16 = false) {
  bf16_t *a, *b;
  float *c32, *r32;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c32, (size_t)M * N * 4));
  CK(hipMalloc(&r32, (size_t)M * N * 4));
  CK(hipMemset(a, 0x3c, (size_t)M * K * 2));
  CK(hipMemset(b, 0x3c, (size_t)N * K * 2));
  CK(hipMemset(r32, 0, (size_t)M * N * 4));
  vqa_gemm_desc d{};
  d.a = a; d.lda = K; d.b = b; d.ldb = K; d.m = M; d.n = N; d.k = K;
  d.alpha = 1.f; d.batch = 1;
  if (c16) {
    d.c16 = (bf16_t*)c32; d.ldc16 = N; d.bias = r32; d.relu = 1;      // (r32 zeroed: a zero bias)
    if (res) { d.res16 = (bf16_t*)r32 + (size_t)M * N; d.ldres = N; }
  } else {
    d.c32 = c32; d.ldc32 = N;
    if (res) { d.res32 = r32; d.ldres = N; }
  }
  void* ws = nullptr;
  if (splitk > 1) {
    int kper;
    const int S_ = effective_splitk(K, splitk, &kper);
    const long long need = 2 * splitk_bytes(64, 64, M, N, 1, S_) + splitk_bytes(BM, BN, M, N, 1, S_);
    CK(hipMalloc(&ws, need));
    CK(hipMemset(ws, 0, need));
    d.splitk = splitk; d.workspace = ws; d.workspace_bytes = need;
    d.config = 0;
  }
  GemmParams P;
  // prepare() sizes the split-K workspace by the config's tile; check it against this tile
  if (prepare(&d, P)) { printf("prepare failed: %s\n", vqa_last_error()); exit(1); }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ev;
  for (int r = 0; r < 25; ++r) {
    CK(hipEventRecord(e0, 0));
    GemmParams Q = P;
    launch<BM, BN, S, NWM, NWN, true, true, false, false, BKT>(Q, 1, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 5) ev.push_back(ms * 1e3f);
  }
  std::sort(ev.begin(), ev.end());
  const int nwg = vqa::cdiv(M, BM) * vqa::cdiv(N, BN) * (P.splitk > 1 ? P.splitk : 1);
  std::vector<unsigned long long> st((size_t)nwg * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_st), st.size() * 8));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const double us = 1e3 / rate_khz;                     // microseconds per tick
  unsigned long long t0 = ~0ull, t0max = 0, t4 = 0;
  std::vector<double> ph[4];
  for (int w = 0; w < nwg; ++w) {
    const unsigned long long* s = &st[(size_t)w * 8];
    t0 = std::min(t0, s[0]);
    t0max = std::max(t0max, s[0]);
    t4 = std::max(t4, s[4]);
    for (int p = 0; p < 4; ++p) ph[p].push_back((double)(s[p + 1] - s[p]) * us);
  }
  double busy = 0;                                      // sum of workgroup lifetimes
  for (int w = 0; w < nwg; ++w) busy += (double)(st[(size_t)w * 8 + 4] - st[(size_t)w * 8]) * us;
  for (auto& v : ph) std::sort(v.begin(), v.end());
  auto med = [](std::vector<double>& v) { return v[v.size() / 2]; };
  auto mx = [](std::vector<double>& v) { return v.back(); };
  printf("%-6s %4dx%4dx%4d %3dx%3d s%d bk%3d k%d wg %4d | event %6.2f us | span %6.2f  entry-skew %5.2f | "
         "init %5.2f  first-tile %5.2f  k-loop %6.2f (max %6.2f)  epilogue %5.2f (max %5.2f) | wg life %5.2f, "
         "resident per CU %4.2f\n",
         tag, M, N, K, BM, BN, S, BKT, P.splitk, nwg, ev[ev.size() / 2], (t4 - t0) * us, (t0max - t0) * us, med(ph[0]), med(ph[1]),
         med(ph[2]), mx(ph[2]), med(ph[3]), mx(ph[3]), busy / nwg, busy / ((t4 - t0) * us) / 256.0);
  CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c32)); CK(hipFree(r32));
  if (ws) CK(hipFree(ws));
}

// r05: the same tile body in a persistent grid -- G workgroups, workgroup w runs linear tile
// ids w, w + G, w + 2G, ... (G a multiple of 8 keeps every id on the XCD the remap assigns it);
// the question: is a launch of thousands of short-lived workgroups bound by the dispatcher?
// (launch bounds pin the library kernel's occupancy: unconstrained, the loop let the compiler
// hoist per-tile values into registers -- 121 VGPRs, 3 waves per SIMD instead of 66 and 5)
template <int BM, int BN, int S, int NWM, int NWN, int BKT>
__global__ __launch_bounds__(64 * NWM * NWN, (BM * BN <= 4096 && BKT == 64 ? 5 : 3)) void gemm_persist(GemmParams P, int nwg) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<BM, BN, S, BKT>::LDS];
  for (int bid = blockIdx.x; bid < nwg; bid += gridDim.x) {
    gemm_body<BM, BN, S, NWM, NWN, true, true, false, false, false, BKT>(P, bid, smem);
    __syncthreads();                                    // the ring / epilogue image is reused
  }
}

template <int BM, int BN, int S, int NWM = 2, int NWN = 2, int BKT = 64>
void persist(const char* tag, int M, int N, int K, bool res) {
  bf16_t *a, *b, *c, *c2, *r;
  float* bias;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  CK(hipMalloc(&c2, (size_t)M * N * 2));
  CK(hipMalloc(&r, (size_t)M * N * 2));
  CK(hipMalloc(&bias, (size_t)N * 4));
  CK(hipMemset(a, 0x3c, (size_t)M * K * 2));
  CK(hipMemset(b, 0x3b, (size_t)N * K * 2));
  CK(hipMemset(r, 0x3a, (size_t)M * N * 2));
  CK(hipMemset(bias, 0, (size_t)N * 4));
  vqa_gemm_desc d{};
  d.a = a; d.lda = K; d.b = b; d.ldb = K; d.m = M; d.n = N; d.k = K;
  d.alpha = 1.f; d.batch = 1; d.c16 = c; d.ldc16 = N; d.bias = bias; d.relu = 1;
  if (res) { d.res16 = r; d.ldres = N; }
  GemmParams P;
  if (prepare(&d, P)) { printf("prepare failed: %s\n", vqa_last_error()); exit(1); }
  P.tiles_m = vqa::cdiv(M, BM);
  P.tiles_n = vqa::cdiv(N, BN);
  const int nwg = P.tiles_m * P.tiles_n;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto f) {
    std::vector<float> v;
    for (int q = 0; q < 8; ++q) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) f();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (q) v.push_back(ms * 1e3f / 20);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const float t0 = timeit([&]() { GemmParams Q = P; launch<BM, BN, S, NWM, NWN, true, true, false, false, BKT>(Q, 1, 0); });
  std::vector<unsigned short> ref((size_t)M * N), out((size_t)M * N);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), c, ref.size() * 2, hipMemcpyDeviceToHost));
  printf("%-6s %6dx%5dx%5d %3dx%3d s%d bk%3d: grid %5d (one tile each) %7.2f us\n", tag, M, N, K, BM, BN, S, BKT, nwg, t0);
  for (int per : {2, 3, 4, 5, 6, 8}) {
    const int G = std::min(nwg, 256 * per) / 8 * 8;
    CK(hipMemset(c, 0xff, (size_t)M * N * 2));
    const float t = timeit([&]() {
      hipLaunchKernelGGL((gemm_persist<BM, BN, S, NWM, NWN, BKT>), dim3(G), dim3(64 * NWM * NWN), 0, 0, P, nwg);
    });
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), c, out.size() * 2, hipMemcpyDeviceToHost));
    const bool same = memcmp(out.data(), ref.data(), out.size() * 2) == 0;
    printf("%-6s   persistent grid %5d (%d per CU)                    %7.2f us  %s\n", tag, G, per, t, same ? "bitwise==lib" : "MISMATCH");
    if (G == nwg / 8 * 8) break;
  }
  fflush(stdout);
  CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c)); CK(hipFree(c2)); CK(hipFree(r)); CK(hipFree(bias));
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'p') {                  // r05: persistent grids on the ResNet's 1x1 shapes
    persist<64, 64, 2>("l3exp", 12544, 1024, 256, true);
    persist<64, 64, 2>("l3red", 12544, 256, 1024, false);
    persist<128, 64, 2>("l1exp", 200704, 256, 64, true);
    persist<64, 128, 2>("l1exp", 200704, 256, 64, true);
    persist<64, 64, 2>("l1exp", 200704, 256, 64, true);
    persist<128, 64, 2>("l1red", 200704, 64, 256, false);
    persist<64, 64, 2>("l2exp", 50176, 512, 128, true);
    persist<64, 64, 2>("l2red", 50176, 128, 512, false);
    persist<64, 64, 2>("l4exp", 3136, 2048, 512, true);
    persist<64, 64, 2, 2, 2, 128>("o", 2048, 768, 768, true);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'r') {                  // r05: the frozen ResNet's 1x1 convolutions (B = 64)
    run<64, 64, 2>("l3exp", 12544, 1024, 256, true, 0, true);
    run<64, 128, 2>("l3exp", 12544, 1024, 256, true, 0, true);
    run<128, 128, 2>("l3exp", 12544, 1024, 256, true, 0, true);
    run<128, 256, 2, 2, 4>("l3exp", 12544, 1024, 256, true, 0, true);
    run<64, 64, 2>("l3red", 12544, 256, 1024, false, 0, true);
    run<64, 64, 2, 2, 2, 128>("l3red", 12544, 256, 1024, false, 0, true);
    run<128, 64, 2>("l1exp", 200704, 256, 64, true, 0, true);
    run<64, 128, 2>("l1exp", 200704, 256, 64, true, 0, true);
    run<128, 128, 2>("l1exp", 200704, 256, 64, true, 0, true);
    run<128, 64, 2>("l1red", 200704, 64, 256, false, 0, true);
    run<64, 64, 2>("l2exp", 50176, 512, 128, true, 0, true);
    run<128, 128, 2>("l2exp", 50176, 512, 128, true, 0, true);
    return 0;
  }
  if (argc > 1) {                                       // r04: wave / stage variants on the 2048-row shape
    run<64, 64, 2, 2, 2, 128>("o", 2048, 768, 768, true);
    run<64, 64, 3, 2, 2, 128>("o", 2048, 768, 768, true);
    run<64, 64, 2, 1, 1, 128>("o", 2048, 768, 768, true);
    run<64, 64, 2, 2, 1, 128>("o", 2048, 768, 768, true);
    run<128, 64, 2, 4, 2>("o", 2048, 768, 768, true);
    run<64, 128, 2, 2, 4, 128>("o", 2048, 768, 768, true);
    run<64, 64, 2, 1, 1, 128>("qkv", 2048, 2304, 768, false);
    run<64, 128, 2, 2, 2, 128>("qkv", 2048, 2304, 768, false);
    run<64, 128, 2, 2, 4, 128>("qkv", 2048, 2304, 768, false);
    return 0;
  }
  run<64, 64, 2>("o", 2048, 768, 768, true);
  run<64, 64, 2, 2, 2, 128>("o", 2048, 768, 768, true);
  run<128, 64, 2, 2, 2, 128>("o", 2048, 768, 768, true);
  run<64, 128, 2>("qkv", 2048, 2304, 768, false);
  run<64, 128, 2, 2, 2, 128>("qkv", 2048, 2304, 768, false);
  run<64, 64, 2, 2, 2, 128>("qkv", 2048, 2304, 768, false);
  run<64, 128, 2>("wi", 2048, 3072, 768, false);
  run<64, 128, 2, 2, 2, 128>("wi", 2048, 3072, 768, false);
  run<64, 64, 4>("wo", 2048, 768, 3072, true);
  run<64, 64, 2, 2, 2, 128>("wo", 2048, 768, 3072, true);
  run<128, 64, 2, 2, 2, 128>("wo", 2048, 768, 3072, true);
  return 0;
}
