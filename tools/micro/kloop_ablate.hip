// What paces the library's k-loop (gemm_body.h): the same loop -- LDS-DMA ring, counted vmcnt,
// s_barrier, ds_read fragments, 32x32x16 MFMAs -- with parts switched off (results wrong where
// a part is off; timing only), event-timed back-to-back on a 2048-row projection and a long-K
// shape.  The k-loop's marginal cost per k-tile is read from two K values.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include kloop_ablate.hip -o kloop_ablate
#include <hip/hip_runtime.h>
#include "../../t5-resnet-vqa_amd/csrc/gemm_common.h"
#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

enum { F_DMA = 1, F_BAR = 2, F_READ = 4, F_MFMA = 8, F_WAIT = 16, ALL = 31 };

template <int BM, int BN, int S, int NWM, int NWN, int BKT, int FL>
__global__ __launch_bounds__(64 * NWM * NWN) void kloop(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem[S * (BM + BN) * BKT * 2];
  constexpr int NW = NWM * NWN, WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int A_BYTES = BM * BKT * 2, ST_BYTES = (BM + BN) * BKT * 2;
  using LA = Loader<BM, true, false, NW, BKT>;
  using LB = Loader<BN, true, false, NW, BKT>;
  constexpr int NL = LA::NI + LB::NI;
  const int tiles_n = (N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, wm = w / NWN, wn = w % NWN;
  LA la;
  LB lb;
  vqa_conv_geom g{};
  la.init(m0, M, K, g);
  lb.init(n0, N, K, g);
  FragAddr<BM, true, TM, BKT> fra;
  FragAddr<BN, true, TN, BKT> frb;
  fra.init(wm * WM);
  frb.init(wn * WN);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = K / BKT;
#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    la.issue(A, K, smem + s * ST_BYTES, s * BKT, K, g);
    lb.issue(B, K, smem + s * ST_BYTES + A_BYTES, s * BKT, K, g);
  }
  for (int kt = 0; kt < nk; ++kt) {
    if (FL & F_WAIT) wait_tiles<NL, S>(min(nk - 1, kt + S - 2) - kt);
    if (FL & F_BAR) barrier();
    const int nt = kt + S - 1;
    if ((FL & F_DMA) && nt < nk) {
      char* st = smem + (nt % S) * ST_BYTES;
      la.issue(A, K, st, nt * BKT, K, g);
      lb.issue(B, K, st + A_BYTES, nt * BKT, K, g);
    }
    const uint32_t cur = lds0 + (kt % S) * ST_BYTES;
    i32x4_t fa[2][TM], fb[2][TN];
    if (FL & F_READ) {
      fra.read(cur, 0, fa[0]);
      frb.read(cur + A_BYTES, 0, fb[0]);
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[0][i] = fa[1][i] = i32x4_t{kt, 1, 2, 3};
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[0][j] = fb[1][j] = i32x4_t{kt, 3, 2, 1};
    }
    constexpr int R = FragAddr<BM, true, TM, BKT>::READS + FragAddr<BN, true, TN, BKT>::READS;
#pragma unroll
    for (int s = 0; s < BKT / 16; ++s) {
      if (FL & F_READ) {
        if (s + 1 < BKT / 16) {
          fra.read(cur, s + 1, fa[(s + 1) & 1]);
          frb.read(cur + A_BYTES, s + 1, fb[(s + 1) & 1]);
          wait_lgkm<R>();
        } else {
          wait_lgkm<0>();
        }
      }
      if (FL & F_MFMA) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[s & 1][j]),
                                                                __builtin_bit_cast(bf16x8_t, fa[s & 1][i]), acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][0][0] += __int_as_float(fa[s & 1][i][0] ^ fb[s & 1][0][1]);
      }
    }
  }
  wait_vm<0>();
  // minimal epilogue: one fp32 store per accumulator element (keeps every MFMA live)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * WM + i * 32 + (l & 31), col = n0 + wn * WN + j * 32 + 8 * (e >> 2) + 4 * (l >> 5) + (e & 3);
        if (row < M && col < N) C[(long)row * N + col] = acc[i][j][e];
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

bf16_t *gA, *gB;
float* gC;

template <int BM, int BN, int S, int NWM, int NWN, int BKT, int FL>
float run(int M, int N, int K) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return timeit([&]() {
    hipLaunchKernelGGL((kloop<BM, BN, S, NWM, NWN, BKT, FL>), dim3(grid), dim3(64 * NWM * NWN), 0, 0, gA, gB, gC, M, N, K);
  });
}

template <int BM, int BN, int S, int NWM, int NWN, int BKT>
void sweep(const char* tag, int M, int N, int K1, int K2) {
  const char* names[] = {"full", "no-dma", "no-barrier", "no-dsread", "no-mfma", "no-wait", "mfma-only", "dma+wait+bar"};
  float t[8][2];
  const int Ks[2] = {K1, K2};
  for (int q = 0; q < 2; ++q) {
    const int K = Ks[q];
    t[0][q] = run<BM, BN, S, NWM, NWN, BKT, ALL>(M, N, K);
    t[1][q] = run<BM, BN, S, NWM, NWN, BKT, ALL & ~F_DMA>(M, N, K);
    t[2][q] = run<BM, BN, S, NWM, NWN, BKT, ALL & ~F_BAR>(M, N, K);
    t[3][q] = run<BM, BN, S, NWM, NWN, BKT, ALL & ~F_READ>(M, N, K);
    t[4][q] = run<BM, BN, S, NWM, NWN, BKT, ALL & ~F_MFMA>(M, N, K);
    t[5][q] = run<BM, BN, S, NWM, NWN, BKT, ALL & ~F_WAIT>(M, N, K);
    t[6][q] = run<BM, BN, S, NWM, NWN, BKT, F_MFMA>(M, N, K);
    t[7][q] = run<BM, BN, S, NWM, NWN, BKT, F_DMA | F_WAIT | F_BAR>(M, N, K);
  }
  const int dk = (K2 - K1) / BKT;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  printf("%s M=%d N=%d tile %dx%d s%d %dx%d bk%d (%d tiles): us at K=%d / K=%d, marginal ns per k-tile\n", tag, M, N, BM, BN,
         S, NWM, NWN, BKT, tiles, K1, K2);
  for (int v = 0; v < 8; ++v)
    printf("   %-14s %8.2f %8.2f   %7.1f ns/k-tile\n", names[v], t[v][0], t[v][1], (t[v][1] - t[v][0]) * 1e3 / dk);
  fflush(stdout);
}

int main() {
  const size_t NA = 12544L * 4608, NB = 3072L * 4608;
  CK(hipMalloc(&gA, NA * 2));
  CK(hipMalloc(&gB, NB * 2));
  CK(hipMalloc(&gC, 12544L * 3072 * 4));
  CK(hipMemset(gA, 0x3c, NA * 2));
  CK(hipMemset(gB, 0x3c, NB * 2));
  sweep<64, 64, 2, 2, 2, 128>("o-proj", 2048, 768, 768, 3072);
  sweep<64, 64, 2, 2, 2, 64>("o-proj", 2048, 768, 768, 3072);
  sweep<128, 64, 2, 2, 2, 64>("qkv", 2048, 2304, 768, 3072);
  sweep<128, 128, 2, 2, 2, 64>("c3", 12544, 256, 1152, 4608);
  sweep<128, 128, 3, 2, 2, 64>("c3", 12544, 256, 1152, 4608);
  sweep<256, 256, 2, 2, 4, 64>("big", 12544, 2048, 512, 2048);
  return 0;
}
