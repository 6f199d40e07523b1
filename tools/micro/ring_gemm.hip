// Barrier-free producer/consumer GEMM ring vs the library's barrier ring (gemm_body.h).
//
// ring_kernel: NL loader waves move whole k-tiles of A [M][K] and B [N][K] (k-contiguous bf16)
// into an S-slot LDS ring by LDS-DMA and publish each slot with a FULL counter once their
// counted vmcnt shows it landed (D k-tiles in flight per loader wave); NWM x NWN consumer waves
// poll FULL, read the slot's fragments into registers, release the slot with a FREE counter
// (before their MFMAs) and accumulate with the library's swapped-operand 32x32x16 MFMA in the
// library's k order -- so the output is bitwise equal to gemm_kernel's.  No workgroup barrier in
// the k-loop; the epilogue is the library's tile_epilogue (the loader waves have exited).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include ring_gemm.hip ../../t5-resnet-vqa_amd/csrc/api.hip \
//     -o ring_gemm
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../t5-resnet-vqa_amd/csrc/gemm_body.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

namespace {

__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void lds_add(uint32_t a, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_wait_ge(uint32_t a, uint32_t target) {
  while (lds_ld(a) < target) __builtin_amdgcn_s_sleep(1);
}
template <int N>
__device__ __forceinline__ void vm_le(int n) {        // s_waitcnt vmcnt(<= n) for n in [0, N] (multiples not needed)
  if constexpr (N > 0) {
    if (n >= N) { wait_vm<N>(); return; }
    vm_le<N - 1>(n);
  } else {
    wait_vm<0>();
  }
}

template <int BM, int BN, int BKT, int S, int D, int NL, int NWM, int NWN>
__global__ __launch_bounds__(64 * (NWM * NWN + NL)) void ring_kernel(GemmParams P) {
  constexpr int NW = NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2, ST_BYTES = A_BYTES + B_BYTES;
  constexpr int KCPR = BKT / 8, RPI = 64 / KCPR;        // 16-B chunks per image row, rows per 1-KiB instruction
  constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024, NI = NIA + NIB;
  static_assert(NI % NL == 0, "k-tile instructions split evenly over the loader waves");
  constexpr int NIW = NI / NL;                          // instructions per loader wave per k-tile
  static_assert((D - 1) * NIW <= 63, "vmcnt is 6 bits");
  static_assert(S >= D + 1, "ring too short");
  __shared__ __attribute__((aligned(1024))) char smem[S * ST_BYTES + 256];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const uint32_t fullw = lds0 + S * ST_BYTES, freew = fullw + 64;

  const int nwg = P.tiles_m * P.tiles_n;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  if (tid < 32) reinterpret_cast<uint32_t*>(smem + S * ST_BYTES)[tid] = 0u;
  __syncthreads();
  const int nk = (P.k + BKT - 1) / BKT;

  if (w >= NW) {                                        // ---------------- loader waves
    // wave-uniform role index (readfirstlane: the LDS-DMA destination must be uniform, and a
    // per-lane operand select would make the compiler reload the parameter block per DMA)
    const int lw = __builtin_amdgcn_readfirstlane(w - NW);
    const bf16_t* __restrict__ pa = P.a;
    const bf16_t* __restrict__ pb = P.b;
    const long lda = P.lda, ldb = P.ldb;
    const int K = P.k;
    const bf16_t* base[NIW];
    int kof[NIW];
    bool ok[NIW];
    int dst[NIW];
#pragma unroll
    for (int jj = 0; jj < NIW; ++jj) {
      const int j = lw * NIW + jj;                      // instruction index within the k-tile (uniform)
      const bool isa = j < NIA;
      const int jr = isa ? j : j - NIA;
      const int row = jr * RPI + l / KCPR;
      const int ch = (l % KCPR) ^ kc_swz_t<BKT>(row);
      const int grow = (isa ? m0 : n0) + row;
      ok[jj] = grow < (isa ? P.m : P.n);
      kof[jj] = ch * 8;
      base[jj] = isa ? pa + (long)grow * lda + ch * 8 : pb + (long)grow * ldb + ch * 8;
      dst[jj] = (isa ? 0 : A_BYTES) + jr * 1024;
    }
    auto issue = [&](int t) {
      char* st = smem + (t % S) * ST_BYTES;
      const int k0 = t * BKT;
#pragma unroll
      for (int jj = 0; jj < NIW; ++jj) {
        const void* src = (ok[jj] && k0 + kof[jj] < K) ? (const void*)(base[jj] + k0) : (const void*)vqa_zero_page;
        glds16(src, st + dst[jj]);
      }
    };
    for (int t = 0; t < nk; ++t) {
      if (t >= S) lds_wait_ge(freew + 4 * (t % S), (uint32_t)(NW * (t / S)));
      issue(t);
      if (t >= D - 1) {
        wait_vm<(D - 1) * NIW>();                       // k-tile t-D+1 landed (this wave's part)
        if (l == 0) lds_add(fullw + 4 * ((t - D + 1) % S), 1u);
      }
    }
    for (int u = nk - D + 1 < 0 ? 0 : nk - D + 1; u < nk; ++u) {
      vm_le<(D - 1) * NIW>((nk - 1 - u) * NIW);
      if (l == 0) lds_add(fullw + 4 * (u % S), 1u);
    }
    return;                                             // s_barrier no longer counts this wave
  }
  // ---------------------------------------------------------------- consumer waves
  const int wm = w / NWN, wn = w % NWN;
  FragAddr<BM, true, TM, BKT> fra;
  FragAddr<BN, true, TN, BKT> frb;
  fra.init(wm * WM);
  frb.init(wn * WN);
  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  constexpr int KS = BKT / 16;
  for (int t = 0; t < nk; ++t) {
    const int s = t % S;
    lds_wait_ge(fullw + 4 * s, (uint32_t)(NL * (t / S + 1)));
    const uint32_t cur = lds0 + s * ST_BYTES;
    i32x4_t fa[KS][TM], fb[KS][TN];
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      fra.read(cur, q, fa[q]);
      frb.read(cur + A_BYTES, q, fb[q]);
    }
    wait_lgkm<0>();
    if (l == 0) lds_add(freew + 4 * s, 1u);            // the slot is free once its fragments are in VGPRs
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[q][j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[q][i]), acc[i][j], 0, 0, 0);
  }
  tile_epilogue<BM, BN, S, NWM, NWN, false, BKT>(P, acc, 0, m0, n0, P.m, smem);
}

}  // namespace

template <typename F>
float timeit(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

static GemmParams params(const bf16_t* a, const bf16_t* b, bf16_t* c, int m, int n, int k) {
  GemmParams P{};
  P.a = a; P.lda = k; P.b = b; P.ldb = k; P.m = m; P.n = n; P.k = k;
  P.c16 = c; P.ldc16 = n; P.alpha = 1.f; P.vec = (n % 8 == 0);
  return P;
}

template <int BM, int BN, int BKT, int S, int D, int NL, int NWM, int NWN>
void run_ring(const char* tag, const bf16_t* a, const bf16_t* b, bf16_t* c, const bf16_t* ref, int m, int n, int k,
              size_t bytes) {
  GemmParams P = params(a, b, c, m, n, k);
  P.tiles_m = (m + BM - 1) / BM;
  P.tiles_n = (n + BN - 1) / BN;
  const int grid = P.tiles_m * P.tiles_n;
  CK(hipMemset(c, 0, bytes));
  auto go = [&] {
    hipLaunchKernelGGL((ring_kernel<BM, BN, BKT, S, D, NL, NWM, NWN>), dim3(grid), dim3(64 * (NWM * NWN + NL)), 0, 0, P);
  };
  go();
  CK(hipDeviceSynchronize());
  std::vector<bf16_t> h(bytes / 2), r(bytes / 2);
  CK(hipMemcpy(h.data(), c, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), ref, bytes, hipMemcpyDeviceToHost));
  long bad = 0;
  for (size_t i = 0; i < h.size(); ++i) bad += h[i] != r[i];
  const float us = timeit(go, 50);
  printf("  %-40s grid %5d  %8.2f us  %7.1f TF/s  mismatches %ld\n", tag, grid, us, 2.0 * m * n * k / us * 1e-6, bad);
}

template <int BM, int BN, int ST, int NWM, int NWN, int BKT>
float run_lib(const char* tag, const bf16_t* a, const bf16_t* b, bf16_t* c, int m, int n, int k) {
  GemmParams P = params(a, b, c, m, n, k);
  auto go = [&] { launch<BM, BN, ST, NWM, NWN, true, true, false, false, BKT>(P, 1, 0); };
  go();
  CK(hipDeviceSynchronize());
  const float us = timeit(go, 50);
  printf("  %-40s grid %5d  %8.2f us  %7.1f TF/s\n", tag, P.tiles_m * P.tiles_n, us, 2.0 * m * n * k / us * 1e-6);
  return us;
}

int main() {
  const int shapes[][3] = {{2048, 768, 768}, {2048, 2304, 768}, {2048, 3072, 768}, {2048, 768, 3072}, {2048, 1536, 768}};
  for (auto& sh : shapes) {
    const int m = sh[0], n = sh[1], k = sh[2];
    std::vector<bf16_t> ha((size_t)m * k), hb((size_t)n * k);
    srand(1);
    for (auto& x : ha) x = (bf16_t)(0x3c00 + (rand() & 0x3ff) - 0x200 + ((rand() & 1) << 15));
    for (auto& x : hb) x = (bf16_t)(0x3c00 + (rand() & 0x3ff) - 0x200 + ((rand() & 1) << 15));
    bf16_t *a, *b, *c, *ref;
    const size_t cb = (size_t)m * n * 2;
    CK(hipMalloc(&a, ha.size() * 2));
    CK(hipMalloc(&b, hb.size() * 2));
    CK(hipMalloc(&c, cb));
    CK(hipMalloc(&ref, cb));
    CK(hipMemcpy(a, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    printf("M %d N %d K %d\n", m, n, k);
    run_lib<64, 64, 2, 2, 2, 128>("lib cfg21 64x64 k128 2st", a, b, ref, m, n, k);
    run_lib<64, 64, 2, 2, 2, 64>("lib cfg4 64x64 k64 2st", a, b, c, m, n, k);
    run_lib<128, 64, 2, 2, 2, 64>("lib cfg6 128x64 k64 2st", a, b, c, m, n, k);
    run_lib<64, 128, 2, 2, 2, 64>("lib cfg7 64x128 k64 2st", a, b, c, m, n, k);
    run_ring<64, 64, 128, 4, 2, 2, 2, 2>("ring 64x64 k128 S4 D2 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<64, 64, 128, 4, 3, 4, 2, 2>("ring 64x64 k128 S4 D3 NL4", a, b, c, ref, m, n, k, cb);
    run_ring<64, 64, 64, 6, 3, 1, 2, 2>("ring 64x64 k64 S6 D3 NL1", a, b, c, ref, m, n, k, cb);
    run_ring<64, 64, 64, 6, 4, 2, 2, 2>("ring 64x64 k64 S6 D4 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<64, 64, 64, 8, 5, 2, 2, 2>("ring 64x64 k64 S8 D5 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<128, 64, 64, 5, 3, 2, 2, 2>("ring 128x64 k64 S5 D3 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<64, 128, 64, 5, 3, 2, 2, 2>("ring 64x128 k64 S5 D3 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<128, 128, 64, 4, 2, 2, 2, 2>("ring 128x128 k64 S4 D2 NL2", a, b, c, ref, m, n, k, cb);
    run_ring<64, 64, 128, 3, 2, 2, 2, 2>("ring 64x64 k128 S3 D2 NL2", a, b, c, ref, m, n, k, cb);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(c));
    CK(hipFree(ref));
  }
  return 0;
}
