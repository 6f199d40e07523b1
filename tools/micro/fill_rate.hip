// L2 -> LDS operand-fill rate of one workgroup, by staging mechanism (no MFMA):
// each workgroup streams T tiles of BYTES from an L2-resident 2 MiB buffer into a
// STAGES-deep LDS ring, waiting for the oldest tile each iteration (the GEMM k-loop's
// structure without its arithmetic), then reads one word per lane so nothing is dead.
//   glds  : global_load_lds_dwordx4 (LDS-DMA), counted vmcnt, s_barrier
//   reg   : global_load_dwordx4 into VGPRs one tile ahead, ds_write_b128 after the wait
// Grid = WG workgroups (1 or 2 per CU); prints GB/s per workgroup and per chip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 fill_rate.hip -o fill_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void_t;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// BYTES per tile, NW waves: each wave issues BYTES / (1024 * NW) LDS-DMA instructions per tile
template <int BYTES, int NW, int STAGES>
__global__ __launch_bounds__(64 * NW) void fill_glds(const char* __restrict__ src, long span, int tiles, float* out) {
  __shared__ __attribute__((aligned(1024))) char ring[STAGES * BYTES];
  constexpr int NI = BYTES / (1024 * NW);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long base = ((long)blockIdx.x * 7919 * BYTES) % span;
  auto issue = [&](int t) {
    char* st = ring + (t % STAGES) * BYTES;
    const long off = (base + (long)t * BYTES) % span;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const char* g = src + off + (long)((w * NI + j) * 1024 + l * 16);
      __builtin_amdgcn_global_load_lds(g, (lds_void_t*)(st + (w * NI + j) * 1024), 16, 0, 0);
    }
  };
  for (int s = 0; s < STAGES - 1; ++s) issue(s);
  float acc = 0.f;
  for (int t = 0; t < tiles; ++t) {
    if constexpr (STAGES >= 3) {
      if (t + 1 < tiles) wait_vm<(STAGES - 2) * NI>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    bar();
    if (t + STAGES - 1 < tiles) issue(t + STAGES - 1);
    acc += *reinterpret_cast<volatile float*>(ring + (t % STAGES) * BYTES + threadIdx.x * 4);
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

template <int BYTES, int NW>
__global__ __launch_bounds__(64 * NW) void fill_reg(const char* __restrict__ src, long span, int tiles, float* out) {
  __shared__ __attribute__((aligned(1024))) char ring[2 * BYTES];
  constexpr int NI = BYTES / (1024 * NW);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long base = ((long)blockIdx.x * 7919 * BYTES) % span;
  uint4 r[NI];
  auto load = [&](int t) {
    const long off = (base + (long)t * BYTES) % span;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      r[j] = *reinterpret_cast<const uint4*>(src + off + (long)((w * NI + j) * 1024 + l * 16));
  };
  auto store = [&](int t) {
    char* st = ring + (t & 1) * BYTES;
#pragma unroll
    for (int j = 0; j < NI; ++j) *reinterpret_cast<uint4*>(st + (w * NI + j) * 1024 + l * 16) = r[j];
  };
  load(0);
  float acc = 0.f;
  for (int t = 0; t < tiles; ++t) {
    store(t);                            // waits for tile t's registers
    if (t + 1 < tiles) load(t + 1);      // next tile in flight while this one is consumed
    __syncthreads();
    acc += *reinterpret_cast<volatile float*>(ring + (t & 1) * BYTES + threadIdx.x * 4);
    __syncthreads();
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

// no workgroup barrier: every wave streams its OWN slice of each tile into its own ring and
// waits only for its own LDS-DMA (vmcnt) -- what the per-slot barrier of the GEMM ring costs
template <int BYTES, int NW, int STAGES>
__global__ __launch_bounds__(64 * NW) void fill_glds_nobar(const char* __restrict__ src, long span, int tiles, float* out) {
  __shared__ __attribute__((aligned(1024))) char ring[STAGES * BYTES];
  constexpr int NI = BYTES / (1024 * NW);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long base = ((long)blockIdx.x * 7919 * BYTES) % span;
  auto issue = [&](int t) {
    char* st = ring + (t % STAGES) * BYTES;
    const long off = (base + (long)t * BYTES) % span;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const char* g = src + off + (long)((w * NI + j) * 1024 + l * 16);
      __builtin_amdgcn_global_load_lds(g, (lds_void_t*)(st + (w * NI + j) * 1024), 16, 0, 0);
    }
  };
  for (int s = 0; s < STAGES - 1; ++s) issue(s);
  float acc = 0.f;
  for (int t = 0; t < tiles; ++t) {
    if constexpr (STAGES >= 3) {
      if (t + 1 < tiles) wait_vm<(STAGES - 2) * NI>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    acc += *reinterpret_cast<volatile float*>(ring + (t % STAGES) * BYTES + (w * NI) * 1024 + l * 4);
    if (t + STAGES - 1 < tiles) issue(t + STAGES - 1);
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

// register loads with many in flight per lane (no LDS): NI 16-B loads per lane per tile, one
// tile ahead, summed so nothing is dead
template <int BYTES, int NW>
__global__ __launch_bounds__(64 * NW) void fill_reg_deep(const char* __restrict__ src, long span, int tiles, float* out) {
  constexpr int NI = BYTES / (1024 * NW);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long base = ((long)blockIdx.x * 7919 * BYTES) % span;
  float acc = 0.f;
  uint4 r[2][NI];
  auto load = [&](int t, uint4 (&d)[NI]) {
    const long off = (base + (long)t * BYTES) % span;
#pragma unroll
    for (int j = 0; j < NI; ++j) d[j] = *reinterpret_cast<const uint4*>(src + off + (long)((w * NI + j) * 1024 + l * 16));
  };
  load(0, r[0]);
  for (int t = 0; t < tiles; t += 2) {
    if (t + 1 < tiles) load(t + 1, r[1]);
#pragma unroll
    for (int j = 0; j < NI; ++j) acc += __uint_as_float(r[0][j].x);
    if (t + 2 < tiles) load(t + 2, r[0]);
#pragma unroll
    for (int j = 0; j < NI; ++j) acc += __uint_as_float(r[1][j].x);
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

template <typename K>
float timeit(K k, int grid, int block, const char* src, long span, int tiles, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, src, span, tiles, out);
  hipEventRecord(a, 0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, src, span, tiles, out);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const long span = 2 << 20;
  char* src;
  float* out;
  CK(hipMalloc(&src, span + (1 << 20)));
  CK(hipMemset(src, 1, span + (1 << 20)));
  CK(hipMalloc(&out, 4096 * 4));
  const int tiles = 400;
  auto rep = [&](const char* tag, float ms, int grid, int bytes) {
    const double tot = (double)grid * tiles * bytes;
    printf("%-34s grid %4d  %7.1f us  %6.1f GB/s per WG  %6.2f TB/s chip\n", tag, grid, ms * 1e3, tot / grid / (ms * 1e-3) / 1e9,
           tot / (ms * 1e-3) / 1e12);
  };
  for (int grid : {256, 512}) {
    rep("glds-nobar 16K 4 waves 2 stages", timeit(fill_glds_nobar<16384, 4, 2>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("glds-nobar 16K 4 waves 4 stages", timeit(fill_glds_nobar<16384, 4, 4>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("glds-nobar 32K 4 waves 4 stages", timeit(fill_glds_nobar<32768, 4, 4>, grid, 256, src, span, tiles, out), grid, 32768);
    rep("reg-deep 16K 4 waves (4/lane x2)", timeit(fill_reg_deep<16384, 4>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("reg-deep 32K 4 waves (8/lane x2)", timeit(fill_reg_deep<32768, 4>, grid, 256, src, span, tiles, out), grid, 32768);
    rep("reg-deep 32K 8 waves (4/lane x2)", timeit(fill_reg_deep<32768, 8>, grid, 512, src, span, tiles, out), grid, 32768);
  }
  for (int grid : {256, 384, 512}) {
    rep("glds 32K 4 waves 2 stages", timeit(fill_glds<32768, 4, 2>, grid, 256, src, span, tiles, out), grid, 32768);
    rep("glds 48K 4 waves 2 stages", timeit(fill_glds<49152, 4, 2>, grid, 256, src, span, tiles, out), grid, 49152);
    rep("glds 64K 8 waves 2 stages", timeit(fill_glds<65536, 8, 2>, grid, 512, src, span, tiles, out), grid, 65536);
    rep("glds 16K 4 waves 2 stages", timeit(fill_glds<16384, 4, 2>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("glds 16K 4 waves 3 stages", timeit(fill_glds<16384, 4, 3>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("glds 16K 4 waves 4 stages", timeit(fill_glds<16384, 4, 4>, grid, 256, src, span, tiles, out), grid, 16384);
    rep("glds 16K 8 waves 3 stages", timeit(fill_glds<16384, 8, 3>, grid, 512, src, span, tiles, out), grid, 16384);
    rep("glds 32K 4 waves 3 stages", timeit(fill_glds<32768, 4, 3>, grid, 256, src, span, tiles, out), grid, 32768);
    rep("glds 32K 8 waves 3 stages", timeit(fill_glds<32768, 8, 3>, grid, 512, src, span, tiles, out), grid, 32768);
  }
  return 0;
}
