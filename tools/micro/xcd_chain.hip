// Persistent row-group GEMM chain vs one launch per GEMM (prototype for the T5 layer).
//
// The T5 forward's four weight GEMMs per layer (q|k|v 2048x2304x768, o 2048x768x768 + residual,
// wi 2048x3072x768 + ReLU, wo 2048x768x3072 + residual) for 12 layers, run
//   A  as 48 launches of the library tile kernel (the tuned configs), captured in one hipGraph;
//   B  as ONE launch of 256 workgroups in 8 row groups (group g = blockIdx % 8, i.e. one XCD
//      under round-robin placement -- speed only): group g owns rows [256 g, 256 g + 256) and
//      runs every phase on them, its 32 workgroups striding over the phase's tiles; a group
//      barrier (agent-scope counter, relaxed poll, one acquire) separates the phases.
// Both variants accumulate every output in the same K order, so the final activations must
// match bit for bit.  Prints the time per 12-layer chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include xcd_chain.hip ../../t5-resnet-vqa_amd/csrc/api.hip -o xcd_chain
#include <hip/hip_runtime.h>
#define VQA_GEMM_MICRO 1
#include "../../t5-resnet-vqa_amd/csrc/gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int T = 2048, D = 768, F = 3072, Q3 = 2304, NL = 12, G = 8, R = T / G;

struct Phase {
  GemmParams P;          // the group-0 problem (m = R rows); group g adds g*R rows to every row pointer
  int kind;              // 0 qkv, 1 o, 2 wi, 3 wo
  int tiles;
};

__device__ __forceinline__ void group_barrier(unsigned* cnt, unsigned target, unsigned* tmo, int release) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every wave: its stores have left
  __syncthreads();
  if (threadIdx.x == 0) {
    if (release) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();     // 100 MHz
    while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {          // 20 ms: give up, flag it
        __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int C> struct Cfg;
template <> struct Cfg<0> { static constexpr int BM = 64, BN = 64, S = 2, K = 64; };
template <> struct Cfg<1> { static constexpr int BM = 128, BN = 64, S = 2, K = 64; };
template <> struct Cfg<2> { static constexpr int BM = 64, BN = 128, S = 2, K = 64; };
template <> struct Cfg<3> { static constexpr int BM = 128, BN = 128, S = 2, K = 64; };
template <> struct Cfg<4> { static constexpr int BM = 64, BN = 64, S = 2, K = 128; };
template <> struct Cfg<5> { static constexpr int BM = 64, BN = 128, S = 2, K = 128; };
template <> struct Cfg<6> { static constexpr int BM = 128, BN = 64, S = 2, K = 128; };
template <> struct Cfg<7> { static constexpr int BM = 64, BN = 64, S = 3, K = 64; };

template <int C>
__device__ __forceinline__ void tile(const GemmParams& P, int t, char* smem) {
  using X = Cfg<C>;
  gemm_body<X::BM, X::BN, X::S, 2, 2, true, true, false, false, false, X::K>(P, t, smem);
}

// LDS: 96 KB = one workgroup per CU (WPG 32 per group); 32 KB = up to four per CU (WPG 128)
template <int C0, int C1, int C2, int C3, int LDS_MAX = 98304, int WPG = 32>
__global__ __launch_bounds__(256) void chain_kernel(const Phase* __restrict__ ph, int nph, unsigned* sync, int release) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_MAX];
  const int g = blockIdx.x % G, r = blockIdx.x / G;
  for (int p = 0; p < nph; ++p) {
    Phase x = ph[p];
    GemmParams P = x.P;
    const long ro = (long)g * R;
    P.a += ro * P.lda;
    if (P.c32) P.c32 += ro * P.ldc32;
    if (P.c16) P.c16 += ro * P.ldc16;
    if (P.res32) P.res32 += ro * P.ldres;
    if (P.res16) P.res16 += ro * P.ldres;
    for (int t = r; t < x.tiles; t += WPG) {
      switch (x.kind) {
        case 0: tile<C0>(P, t, smem); break;
        case 1: tile<C1>(P, t, smem); break;
        case 2: tile<C2>(P, t, smem); break;
        default: tile<C3>(P, t, smem); break;
      }
      __syncthreads();                                   // the ring / epilogue image is reused by the next tile
    }
    group_barrier(sync + 16 * g, (unsigned)(p + 1) * WPG, sync + 16 * G, release);
  }
}

static void tiles_of(int c, int& bm, int& bn) {
  static const int t[8][2] = {{64, 64}, {128, 64}, {64, 128}, {128, 128}, {64, 64}, {64, 128}, {128, 64}, {64, 64}};
  bm = t[c][0];
  bn = t[c][1];
}

struct Bufs {
  bf16_t *x[2], *qkv, *h16, *hid;
  bf16_t *wq[NL], *wo[NL], *wi[NL], *wo2[NL];
};

static vqa_gemm_desc desc(const bf16_t* a, int lda, const bf16_t* b, int m, int n, int k, bf16_t* c16, const bf16_t* res16,
                          int relu) {
  vqa_gemm_desc d{};
  d.a = a; d.lda = lda; d.b = b; d.ldb = k; d.m = m; d.n = n; d.k = k;
  d.c16 = c16; d.ldc16 = n; d.alpha = 1.f; d.batch = 1; d.relu = relu;
  if (res16) { d.res16 = res16; d.ldres = n; }
  return d;
}

// the four GEMMs of layer l as descriptors over `m` rows starting at the given row pointers
static void layer_descs(const Bufs& b, int l, int m, vqa_gemm_desc (&d)[4]) {
  const bf16_t* x = b.x[l & 1];
  d[0] = desc(x, D, b.wq[l], m, Q3, D, b.qkv, nullptr, 0);
  d[1] = desc(b.qkv, Q3, b.wo[l], m, D, D, b.h16, x, 0);        // reads q (the first 768 columns) as the context
  d[2] = desc(b.h16, D, b.wi[l], m, F, D, b.hid, nullptr, 1);
  d[3] = desc(b.hid, F, b.wo2[l], m, D, F, b.x[(l + 1) & 1], b.h16, 0);
}

template <int C>
static void launch_cfg(GemmParams P, hipStream_t s) {
  using X = Cfg<C>;
  launch<X::BM, X::BN, X::S, 2, 2, true, true, false, false, X::K>(P, 1, s);
}

static void launch_kind(int c, GemmParams P, hipStream_t s) {
  switch (c) {
    case 0: launch_cfg<0>(P, s); break;
    case 1: launch_cfg<1>(P, s); break;
    case 2: launch_cfg<2>(P, s); break;
    case 3: launch_cfg<3>(P, s); break;
    case 4: launch_cfg<4>(P, s); break;
    case 5: launch_cfg<5>(P, s); break;
    case 6: launch_cfg<6>(P, s); break;
    default: launch_cfg<7>(P, s); break;
  }
}

static float time_graph(hipGraphExec_t ge, hipStream_t s, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

static std::vector<unsigned short> fetch(const bf16_t* p, size_t n) {
  std::vector<unsigned short> h(n);
  CK(hipMemcpy(h.data(), p, n * 2, hipMemcpyDeviceToHost));
  return h;
}

int main(int argc, char** argv) {
  Bufs b;
  auto alloc = [](bf16_t** p, size_t n, unsigned seed) {
    CK(hipMalloc(p, n * 2));
    std::vector<unsigned short> h(n);
    unsigned s = seed * 2654435761u + 1;
    for (size_t i = 0; i < n; ++i) {
      s = s * 1664525u + 1013904223u;
      const float v = ((float)((s >> 9) & 0xffff) / 65536.f - 0.5f) * 0.08f;
      unsigned u;
      memcpy(&u, &v, 4);
      h[i] = (unsigned short)(u >> 16);
    }
    CK(hipMemcpy(*p, h.data(), n * 2, hipMemcpyHostToDevice));
  };
  alloc(&b.x[0], (size_t)T * D, 1);
  alloc(&b.x[1], (size_t)T * D, 2);
  alloc(&b.qkv, (size_t)T * Q3, 3);
  alloc(&b.h16, (size_t)T * D, 4);
  alloc(&b.hid, (size_t)T * F, 5);
  for (int l = 0; l < NL; ++l) {
    alloc(&b.wq[l], (size_t)Q3 * D, 10 + l);
    alloc(&b.wo[l], (size_t)D * D, 30 + l);
    alloc(&b.wi[l], (size_t)F * D, 50 + l);
    alloc(&b.wo2[l], (size_t)D * F, 70 + l);
  }
  std::vector<unsigned short> x0 = fetch(b.x[0], (size_t)T * D);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int reps = 20;

  // ---- A: one launch per GEMM (library configs of the tuned table), one graph
  const int ca[4] = {1, 4, 1, 7};                        // qkv 128x64, o 64x64/128-deep, wi 128x64, wo 64x64x3
  hipGraph_t ga;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int l = 0; l < NL; ++l) {
    vqa_gemm_desc d[4];
    layer_descs(b, l, T, d);
    for (int k = 0; k < 4; ++k) {
      GemmParams P;
      if (prepare(&d[k], P)) { printf("prepare: %s\n", vqa_last_error()); return 1; }
      launch_kind(ca[k], P, s);
    }
  }
  CK(hipStreamEndCapture(s, &ga));
  hipGraphExec_t gea;
  CK(hipGraphInstantiate(&gea, ga, nullptr, nullptr, 0));
  CK(hipMemcpy(b.x[0], x0.data(), x0.size() * 2, hipMemcpyHostToDevice));
  CK(hipGraphLaunch(gea, s));
  CK(hipStreamSynchronize(s));
  std::vector<unsigned short> ra = fetch(b.x[0], (size_t)T * D);
  const float ta = time_graph(gea, s, reps);
  printf("A  48 launches in one graph: %8.1f us per 12-layer chain (%5.1f us per layer)\n", ta, ta / NL);

  // ---- B: persistent row groups
  unsigned* sync;
  const size_t sync_bytes = 16 * (G + 1) * 4;
  CK(hipMalloc(&sync, sync_bytes));
  Phase* dph;
  CK(hipMalloc(&dph, sizeof(Phase) * 4 * NL));
  auto run_b = [&](const char* tag, auto kern, const int (&cb)[4], int release, int WPG = 32) {
    std::vector<Phase> ph(4 * NL);
    for (int l = 0; l < NL; ++l) {
      vqa_gemm_desc d[4];
      layer_descs(b, l, R, d);
      for (int k = 0; k < 4; ++k) {
        Phase& x = ph[4 * l + k];
        if (prepare(&d[k], x.P)) { printf("prepare: %s\n", vqa_last_error()); exit(1); }
        int bm, bn;
        tiles_of(cb[k], bm, bn);
        x.P.tiles_m = vqa::cdiv(R, bm);
        x.P.tiles_n = vqa::cdiv(d[k].n, bn);
        x.tiles = x.P.tiles_m * x.P.tiles_n;
        x.kind = k;
      }
    }
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
    if (per_cu * 256 < G * WPG) {                        // a grid barrier needs every block resident
      printf("B  %-34s skipped: %d blocks per CU resident < %d needed\n", tag, per_cu, G * WPG / 256);
      return;
    }
    CK(hipMemcpy(dph, ph.data(), sizeof(Phase) * ph.size(), hipMemcpyHostToDevice));
    hipGraph_t gb;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(sync, 0, sync_bytes, s));
    hipLaunchKernelGGL(kern, dim3(G * WPG), dim3(256), 0, s, dph, 4 * NL, sync, release);
    CK(hipStreamEndCapture(s, &gb));
    hipGraphExec_t geb;
    CK(hipGraphInstantiate(&geb, gb, nullptr, nullptr, 0));
    CK(hipMemcpy(b.x[0], x0.data(), x0.size() * 2, hipMemcpyHostToDevice));
    CK(hipGraphLaunch(geb, s));
    CK(hipStreamSynchronize(s));
    unsigned tmo = 0;
    CK(hipMemcpy(&tmo, sync + 16 * G, 4, hipMemcpyDeviceToHost));
    std::vector<unsigned short> rb = fetch(b.x[0], (size_t)T * D);
    size_t diff = 0;
    for (size_t i = 0; i < rb.size(); ++i) diff += rb[i] != ra[i];
    const float tb = time_graph(geb, s, reps);
    printf("B  %-34s release %d: %8.1f us per chain (%5.1f us per layer)  timeout %u  differing %zu of %zu\n", tag, release, tb,
           tb / NL, tmo, diff, rb.size());
    CK(hipGraphExecDestroy(geb));
    CK(hipGraphDestroy(gb));
  };
  {
    const int c[4] = {1, 0, 3, 0};
    run_b("qkv 128x64 o 64x64 wi 128x128 wo 64x64", chain_kernel<1, 0, 3, 0>, c, 1);
    run_b("qkv 128x64 o 64x64 wi 128x128 wo 64x64", chain_kernel<1, 0, 3, 0>, c, 0);
  }
  {
    const int c[4] = {0, 0, 0, 0};
    run_b("all 64x64, 3 per CU", chain_kernel<0, 0, 0, 0, 32768, 96>, c, 1, 96);
    run_b("all 64x64, 3 per CU", chain_kernel<0, 0, 0, 0, 32768, 96>, c, 0, 96);
    const int c2[4] = {1, 0, 1, 7};
    run_b("qkv/wi 128x64 o 64x64 wo 64x64x3, 2 per CU", chain_kernel<1, 0, 1, 7, 49152, 64>, c2, 1, 64);
  }
  {
    const int c[4] = {5, 4, 5, 4};
    run_b("qkv 64x128/128 o 64x64/128 wi 64x128/128 wo 64x64/128", chain_kernel<5, 4, 5, 4>, c, 1);
  }
  {
    const int c[4] = {3, 2, 3, 2};
    run_b("qkv 128x128 o 64x128 wi 128x128 wo 64x128", chain_kernel<3, 2, 3, 2>, c, 1);
  }
  return 0;
}
