// GEMM tile body with VGPR-staged operand loads (r05 micro, tools/micro/gemm_rv.hip): each
// thread loads its 16-B pieces of the next k-tiles with global_load_dwordx4 into registers two
// k-tiles ahead and writes them to the LDS image with ds_write_b128 (the pieces, swizzles and
// zero-page padding of gemm_common.h's Loader, which moves the same pieces by LDS-DMA), one
// barrier per k-tile.  The question it answers: is the LDS-DMA issue cost inside the compute
// waves what paces the library's k-loop (MI355X_MICROARCH.md: 60-185 cycles per 1-KiB piece)?
#pragma once
#include "../../t5-resnet-vqa_amd/csrc/gemm_common.h"
#include "gemm_rv.h"            // gload16

namespace {

__device__ __forceinline__ void ds_w128(uint32_t addr, i32x4_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// the source address of every 16-B piece this thread moves for one operand k-tile (plain
// operands: Loader's non-gather paths), its LDS byte offset inside the stage
template <int ROWS, bool KC, int NW, int BKT>
struct VsLoader : Loader<ROWS, KC, false, NW, BKT> {
  using Base = Loader<ROWS, KC, false, NW, BKT>;
  using Base::NI;
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int k0, int K, i32x4_t (&r)[NI]) const {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const void* src = vqa_zero_page;
      const int kk = k0 + this->kof[j];
      if (this->ok[j] && kk < K) src = KC ? (const void*)(base + this->off[j] + k0) : (const void*)(base + (long)kk * ld + this->off[j]);
      // a plain (compiler-visible) load: the waitcnt pass then orders every use of r[j] after its
      // data has landed (r05: with the loads as inline asm the register allocator moved the
      // not-yet-landed destination registers through loop-carried copies and reused them for
      // addresses -- a memory-aperture fault)
      r[j] = *reinterpret_cast<const i32x4_t*>(src);
    }
  }
  __device__ __forceinline__ void store(uint32_t stage, const i32x4_t (&r)[NI]) const {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) ds_w128(stage + (w * NI + j) * 1024 + l * 16, r[j]);
  }
};

template <int BM, int BN, int NWM, int NWN, bool AKC, bool BKC, int BKT>
struct VsCfg {
  static constexpr int ST = (BM + BN) * BKT * 2;
  static constexpr int LDS = 2 * ST;
};

template <int BM, int BN, int NWM, int NWN, bool AKC, bool BKC, int BKT>
__device__ __forceinline__ void gemm_body_vs(const GemmParams& P, const int bid, char* smem) {
  constexpr int NW = NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int A_BYTES = BM * BKT * 2, ST = VsCfg<BM, BN, NWM, NWN, AKC, BKC, BKT>::ST;
  using LA = VsLoader<BM, AKC, NW, BKT>;
  using LB = VsLoader<BN, BKC, NW, BKT>;
  constexpr int NA = LA::NI, NB = LB::NI, NL = NA + NB;
  const int ntile = P.tiles_m * P.tiles_n;
  const int xcd = bid & 7, q8 = ntile >> 3, r8 = ntile & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;
  const bf16_t* A = P.a + (long)z * P.sa;
  const bf16_t* B = P.b + (long)z * P.sb;
  const int tid = threadIdx.x, w = tid >> 6;
  const int wm = w / NWN, wn = w % NWN;
  LA la;
  LB lb;
  la.init(m0, P.m, P.lda, P.ga);
  lb.init(n0, P.n, P.ldb, P.gb);
  FragAddr<BM, AKC, TM, BKT> fra;
  FragAddr<BN, BKC, TN, BKT> frb;
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
  const int K = P.k, nk = (K + BKT - 1) / BKT;
  i32x4_t ra[2][NA], rb[2][NB];
  auto load = [&](int t, i32x4_t (&xa)[NA], i32x4_t (&xb)[NB]) {
    la.load(A, P.lda, t * BKT, K, xa);
    lb.load(B, P.ldb, t * BKT, K, xb);
  };
  auto compute = [&](uint32_t cur) {
    constexpr int R = FragAddr<BM, AKC, TM, BKT>::READS + FragAddr<BN, BKC, TN, BKT>::READS;
    i32x4_t fa[2][TM], fb[2][TN];
    fra.read(cur, 0, fa[0]);
    frb.read(cur + A_BYTES, 0, fb[0]);
#pragma unroll
    for (int s = 0; s < BKT / 16; ++s) {
      if (s + 1 < BKT / 16) {
        fra.read(cur, s + 1, fa[(s + 1) & 1]);
        frb.read(cur + A_BYTES, s + 1, fb[(s + 1) & 1]);
        wait_lgkm<R>();
      } else {
        wait_lgkm<0>();
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[s & 1][j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[s & 1][i]), acc[i][j], 0, 0, 0);
    }
  };
  // prologue: tiles 0 and 1 in flight; tile 0 into slot 0
  load(0, ra[0], rb[0]);
  if (nk > 1) load(1, ra[1], rb[1]);
  if (nk > 1) wait_vm<NL>(); else wait_vm<0>();
  __builtin_amdgcn_sched_barrier(0);
  la.store(lds0, ra[0]);
  lb.store(lds0 + A_BYTES, rb[0]);
  wait_lgkm<0>();
  if (nk > 2) load(2, ra[0], rb[0]);
  barrier();
  // tile t sits in registers buffer t & 1 from two iterations before its use, in LDS slot t & 1
  for (int kt0 = 0; kt0 < nk; kt0 += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kt = kt0 + u;
      if (kt >= nk) break;
      compute(lds0 + u * ST);
      if (kt + 1 < nk) {
        if (kt + 2 < nk) wait_vm<NL>(); else wait_vm<0>();   // tile kt+1 landed (kt+2 may be in flight)
        __builtin_amdgcn_sched_barrier(0);
        la.store(lds0 + (1 - u) * ST, ra[1 - u]);
        lb.store(lds0 + (1 - u) * ST + A_BYTES, rb[1 - u]);
        wait_lgkm<0>();
        if (kt + 3 < nk) load(kt + 3, ra[1 - u], rb[1 - u]);
        barrier();
      }
    }
  }
  tile_epilogue<BM, BN, 2, NWM, NWN, false, BKT>(P, acc, z, m0, n0, P.m, smem);
}

template <int BM, int BN, int NWM, int NWN, bool AKC, bool BKC, int BKT>
__global__ __launch_bounds__(64 * NWM * NWN) void gemm_vs_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(1024))) char smem[VsCfg<BM, BN, NWM, NWN, AKC, BKC, BKT>::LDS];
  gemm_body_vs<BM, BN, NWM, NWN, AKC, BKC, BKT>(P, blockIdx.x, smem);
}

template <int BM, int BN, int NWM, int NWN, bool AKC, bool BKC, int BKT>
int launch_vs(GemmParams& P, int batch, hipStream_t s) {
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  hipLaunchKernelGGL((gemm_vs_kernel<BM, BN, NWM, NWN, AKC, BKC, BKT>), dim3(P.tiles_m * P.tiles_n, 1, batch),
                     dim3(64 * NWM * NWN), 0, s, P);
  return vqa::check_launch("vqa_gemm (vgpr-staged)");
}

}  // namespace
