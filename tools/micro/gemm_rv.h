// GEMM tile body with ONE operand read straight from global memory into the MFMA operand
// registers ("register-direct", rv) and only the other one staged through the LDS-DMA ring.
//
// Why: the barrier ring of gemm_body.h moves both operands by LDS-DMA, and its
// k-loop is paced by the per-wave cost of issuing those 1-KiB pieces (60-185 cycles each,
// MI355X_MICROARCH.md 'LDS-DMA piece issue cost'), not by the MFMAs: a 64x64x128 slot of 32 KB
// takes ~0.63 us against ~0.21 us of matrix work.  A k-contiguous operand's 32x32x16 MFMA
// fragment is 16 contiguous bytes per lane (row l & 31, k-chunk l >> 5), so it can be loaded
// with one buffer_load_dwordx4 per fragment and no LDS round trip at all; the LDS ring then
// carries the other operand alone: half the DMA pieces per k-tile, half the ring, room for a
// deeper prefetch.  Each wave loads only the fragments of its own columns (DB: B) or rows
// (!DB: A), so with a 1 x NWN wave grid (DB) no byte is loaded twice.
//
// Pipelining: k-tile t's group = {direct loads of t, LDS-DMA of t} is issued PD k-tiles ahead
// (ring of PD + 1 slots, PD + 1 register buffers, the k-loop unrolled by PD + 1 so every buffer
// index is static).  At k-tile t the wave waits until only the groups issued after t's are in
// flight (counted vmcnt: loads and LDS-DMA retire in issue order), then the barrier (every
// wave's DMA pieces of slot t have landed and every wave is done with the slot refilled next).
//
// Each output element accumulates its 16-deep MFMA steps in increasing k exactly as gemm_body
// does, so results are bit-identical to every other tile config (test_all_tile_configs_bitwise).
#pragma once
#include "../../t5-resnet-vqa_amd/csrc/gemm_common.h"

namespace {

// zeros for the direct loads of rows past the matrix (a k-tile of 128 bf16 = 256 B past the lane's
// 16-B chunk offset)
static __device__ __attribute__((aligned(64))) uint4 vqa_zero_rv[32];

template <int OFF>
__device__ __forceinline__ i32x4_t gload16(const char* p) {
  i32x4_t v;
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(v) : "v"(p), "n"(OFF) : "memory");
  return v;
}

// the KS 16-deep k-steps of one fragment row: loads at byte offsets 0, 32, 64, ... (immediates)
template <int S, int KS>
__device__ __forceinline__ void gload_steps(i32x4_t (&d)[KS], const char* p) {
  if constexpr (S < KS) {
    d[S] = gload16<32 * S>(p);
    gload_steps<S + 1, KS>(d, p);
  }
}

template <int NL, int PD>
__device__ __forceinline__ void wait_groups(int younger) {
  // keep `younger` groups (NL vector-memory ops each) in flight, retire everything older
  if constexpr (PD >= 3) {
    if (younger >= 2) { wait_vm<2 * NL>(); __builtin_amdgcn_sched_barrier(0); return; }
  }
  if constexpr (PD >= 2) {
    if (younger >= 1) { wait_vm<NL>(); __builtin_amdgcn_sched_barrier(0); return; }
  }
  wait_vm<0>();
  __builtin_amdgcn_sched_barrier(0);
}

template <int BM, int BN, int NWM, int NWN, bool DB, bool LKC, int BKT, int PD>
struct RvCfg {
  static constexpr int NW = NWM * NWN;
  static constexpr int LROWS = DB ? BM : BN;                       // rows of the LDS operand's tile
  static constexpr int SLOT = LROWS * BKT * 2;
  static constexpr int RING = (PD + 1) * SLOT;
  static constexpr int EPI = (BM + BN) * BKT * 2;                  // tile_epilogue's image (1 "stage")
  static constexpr int LDS = RING > EPI ? RING : EPI;
};

template <int BM, int BN, int NWM, int NWN, bool DB, bool LKC, int BKT, int PD>
__device__ __forceinline__ void gemm_body_rv(const GemmParams& P, const int bid, char* smem) {
  using C = RvCfg<BM, BN, NWM, NWN, DB, LKC, BKT, PD>;
  constexpr int NW = C::NW;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "wave sub-tile must be whole 32x32 blocks");
  static_assert(PD >= 1 && PD <= 3, "prefetch distance 1..3");
  constexpr int KS = BKT / 16;                                     // 16-deep MFMA steps per k-tile
  constexpr int TD = DB ? TN : TM;                                 // direct fragments per k-step
  using LL = Loader<C::LROWS, LKC, false, NW, BKT>;
  constexpr int NL = LL::NI + TD * KS;                             // vector-memory ops per thread per k-tile

  // XCD-aware bijective remap (gemm_body): consecutive tiles share an XCD's L2
  const int ntile = P.tiles_m * P.tiles_n;
  const int xcd = bid & 7, q8 = ntile >> 3, r8 = ntile & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;
  const bf16_t* A = P.a + (long)z * P.sa;
  const bf16_t* B = P.b + (long)z * P.sb;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w / NWN, wn = w % NWN;

  // LDS operand: the ring loader and fragment addresses of gemm_body
  LL ll;
  if constexpr (DB) ll.init(m0, P.m, P.lda, P.ga);
  else ll.init(n0, P.n, P.ldb, P.gb);
  FragAddr<C::LROWS, LKC, DB ? TM : TN, BKT> fl;
  fl.init(DB ? wm * WM : wn * WN);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // direct operand: lane l owns row (l & 31) of each 32-row fragment, k-chunk l >> 5; rows past
  // the matrix read the zero page (and do not advance with k).  K % BKT == 0 (host check), so a
  // k-tile never straddles the end of a row.
  const bf16_t* D = DB ? B : A;
  const long ldd = DB ? P.ldb : P.lda;
  const int drows = DB ? P.n : P.m;
  const char* dptr[TD];
  int dadv[TD];
  const int r0 = DB ? n0 + wn * WN : m0 + wm * WM;
#pragma unroll
  for (int i = 0; i < TD; ++i) {
    const int row = r0 + i * 32 + (l & 31);
    const bool ok = row < drows;
    dptr[i] = ok ? reinterpret_cast<const char*>(D + (long)row * ldd) + 16 * (l >> 5)
                 : reinterpret_cast<const char*>(vqa_zero_rv);
    dadv[i] = ok ? BKT * 2 : 0;
  }
  const int K = P.k;

  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  i32x4_t dr[PD + 1][TD][KS];                                      // direct fragments, one buffer per k-tile
  const int nk = (K + BKT - 1) / BKT;

  // issue k-tile t's group: its direct fragments into buffer `buf`, its LDS tile into slot t % (PD+1)
  auto issue = [&](int t, i32x4_t (&db)[TD][KS]) {
    // the direct fragments by inline asm: the compiler's waitcnt pass cannot see the counted
    // group waits above and put `s_waitcnt vmcnt(0)` in front of the k-loop's MFMAs when these
    // were builtins; every use sits behind wait_groups (+ sched_barrier)
#pragma unroll
    for (int i = 0; i < TD; ++i) {
      gload_steps<0, KS>(db[i], dptr[i] + (long)t * dadv[i]);
    }
    char* st = smem + (t % (PD + 1)) * C::SLOT;
    if constexpr (DB) ll.issue(A, P.lda, st, t * BKT, K, P.ga);
    else ll.issue(B, P.ldb, st, t * BKT, K, P.gb);
  };

#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < nk) issue(p, dr[p]);

  for (int kt0 = 0; kt0 < nk; kt0 += PD + 1) {
#pragma unroll
    for (int u = 0; u <= PD; ++u) {
      const int kt = kt0 + u;
      if (kt >= nk) break;
      wait_groups<NL, PD>(min(PD - 1, nk - 1 - kt));
      barrier();
      if (kt + PD < nk) issue(kt + PD, dr[(u + PD) % (PD + 1)]);
      const uint32_t cur = lds0 + u * C::SLOT;                     // kt0 % (PD + 1) == 0
      constexpr int TL = DB ? TM : TN;
      constexpr int R = decltype(fl)::READS;
      i32x4_t fr[2][TL];
      fl.read(cur, 0, fr[0]);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (s + 1 < KS) {
          fl.read(cur, s + 1, fr[(s + 1) & 1]);
          wait_lgkm<R>();
        } else {
          wait_lgkm<0>();
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            i32x4_t fa, fb;
            if constexpr (DB) {
              fa = fr[s & 1][i];
              fb = dr[u][j][s];
            } else {
              fa = dr[u][i][s];
              fb = fr[s & 1][j];
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb),
                                                                __builtin_bit_cast(bf16x8_t, fa), acc[i][j], 0, 0, 0);
          }
      }
    }
  }
  tile_epilogue<BM, BN, 1, NWM, NWN, false, BKT>(P, acc, z, m0, n0, P.m, smem);
}

template <int BM, int BN, int NWM, int NWN, bool DB, bool LKC, int BKT, int PD>
__global__ __launch_bounds__(64 * NWM * NWN) void gemm_rv_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(1024))) char smem[RvCfg<BM, BN, NWM, NWN, DB, LKC, BKT, PD>::LDS];
  gemm_body_rv<BM, BN, NWM, NWN, DB, LKC, BKT, PD>(P, blockIdx.x, smem);
}

template <int BM, int BN, int NWM, int NWN, bool DB, bool LKC, int BKT, int PD>
int launch_rv(GemmParams& P, int batch, hipStream_t s) {
  if (P.splitk > 1) return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: register-direct tile configs take no split-K");
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  hipLaunchKernelGGL((gemm_rv_kernel<BM, BN, NWM, NWN, DB, LKC, BKT, PD>), dim3(P.tiles_m * P.tiles_n, 1, batch),
                     dim3(64 * NWM * NWN), 0, s, P);
  return vqa::check_launch("vqa_gemm (register-direct)");
}

}  // namespace
