// The GEMM tile body, its kernel and launcher, shared by gemm.hip (bf16 operands) and
// gemm_fp8.hip (e4m3 operands, BASELINE config 5's forward weight GEMMs), which compile as
// separate translation units.
#pragma once
#include "gemm_common.h"

// diagnostic phase stamps (tools/micro/gemm_stamps.hip defines it; a no-op in the library)
#ifndef VQA_GEMM_STAMP
#define VQA_GEMM_STAMP(i)
#endif

namespace {

template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB, bool EXT = false,
          int BKT = BK, bool F8 = false>
__device__ __forceinline__ void gemm_body(const GemmParams& P, const int bid, char* smem) {
  constexpr int NW = NWM * NWN, NT = 64 * NW;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "wave sub-tile must be whole 32x32 blocks");
  constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2, ST_BYTES = A_BYTES + B_BYTES;
  using LA = Loader<BM, AKC, GA, NW, BKT>;
  using LB = Loader<BN, BKC, GB, NW, BKT>;
  constexpr int NL = LA::NI + LB::NI;                 // glds instructions per thread per K-tile

  // XCD-aware bijective remap of the linear block id; with split-K the slices of
  // one tile are consecutive ids, i.e. (mostly) on one XCD, next to their reducer
  const int S = P.splitk > 1 ? P.splitk : 1;
  const int ntile = P.tiles_m * P.tiles_n;
  const int nwg = ntile * S;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = wg / S, slice = wg - tile * S;
  int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  if constexpr (GB) {
    // implicit-im2col B (ConvTranspose2d dW: column = tap * C + c): order the tiles channel
    // block first, so the consecutive tiles an XCD gets are every tap and row tile of ONE
    // channel block -- the 9 taps re-read that slice of the layer4 map from this XCD's L2
    // instead of fetching the whole map 9 times from the Infinity Cache / HBM
    const int cb = P.gb.c / BN;
    if (cb > 0 && P.gb.c % BN == 0 && P.tiles_n % cb == 0) {
      const int taps = P.tiles_n / cb, per = P.tiles_m * taps;
      const int cblk = tile / per, r = tile - cblk * per;
      tm = r / taps;
      tn = (r - tm * taps) * cb + cblk;
    }
  }
  const int m0 = tm * BM, n0 = tn * BN;

  const int z = blockIdx.z;
  const bf16_t* A = P.a + (long)z * P.sa;
  const bf16_t* B = P.b + (long)z * P.sb;

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w / NWN, wn = w % NWN;

  VQA_GEMM_STAMP(0);
  LA la;
  LB lb;
  la.init(m0, P.m, P.lda, P.ga);
  lb.init(n0, P.n, P.ldb, P.gb);
  using FA = FragAddr<BM, AKC, TM, BKT>;
  using FB = FragAddr<BN, BKC, TN, BKT>;
  static_assert(!F8 || (AKC && BKC && !GA && !GB), "fp8 operands: k-contiguous A and B, no implicit im2col");
  FA fra;
  FB frb;
  FragAddr8<TM, BKT> f8a;
  FragAddr8<TN, BKT> f8b;
  if constexpr (F8) {
    f8a.init(wm * WM);
    f8b.init(wn * WN);
  } else {
    fra.init(wm * WM);
    frb.init(wn * WN);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk_all = (P.k + BKT - 1) / BKT;
  const int kb = S > 1 ? slice * P.kper : 0;                  // this slice's first k-tile
  const int nk = S > 1 ? min(nk_all - kb, P.kper) : nk_all;   // >= 1 (host checks)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (s < nk) {
      la.issue(A, P.lda, smem + s * ST_BYTES, (kb + s) * BKT, P.k, P.ga);
      lb.issue(B, P.ldb, smem + s * ST_BYTES + A_BYTES, (kb + s) * BKT, P.k, P.gb);
    }
  }
  VQA_GEMM_STAMP(1);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + STAGES - 2) - kt;
    wait_tiles<NL, STAGES>(ahead);
    barrier();
    if (kt == 0) VQA_GEMM_STAMP(2);
    const int nt = kt + STAGES - 1;
    if (nt < nk) {
      char* st = smem + (nt % STAGES) * ST_BYTES;
      la.issue(A, P.lda, st, (kb + nt) * BKT, P.k, P.ga);
      lb.issue(B, P.ldb, st + A_BYTES, (kb + nt) * BKT, P.k, P.gb);
    }
    const uint32_t cur = lds0 + (kt % STAGES) * ST_BYTES;
    if constexpr (F8) {
      // e4m3: one 128-B image row = STEPS x 64 k; scaled MFMA at unit scales (e8m0 127 = 2^0),
      // the per-row / per-column fp32 scales are applied after the k-loop
      constexpr int ST8 = FragAddr8<TM, BKT>::STEPS;
      constexpr int R8 = FragAddr8<TM, BKT>::READS + FragAddr8<TN, BKT>::READS;
      i32x8_t ga[2][TM], gb[2][TN];
      f8a.read(cur, 0, ga[0]);
      f8b.read(cur + A_BYTES, 0, gb[0]);
#pragma unroll
      for (int t = 0; t < ST8; ++t) {
        if (t + 1 < ST8) {
          f8a.read(cur, t + 1, ga[(t + 1) & 1]);
          f8b.read(cur + A_BYTES, t + 1, gb[(t + 1) & 1]);
          wait_lgkm<R8>();
        } else {
          wait_lgkm<0>();
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(gb[t & 1][j], ga[t & 1][i], acc[i][j], 0, 0,
                                                                         0, 127, 0, 127);
      }
      continue;
    }
    constexpr int R = FA::READS + FB::READS;
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
          // swapped operands: D = B^T-tile x A^T-tile, so a lane owns one output ROW and
          // 4 consecutive output COLUMNS per register group (vectorised epilogue)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[s & 1][j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[s & 1][i]),
                                                              acc[i][j], 0, 0, 0);
    }
  }

  if (S > 1) {
    // Split-K hand-off (cdna_hip_programming.md Guideline 16, R1 form): every slice
    // stores its partials WRITE-THROUGH (sc1 buffer stores, 1 KiB contiguous per wave
    // store, fragment order), every storing wave drains, then one lane counts the
    // arrival with a relaxed agent-scope atomic.  The slice that arrives last reads
    // the other slices' partials with sc1 loads (no release/acquire fences needed)
    // and sums all slices IN SLICE ORDER, its own from registers -- the result does
    // not depend on arrival order.  No workgroup waits on another (nothing can
    // hang); the reducer resets the counter for the next launch.
    typedef __attribute__((address_space(1))) unsigned gu32;
    constexpr int FR = TM * TN * 1024;                  // floats per wave
    const long tlin = (long)z * ntile + tile;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(P.slab + tlin * S * (long)(BM * BN), (short)0, S * BM * BN * 4, 0x00020000);
    const int wof = w * FR + l * 4;                     // this lane's float offset inside a slice
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const i32x4_t v = {__float_as_int(acc[i][j][4 * g]), __float_as_int(acc[i][j][4 * g + 1]),
                             __float_as_int(acc[i][j][4 * g + 2]), __float_as_int(acc[i][j][4 * g + 3])};
          __builtin_amdgcn_raw_buffer_store_b128(v, rs, (slice * (BM * BN) + wof + (i * TN + j) * 1024 + g * 256) * 4,
                                                 0, 16);
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // EVERY storing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);           // the ring is idle (the K loop drained every DMA)
    if (tid == 0) {
      gu32* c = (gu32*)(P.cnt + tlin);
      const unsigned prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == (unsigned)(S - 1);
      if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16_t t;
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = 0.f;
        for (int s = 0; s < S; ++s) {
          if (s == slice) {
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] += acc[i][j][e];
          } else {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const i32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(
                  rs, (s * (BM * BN) + wof + (i * TN + j) * 1024 + g * 256) * 4, 0, 16);
              t[4 * g] += __int_as_float(v[0]);
              t[4 * g + 1] += __int_as_float(v[1]);
              t[4 * g + 2] += __int_as_float(v[2]);
              t[4 * g + 3] += __int_as_float(v[3]);
            }
          }
        }
        acc[i][j] = t;
      }
  }

  if constexpr (F8) {                                  // acc(m, n) * scale_a[m] * scale_b[n]
    const float* qa = P.qsa + (long)z * P.sqa;
    const float* qb = P.qsb + (long)z * P.sqb;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * WM + i * 32 + (l & 31);
      const float sa = row < P.m ? qa[row] : 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = n0 + wn * WN + j * 32 + 8 * g + 4 * (l >> 5);    // n % 4 == 0 (host check)
          const float4 sb = col < P.n ? *reinterpret_cast<const float4*>(qb + col) : make_float4(0.f, 0.f, 0.f, 0.f);
          acc[i][j][4 * g] *= sa * sb.x;
          acc[i][j][4 * g + 1] *= sa * sb.y;
          acc[i][j][4 * g + 2] *= sa * sb.z;
          acc[i][j][4 * g + 3] *= sa * sb.w;
        }
    }
  }
  VQA_GEMM_STAMP(3);
  tile_epilogue<BM, BN, STAGES, NWM, NWN, EXT, BKT>(P, acc, z, m0, n0, P.m, smem);
  VQA_GEMM_STAMP(4);
}

template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB, int BKT = BK,
          bool F8 = false>
__global__ __launch_bounds__(64 * NWM * NWN) void gemm_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<BM, BN, STAGES, BKT>::LDS];
  gemm_body<BM, BN, STAGES, NWM, NWN, AKC, BKC, GA, GB, false, BKT, F8>(P, blockIdx.x, smem);
}

// One k-tile (K <= 64: the frozen ResNet's 1x1 convolutions over 64 channels, tile configs 26-28):
// the ring's second stage is never filled (the prologue issues k-tile 0 into stage 0 and the loop
// issues nothing more), so the workgroup allocates ONE stage and the register target follows the
// LDS: 64x128 / 128x64 in 24 KB at 4 workgroups per CU (the two-stage kernels: 48 KB and 140
// VGPRs, 3 per CU), 64x64 in 16 KB at 5.  Same body, same k order: the bits do not change.
template <int BM, int BN, int W, bool AKC, bool BKC, bool GA, bool GB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void gemm_k1_kernel(GemmParams P) {
  // the epilogue parks one 32-row fragment group per pass (TM = 1 or 2 here): it must fit one stage
  static_assert(32 * (BN + 4) * 4 <= TileCfg<BM, BN, 1>::LDS, "epilogue image must fit the single stage");
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<BM, BN, 1>::LDS];
  gemm_body<BM, BN, 2, 2, 2, AKC, BKC, GA, GB>(P, blockIdx.x, smem);
}

// split-K workspace: a fixed 64 KiB counter block first (so any sequence of calls
// sharing a workspace only ever finds zeros there), then the slabs
constexpr long long SPLITK_CNT_BYTES = 65536;
constexpr long long SPLITK_MAX_TILES = SPLITK_CNT_BYTES / 4;
long long splitk_bytes(int bm, int bn, int m, int n, int batch, int S) {
  if (S <= 1) return 0;
  const long long tiles = (long long)vqa::cdiv(m, bm) * vqa::cdiv(n, bn) * batch;
  return SPLITK_CNT_BYTES + tiles * S * bm * bn * 4;
}

template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB, int BKT = BK,
          bool F8 = false>
int launch(GemmParams& P, int batch, hipStream_t s) {
  if (BKT != BK && P.splitk > 1)                        // split-K slices are counted in 64-deep k-tiles
    return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: 128-deep k-tile configs take no split-K");
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  if (P.splitk > 1) {                                   // workspace = [counters | slabs]
    const long long tiles = (long long)P.tiles_m * P.tiles_n * batch;
    if (tiles > SPLITK_MAX_TILES) return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: split-K needs <= %lld tiles", SPLITK_MAX_TILES);
    P.cnt = reinterpret_cast<unsigned*>(P.slab);
    P.slab = reinterpret_cast<float*>(reinterpret_cast<char*>(P.slab) + SPLITK_CNT_BYTES);
  }
  dim3 grid(P.tiles_m * P.tiles_n * (P.splitk > 1 ? P.splitk : 1), 1, batch);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, STAGES, NWM, NWN, AKC, BKC, GA, GB, BKT, F8>), grid, dim3(64 * NWM * NWN), 0,
                     s, P);
  return vqa::check_launch("vqa_gemm");
}

template <int BM, int BN, int W, bool AKC, bool BKC, bool GA, bool GB>
int launch_k1(GemmParams& P, int batch, hipStream_t s) {
  if (P.k > BK || P.splitk > 1)
    return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: tile configs 26-28 take one k-tile (k <= %d), no split-K", BK);
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  dim3 grid(P.tiles_m * P.tiles_n, 1, batch);
  hipLaunchKernelGGL((gemm_k1_kernel<BM, BN, W, AKC, BKC, GA, GB>), grid, dim3(256), 0, s, P);
  return vqa::check_launch("vqa_gemm");
}


}  // namespace
