// Device-side building blocks shared by the GEMM / implicit-GEMM convolution kernels
// (gemm.hip) and the LDS-patch 3x3 convolution (conv_patch.hip): the parameter block,
// the LDS-DMA operand loaders, the fragment readers, the counted waits and the fused
// epilogue.  Included by exactly those translation units (anonymous namespace: each
// code object gets its own copy).
#pragma once
#include "common.h"

static __device__ __attribute__((aligned(64))) uint4 vqa_zero_page[4];   // zero-initialised code-object global

namespace {

constexpr int BK = 64;
typedef __attribute__((address_space(3))) void lds_void_t;

struct GemmParams {
  const bf16_t* a; long lda;
  const bf16_t* b; long ldb;
  int m, n, k;
  float* c32; long ldc32;
  bf16_t* c16; long ldc16;
  const float* bias;
  const float* res32; const bf16_t* res16; long ldres;
  const bf16_t* mask16; long ldmask;
  float alpha, beta; int relu;
  vqa_conv_geom ga, gb;
  long sa, sb, sc32, sc16, sres;
  int tiles_m, tiles_n;
  int vec;                 // LDS-staged 8-wide epilogue legal (N, ld*, pointers 16-B aligned)
  vqa_dropout drop;        // dropout of the (alpha*acc + bias) branch
  int splitk, kper;        // K slices and 64-deep k-tiles per slice (splitk <= 1: no split)
  float* slab;             // [batch][tile][slice][BM*BN] fp32 partials, fragment order
  unsigned* cnt;           // [batch][tile] arrival counters (zero between launches)
  long sbias;              // bias stride per batch element
  int dsite;               // != 0: batch z uses dropout site + z*dsite, element indices from 0
  // fp8 (e4m3) operands (vqa_gemm_desc.fp8): a / b hold bytes (lda, ldb, k, sa, sb in units of
  // 2 bytes, so the bf16 loaders stage them unchanged); acc(m, n) is scaled by qsa[m] * qsb[n]
  const float* qsa; const float* qsb;
  long sqa, sqb;           // scale strides per batch element
};

// byte offset of 16-B chunk `ch` of row `row` in a k-contig image ([rows][BKT bf16]):
// 128-B rows (BKT 64, two rows per 256-B bank row): chunk ^= (row>>1)&7;
// 256-B rows (BKT 128, one row per bank row): chunk ^= row&15, so the 16 lanes of a
// ds_read_b128 group (16 consecutive rows, one logical chunk) hit 16 distinct chunks
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + ((ch ^ kc_swz(row)) << 4); }
template <int BKT>
__device__ __forceinline__ int kc_swz_t(int row) { if constexpr (BKT == 128) return row & 15; else return kc_swz(row); }
template <int BKT>
__device__ __forceinline__ int kc_off_t(int row, int ch) { return row * (BKT * 2) + ((ch ^ kc_swz_t<BKT>(row)) << 4); }
// byte offset of chunk `ch` of k-row `kr` in an m/n-contig image ([64][ROWLEN bf16])
template <int ROWLEN>
__device__ __forceinline__ int mn_swz(int kr) {
  // 256- and 512-B rows: the bank of a chunk depends on its index mod 16 only,
  // so the same XOR keeps ds_read_b64_tr_b16 conflict-free for both
  if constexpr (ROWLEN >= 128) return ((kr & 3) << 2) | ((kr >> 2) & 3);
  else return ((((kr >> 1) & 1) << 2) | ((kr >> 2) & 3));
}
template <int ROWLEN>
__device__ __forceinline__ int mn_off(int kr, int ch) {
  return kr * (ROWLEN * 2) + ((ch ^ mn_swz<ROWLEN>(kr)) << 4);
}

// a / d for 0 <= a < 2^22 via a float reciprocal + one-step correction (no integer division)
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = (int)((float)a * inv);
  q -= (q * d > a) ? 1 : 0;
  q += ((q + 1) * d <= a) ? 1 : 0;
  return q;
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// ---------------------------------------------------------------- LDS-DMA loader
// One operand tile of ROWS (m or n) x 64 (k): ROWS*128 bytes = ROWS/8 wave
// instructions of 1 KiB; NI per wave (NW waves).  KC image: 8 rows per
// instruction; MN image: 1024 / (2*ROWS) k-rows per instruction.
template <int ROWS, bool KC, bool GATHER, int NW, int BKT = BK>
struct Loader {
  static_assert(BKT == 64 || (BKT == 128 && !GATHER), "128-deep k-tiles: plain operands only");
  static constexpr int KCPR = BKT / 8;                   // 16-B chunks per k-contig row
  static_assert(ROWS * BKT * 2 % (1024 * NW) == 0, "operand tile must split evenly over the waves");
  static_assert(KC || ROWS == 64 || ROWS == 128 || ROWS == 256, "m/n-contig image rows: 64, 128 or 256");
  static constexpr int NI = ROWS * BKT * 2 / (1024 * NW);
  static constexpr int RPI = KC ? 64 / KCPR : 1024 / (ROWS * 2);
  static constexpr int CPR = KC ? KCPR : ROWS / 8;       // 16-B chunks per image row
  long off[NI];            // KC: element offset of (row, chunk) at k0 = 0; MN: column index
  int kof[NI];             // KC: k offset of the chunk inside the tile; MN: k-row inside the tile
  int g0[NI], g1[NI], g2[NI];
  bool ok[NI];

  __device__ __forceinline__ void init(int row0, int nrows, long ld, const vqa_conv_geom& g) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int ins = w * NI + j;
      if constexpr (KC) {
        const int row = ins * RPI + l / KCPR;
        const int ch = (l % KCPR) ^ kc_swz_t<BKT>(row);
        const int grow = row0 + row;
        ok[j] = grow < nrows;
        kof[j] = ch * 8;
        off[j] = (long)grow * ld + ch * 8;
        if constexpr (GATHER) {                  // output pixel (img, oh, ow) of this row
          if (ok[j]) {
            const int hw = g.oh * g.ow;
            const int im = grow / hw, rem = grow - im * hw;
            const int oh = rem / g.ow, ow = rem - oh * g.ow;
            g0[j] = im; g1[j] = oh * g.stride - g.pad; g2[j] = ow * g.stride - g.pad;
            // element offset of this chunk at tap (0, 0); a tap adds (kh*W + kw)*C
            off[j] = (((long)im * g.h + g1[j]) * g.w + g2[j]) * g.c + kof[j];
          } else {
            g0[j] = 0; g1[j] = -(1 << 28); g2[j] = -(1 << 28);
          }
        }
      } else {
        const int kr = ins * RPI + l / CPR;
        const int ch = (l % CPR) ^ mn_swz<ROWS>(kr);
        const int col = row0 + ch * 8;
        ok[j] = col < nrows;
        off[j] = col;
        kof[j] = kr;
        if constexpr (GATHER) {                  // feature (kh, kw, c) of this column
          const int tap = col / g.c;
          g1[j] = col - tap * g.c;
          g0[j] = tap / g.kw;
          g2[j] = tap - g0[j] * g.kw;
        }
      }
    }
  }

  __device__ __forceinline__ void issue(const bf16_t* __restrict__ base, long ld, char* stage, int k0, int K,
                                        const vqa_conv_geom& g) {
    const int w = threadIdx.x >> 6;
    // implicit-im2col A: when C is a multiple of the K-tile (every conv but the stem), the
    // whole tile shares one (kh, kw) tap -- one uniform division per tile instead of
    // three per 16-B chunk
    bool cfast = false;
    int tkh = 0, tkw = 0, tc0 = 0;
    long toff = 0;
    float ihw = 0.f, iow = 0.f;
    if constexpr (!KC && GATHER) {
      ihw = 1.f / (float)(g.oh * g.ow);
      iow = 1.f / (float)g.ow;
    }
    // ... and when one kernel row is exactly one K-tile (the space-to-depth stem: C 16,
    // 4 taps), a chunk's (kw, c) is its offset inside the tile: the row is contiguous
    bool rfast = false;
    if constexpr (KC && GATHER) {
      cfast = (g.c & (BK - 1)) == 0;
      rfast = !cfast && g.c * g.kw == BK;
      if (cfast) {
        const int tap = k0 / g.c;
        tc0 = k0 - tap * g.c;
        tkh = tap / g.kw;
        tkw = tap - tkh * g.kw;
        toff = (long)(tkh * g.w + tkw) * g.c + tc0;
      } else if (rfast) {
        tkh = k0 / BK;
        toff = (long)tkh * g.w * g.c;
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const void* src = vqa_zero_page;
      const int kk = k0 + kof[j];
      if (ok[j] && kk < K) {
        if constexpr (KC && !GATHER) {
          src = base + off[j] + k0;
        } else if constexpr (KC && GATHER) {
          if (cfast) {                                  // the K-tile lies inside one tap
            const int ih = g1[j] + tkh, iw = g2[j] + tkw;
            if (ih >= 0 && ih < g.h && iw >= 0 && iw < g.w) src = base + off[j] + toff;
          } else if (rfast) {                           // the K-tile is kernel row tkh
            const int ih = g1[j] + tkh, iw = g2[j] + kof[j] / g.c;
            if (ih >= 0 && ih < g.h && iw >= 0 && iw < g.w) src = base + off[j] + toff;
          } else {
            const int tap = kk / g.c;
            const int c = kk - tap * g.c;
            const int kh = tap / g.kw, kw = tap - kh * g.kw;
            const int ih = g1[j] + kh, iw = g2[j] + kw;
            if (ih >= 0 && ih < g.h && iw >= 0 && iw < g.w)
              src = base + (((long)g0[j] * g.h + ih) * g.w + iw) * g.c + c;
          }
        } else if constexpr (!KC && !GATHER) {
          src = base + (long)kk * ld + off[j];
        } else {
          const int hw = g.oh * g.ow;
          const int im = fdiv(kk, hw, ihw), rem = kk - im * hw;
          const int oh = fdiv(rem, g.ow, iow), ow = rem - oh * g.ow;
          const int kh = g0[j], kw = g2[j];
          const int ih = oh * g.stride - g.pad + kh, iw = ow * g.stride - g.pad + kw;
          if (ih >= 0 && ih < g.h && iw >= 0 && iw < g.w)
            src = base + (((long)im * g.h + ih) * g.w + iw) * g.c + g1[j];
        }
      }
      glds16(src, stage + (w * NI + j) * 1024);
    }
  }
};

// ---------------------------------------------------------------- fragment reads
// Issued as inline asm: the compiler cannot prove a ds_read does not alias an
// in-flight LDS-DMA of the ring and would otherwise put `s_waitcnt vmcnt(0)`
// in front of every K-tile's first read, draining the pipeline.  The waits
// are therefore explicit (counted lgkmcnt + sched_barrier, guide §5.4 rule 18).
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ i32x4_t ds_b128(uint32_t addr) {
  i32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ i32x2_t ds_tr16(uint32_t addr) {
  i32x2_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Per-lane LDS byte offsets of one operand's fragments (k-step 0), relative to
// the operand image base.  KC: lane reads row (base + l&31), chunk 2s + (l>>5);
// MN: two ds_read_b64_tr_b16 per fragment (k rows 16s+8h+q and +4).
template <int ROWS, bool KC, int T, int BKT = BK>
struct FragAddr {
  uint32_t o[KC ? BKT / 16 : 2 * T];
  __device__ __forceinline__ void init(int row_base) {
    const int l = threadIdx.x & 63;
    if constexpr (KC) {
      const int row = row_base + (l & 31);
#pragma unroll
      for (int s = 0; s < BKT / 16; ++s) o[s] = kc_off_t<BKT>(row, 2 * s + (l >> 5));
    } else {
      const int h = l >> 5, g1 = (l >> 4) & 1, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
      for (int i = 0; i < T; ++i) {
        const int col = row_base + i * 32 + 16 * g1 + 4 * p;
        const int ch = col >> 3, half = (col >> 2) & 1;
        const int kr0 = 8 * h + q;
        o[2 * i] = mn_off<ROWS>(kr0, ch) + 8 * half;
        o[2 * i + 1] = mn_off<ROWS>(kr0 + 4, ch) + 8 * half;
      }
    }
  }
  // issue the reads of k-step s for the T fragments of this wave
  __device__ __forceinline__ void read(uint32_t base, int s, i32x4_t (&f)[T]) const {
#pragma unroll
    for (int i = 0; i < T; ++i) {
      if constexpr (KC) {
        f[i] = ds_b128(base + o[s] + i * 32 * (BKT * 2));
      } else {
        const uint32_t so = s * 16 * ROWS * 2;          // 16 k-rows per step; swizzle is s-invariant
        const i32x2_t lo = ds_tr16(base + o[2 * i] + so);
        const i32x2_t hi = ds_tr16(base + o[2 * i + 1] + so);
        f[i] = i32x4_t{lo[0], lo[1], hi[0], hi[1]};
      }
    }
  }
  static constexpr int READS = KC ? T : 2 * T;
};

// Per-lane LDS byte offsets of one e4m3 operand's fragments for the 64-deep scaled MFMA
// (v_mfma_scale_f32_32x32x64_f8f6f4): a 128-B k-contig image row holds 128 fp8 = two steps;
// lane l reads row l&31, 32 contiguous bytes = chunks 4t + 2(l>>5) and +1 of step t.  Both
// operands use the same lane -> k map, so the products are summed over the same k whatever
// order the instruction assigns inside a step.
typedef int i32x8_t __attribute__((ext_vector_type(8)));
template <int T, int BKT = BK>
struct FragAddr8 {
  static constexpr int STEPS = BKT / 32;                  // 64-deep fp8 steps per k-tile
  uint32_t o[STEPS][2];
  __device__ __forceinline__ void init(int row_base) {
    const int l = threadIdx.x & 63;
    const int row = row_base + (l & 31);
#pragma unroll
    for (int t = 0; t < STEPS; ++t)
#pragma unroll
      for (int c = 0; c < 2; ++c) o[t][c] = kc_off_t<BKT>(row, 4 * t + 2 * (l >> 5) + c);
  }
  __device__ __forceinline__ void read(uint32_t base, int t, i32x8_t (&f)[T]) const {
#pragma unroll
    for (int i = 0; i < T; ++i) {
      const i32x4_t lo = ds_b128(base + o[t][0] + i * 32 * (BKT * 2));
      const i32x4_t hi = ds_b128(base + o[t][1] + i * 32 * (BKT * 2));
      f[i] = i32x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
  static constexpr int READS = 2 * T;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int NL, int STAGES>
__device__ __forceinline__ void wait_tiles(int ahead) {
  // keep `ahead` younger K-tiles (NL loads each) in flight, retire everything older
  if constexpr (STAGES >= 4) {
    if (ahead >= 2) { wait_vm<2 * NL>(); return; }
  }
  if constexpr (STAGES >= 3) {
    if (ahead >= 1) { wait_vm<NL>(); return; }
  }
  wait_vm<0>();
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN, int STAGES, int BKT = BK>
struct TileCfg {
  static constexpr int LDS = STAGES * (BM + BN) * BKT * 2;      // LDS ring bytes
};

// One output tile.  `bid` is the tile's linear id within its problem (the
// paired launcher offsets it), `smem` the block's LDS ring (a __shared__ array
// of the calling kernel; inlined, so the LDS address space is preserved).
// NWM x NWN waves, each owning a (BM/NWM) x (BN/NWN) sub-tile.
// The fused epilogue of one output tile (shared by every kernel of this family).
// acc[i][j][4g+t] -> row m0+wm*WM+i*32+(l&31), col n0+wn*WN+j*32+8g+4(l>>5)+t; rows at or
// beyond `mlim` are not stored (the GEMMs pass P.m; the patch convolution the end of its
// tile's valid output rows).
// epilogue activation (vqa_gemm_desc.relu): 1 ReLU, 2 GELU (erf form, torch's default
// nn.functional.gelu: ViT intermediate), 3 tanh (ViT pooler)
// (EXT epilogues only -- one kernel instantiation, gemm_ext_kernel; compact branch-free
// forms: erf by Abramowitz-Stegun 7.1.26, |error| < 1.5e-7, far below the bf16 rounding
// of the output)
__device__ __forceinline__ float epi_act(float v, int a) {
  if (a == 1) return fmaxf(v, 0.f);
  if (a == 2) {
    const float x = v * 0.7071067811865476f, ax = fabsf(x);
    const float t = 1.f / (1.f + 0.3275911f * ax);
    const float y = 1.f - ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t +
                           0.254829592f) * t * __expf(-ax * ax);
    return 0.5f * v * (1.f + copysignf(y, x));
  }
  const float e = __expf(-2.f * fabsf(v));
  return copysignf((1.f - e) / (1.f + e), v);
}

template <int BM, int BN, int STAGES, int NWM, int NWN, bool EXT = false, int BKT = BK>
__device__ __forceinline__ void tile_epilogue(const GemmParams& P, f32x16_t (&acc)[BM / NWM / 32][BN / NWN / 32],
                                              const int z, const int m0, const int n0, const int mlim, char* smem) {
  // no FMA contraction: every tile config and epilogue path (operands prefetched or loaded in the
  // sweep, vectorised or scalar) must round each element the same way -- the config is a speed
  // choice only (tests/test_gemm_gpu.py::test_all_tile_configs_bitwise_identical)
#pragma clang fp contract(off)
  constexpr int NW = NWM * NWN, NT = 64 * NW;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  constexpr int ST_BYTES = (BM + BN) * BKT * 2;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w / NWN, wn = w % NWN;
  // epilogue: acc[i][j][4g+t] -> row m0+wm*WM+i*32+(l&31), col n0+wn*WN+j*32+8g+4(l>>5)+t.
  // Per element: k = [mask > 0] * dropout multiplier (1 if neither), then
  //   v = k*(alpha*acc + bias) + res ; relu ; c32 = v + beta*c32 ; c16 = bf16(v).
  // (relu(k*t) == k*relu(t) for k >= 0, and with a residual relu acts after it.)
  float* C32 = P.c32 ? P.c32 + (long)z * P.sc32 : nullptr;
  bf16_t* C16 = P.c16 ? P.c16 + (long)z * P.sc16 : nullptr;
  const float* R32 = P.res32 ? P.res32 + (long)z * P.sres : nullptr;
  const bf16_t* R16 = P.res16 ? P.res16 + (long)z * P.sres : nullptr;
  const bf16_t* MK = P.mask16 ? P.mask16 + (long)z * P.sres : nullptr;
  const bool beta = P.beta != 0.f && C32;
  vqa_dropout dz = P.drop;
  if (P.dsite) dz.site += (unsigned)(z * P.dsite);
  const DropK dk = drop_init(dz);
  // dropout element index = (z*m + row)*n + col (one site), or row*n + col at site + z*dsite
  const uint32_t ebase = P.dsite ? 0u : (uint32_t)z * (uint32_t)P.m;
  const float* BIAS = P.bias ? P.bias + (long)z * P.sbias : nullptr;
  const int rl = l & 31, ch = l >> 5;
  if (P.vec) {
    // Staged through LDS (the ring is idle now): each wave parks alpha*acc of its
    // fragments as fp32 rows, then all NT threads walk the tile row-major, 8
    // columns (16-32 B) per thread, so every global access -- bias, residual,
    // mask, old C, the stores -- is a full coalesced line instead of 16-B
    // pieces of 32 rows.  One pass per wave row (WM rows) bounds the image.
    constexpr int LDR = BN + 4;                         // fp32 row stride (+16 B: spreads the banks)
    constexpr int RING = STAGES * ST_BYTES;
    // 32-row fragment groups parked per pass: a wave row's whole sub-tile when it fits
    constexpr int G = (TM * 32 * LDR * 4 <= RING) ? TM : ((TM / 2) * 32 * LDR * 4 <= RING ? TM / 2 : 1);
    constexpr int HALF = G * 32;                        // rows per pass
    constexpr int GPW = TM / G;                         // passes per wave row
    static_assert(TM % G == 0 && HALF * LDR * 4 <= RING, "epilogue image must fit the ring");
    float* img = reinterpret_cast<float*>(smem);
    constexpr int TPR = BN / 8;                         // threads per row
    constexpr int RPP = NT / TPR;                       // rows per sweep
    constexpr int NSW = (HALF + RPP - 1) / RPP;         // row sweeps per pass
    // Operand prefetch: the residual (fp32 or bf16) -- or, without one, the old C of a beta
    // epilogue -- and the ReLU mask of every sweep of a pass are loaded BEFORE the pass's LDS
    // staging, so their HBM round trips overlap each other and the staging.  In the sweep loop
    // each sweep's stores precede the next sweep's loads (a C store may alias later operand rows,
    // so the compiler keeps that order): one dependent round trip per sweep, ~4 us per 128 x 64
    // tile of the ResNet's residual 1x1 convolutions (r05 stamps).  Same operands, same
    // arithmetic: the bits do not change.  Up to 4 sweeps (the register budget).
    constexpr bool PF = NSW <= 4;
    const int pfk = R32 ? 1 : (R16 ? 2 : (beta ? 3 : 0));   // what pre[] holds
    f32x4_t pre[PF ? NSW : 1][2];                      // native vectors: register-resident (float4
    i32x4_t mpre[PF ? NSW : 1];                         // structs would live in scratch)
    // __syncthreads (waits for this wave's LDS ops, then barriers); no LDS-DMA is in flight now
    __syncthreads();                                    // every wave is done with the ring
#pragma unroll
    for (int pass = 0; pass < NWM * GPW; ++pass) {
      const int pw = pass / GPW, pg = pass % GPW;
      if constexpr (PF) {
        const int c = (tid % TPR) * 8, col = n0 + c;
#pragma unroll
        for (int sw = 0; sw < NSW; ++sw) {
          const int r = sw * RPP + tid / TPR, row = m0 + pw * WM + pg * HALF + r;
          if ((HALF % RPP != 0 && r >= HALF) || (NT % TPR != 0 && tid >= RPP * TPR) || row >= mlim || col >= P.n)
            continue;
          if (pfk == 1) {
            pre[sw][0] = *reinterpret_cast<const f32x4_t*>(R32 + (long)row * P.ldres + col);
            pre[sw][1] = *reinterpret_cast<const f32x4_t*>(R32 + (long)row * P.ldres + col + 4);
          } else if (pfk == 2) {
            pre[sw][0] = __builtin_bit_cast(f32x4_t, *reinterpret_cast<const i32x4_t*>(R16 + (long)row * P.ldres + col));
          } else if (pfk == 3) {
            pre[sw][0] = *reinterpret_cast<const f32x4_t*>(C32 + (long)row * P.ldc32 + col);
            pre[sw][1] = *reinterpret_cast<const f32x4_t*>(C32 + (long)row * P.ldc32 + col + 4);
          }
          if (MK) mpre[sw] = *reinterpret_cast<const i32x4_t*>(MK + (long)row * P.ldmask + col);
        }
      }
      if (wm == pw) {
#pragma unroll
        for (int ii = 0; ii < G; ++ii)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int i = pg * G + ii;
              const int r = ii * 32 + rl, c = wn * WN + j * 32 + 8 * g + 4 * ch;
              *reinterpret_cast<float4*>(img + r * LDR + c) =
                  make_float4(acc[i][j][4 * g] * P.alpha, acc[i][j][4 * g + 1] * P.alpha,
                              acc[i][j][4 * g + 2] * P.alpha, acc[i][j][4 * g + 3] * P.alpha);
            }
      }
      __syncthreads();                                  // the fragment writes have landed
      const int c = (tid % TPR) * 8, col = n0 + c;
#pragma unroll
      for (int sw = 0; sw < NSW; ++sw) {
        const int r = sw * RPP + tid / TPR, row = m0 + pw * WM + pg * HALF + r;
        if (HALF % RPP != 0 && r >= HALF) continue;
        if (NT % TPR != 0 && tid >= RPP * TPR) continue;   // BN = 192: 24 threads per row, 10 rows per sweep
        if (row >= mlim || col >= P.n) continue;
        const float4 x0 = *reinterpret_cast<const float4*>(img + r * LDR + c);
        const float4 x1 = *reinterpret_cast<const float4*>(img + r * LDR + c + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        float kf[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) kf[t] = 1.f;
        if (MK) {
          const i32x4_t m4 = PF ? mpre[PF ? sw : 0] : *reinterpret_cast<const i32x4_t*>(MK + (long)row * P.ldmask + col);
          const uint32_t mw[4] = {(uint32_t)m4[0], (uint32_t)m4[1], (uint32_t)m4[2], (uint32_t)m4[3]};
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (!(bf2f((t & 1) ? (mw[t >> 1] >> 16) : (mw[t >> 1] & 0xffff)) > 0.f)) kf[t] = 0.f;
        }
        if (dk.on) {
          const uint32_t e = (ebase + (uint32_t)row) * (uint32_t)P.n + (uint32_t)col;
#pragma unroll
          for (int t = 0; t < 8; ++t) kf[t] *= drop_mul(dk, e + t);
        }
        if (BIAS) {
          const float4 b0 = *reinterpret_cast<const float4*>(BIAS + col);
          const float4 b1 = *reinterpret_cast<const float4*>(BIAS + col + 4);
          const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += bb[t];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] *= kf[t];
        if (R32) {
          const bool pr = PF && pfk == 1;
          const f32x4_t a0 = pr ? pre[PF ? sw : 0][0] : *reinterpret_cast<const f32x4_t*>(R32 + (long)row * P.ldres + col);
          const f32x4_t a1 = pr ? pre[PF ? sw : 0][1] : *reinterpret_cast<const f32x4_t*>(R32 + (long)row * P.ldres + col + 4);
          v[0] += a0[0]; v[1] += a0[1]; v[2] += a0[2]; v[3] += a0[3];
          v[4] += a1[0]; v[5] += a1[1]; v[6] += a1[2]; v[7] += a1[3];
        }
        if (R16) {
          const i32x4_t q = (PF && pfk == 2) ? __builtin_bit_cast(i32x4_t, pre[PF ? sw : 0][0])
                               : *reinterpret_cast<const i32x4_t*>(R16 + (long)row * P.ldres + col);
          const uint32_t qw[4] = {(uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3]};
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += bf2f((t & 1) ? (qw[t >> 1] >> 16) : (qw[t >> 1] & 0xffff));
        }
        if (P.relu) {
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] = EXT ? epi_act(v[t], P.relu) : fmaxf(v[t], 0.f);
        }
        if (C32) {
          float4* cp = reinterpret_cast<float4*>(C32 + (long)row * P.ldc32 + col);
          float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
          if (beta) {
            const bool pc = PF && pfk == 3;                 // prefetched old C (no residual)
            const f32x4_t c0 = pc ? pre[PF ? sw : 0][0] : *reinterpret_cast<const f32x4_t*>(cp),
                          c1 = pc ? pre[PF ? sw : 0][1] : *reinterpret_cast<const f32x4_t*>(cp + 1);
            o0.x += P.beta * c0.x; o0.y += P.beta * c0.y; o0.z += P.beta * c0.z; o0.w += P.beta * c0.w;
            o1.x += P.beta * c1.x; o1.y += P.beta * c1.y; o1.z += P.beta * c1.z; o1.w += P.beta * c1.w;
          }
          cp[0] = o0;
          cp[1] = o1;
        }
        if (C16) {
          uint4 u;
          u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
          u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
          *reinterpret_cast<uint4*>(C16 + (long)row * P.ldc16 + col) = u;
        }
      }
      if (pass + 1 < NWM * GPW) __syncthreads();        // image reused by the next pass
    }
  } else {
    // generic scalar path (odd N or leading dimensions)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = m0 + wm * WM + i * 32 + rl;
          const int col = n0 + wn * WN + j * 32 + 8 * (e >> 2) + 4 * ch + (e & 3);
          if (row >= mlim || col >= P.n) continue;
          float kf = 1.f;
          if (MK && !(bf2f(MK[(long)row * P.ldmask + col]) > 0.f)) kf = 0.f;
          if (dk.on) kf *= drop_mul(dk, (ebase + (uint32_t)row) * (uint32_t)P.n + (uint32_t)col);
          float v = kf * (acc[i][j][e] * P.alpha + (BIAS ? BIAS[col] : 0.f));
          if (R32) v += R32[(long)row * P.ldres + col];
          if (R16) v += bf2f(R16[(long)row * P.ldres + col]);
          if (P.relu) v = EXT ? epi_act(v, P.relu) : fmaxf(v, 0.f);
          if (C32) {
            float* cp = C32 + (long)row * P.ldc32 + col;
            *cp = beta ? v + P.beta * *cp : v;
          }
          if (C16) C16[(long)row * P.ldc16 + col] = f2bf(v);
        }
  }
}

}  // namespace
