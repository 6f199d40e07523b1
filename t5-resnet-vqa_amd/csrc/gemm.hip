// bf16 MFMA GEMM / implicit-GEMM convolution for gfx950.
//
// One templated kernel covers every contraction of the training step:
//   forward Linear   Y = X W^T          A k-contig (X [M,K]),  B k-contig (W [N,K])
//   input grad       dX = dY W          A k-contig (dY),       B n-contig (W [N,K] read as [K',N'])
//   weight grad      dW = dY^T X        A m-contig (dY [T,N]), B n-contig (X [T,K])
//   conv forward     implicit im2col of an NHWC activation as A (k = (kh,kw,c))
//   conv weight grad implicit im2col as B (ConvTranspose2d dW, resnet_vqa_model.py:72-78)
//
// Tile BM x BN x 64, 256 threads = 4 waves (2x2), each wave (BM/2)x(BN/2) built
// from 32x32 v_mfma_f32_32x32x16_bf16 tiles.  Operand tiles stream HBM -> LDS
// through a STAGES-deep ring filled by global_load_lds_dwordx4 (LDS-DMA, no
// VGPR staging), retired with a counted `s_waitcnt vmcnt` and a raw s_barrier
// so STAGES-1 K-tiles stay in flight across barriers (cdna_hip_programming.md
// §5 "Pipelining across barriers").  LDS images:
//   k-contig operand  -> [rows][64] (128-B rows), chunk ^= (row>>1)&7,
//                        fragments by ds_read_b128 (conflict-free on its 4x16 lane groups);
//   m/n-contig operand-> [64 k][rows], chunk ^= T10 image-(b) pattern,
//                        fragments by ds_read_b64_tr_b16 (hardware transpose).
// glds writes LDS lane-linearly, so the swizzle is applied to the per-lane
// SOURCE address (an XOR involution); lanes whose element is outside the
// matrix / conv padding read a 16-B zero page instead (no predication).
// Block ids are remapped so that blocks sharing an XCD (b % 8) get a
// contiguous range of tiles (bijective form, cdna_hip_programming.md §5).
#include "common.h"

__device__ __attribute__((aligned(64))) uint4 vqa_zero_page[4];   // zero-initialised code-object global

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
};

// byte offset of 16-B chunk `ch` of row `row` in a k-contig image ([rows][64 bf16])
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + ((ch ^ kc_swz(row)) << 4); }
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
template <int ROWS, bool KC, bool GATHER, int NW>
struct Loader {
  static_assert(ROWS % (8 * NW) == 0, "operand tile must split evenly over the waves");
  static_assert(KC || ROWS == 64 || ROWS == 128 || ROWS == 256, "m/n-contig image rows: 64, 128 or 256");
  static constexpr int NI = ROWS / (8 * NW);
  static constexpr int RPI = KC ? 8 : 1024 / (ROWS * 2);
  static constexpr int CPR = KC ? 8 : ROWS / 8;          // 16-B chunks per image row
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
        const int row = ins * 8 + (l >> 3);
        const int ch = (l & 7) ^ kc_swz(row);
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
template <int ROWS, bool KC, int T>
struct FragAddr {
  uint32_t o[KC ? 4 : 2 * T];
  __device__ __forceinline__ void init(int row_base) {
    const int l = threadIdx.x & 63;
    if constexpr (KC) {
      const int row = row_base + (l & 31);
#pragma unroll
      for (int s = 0; s < 4; ++s) o[s] = kc_off(row, 2 * s + (l >> 5));
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
        f[i] = ds_b128(base + o[s] + i * 32 * 128);
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

template <int BM, int BN, int STAGES>
struct TileCfg {
  static constexpr int LDS = STAGES * (BM + BN) * BK * 2;       // LDS ring bytes
};

// One output tile.  `bid` is the tile's linear id within its problem (the
// paired launcher offsets it), `smem` the block's LDS ring (a __shared__ array
// of the calling kernel; inlined, so the LDS address space is preserved).
// NWM x NWN waves, each owning a (BM/NWM) x (BN/NWN) sub-tile.
template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB>
__device__ __forceinline__ void gemm_body(const GemmParams& P, const int bid, char* smem) {
  constexpr int NW = NWM * NWN, NT = 64 * NW;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "wave sub-tile must be whole 32x32 blocks");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, ST_BYTES = A_BYTES + B_BYTES;
  using LA = Loader<BM, AKC, GA, NW>;
  using LB = Loader<BN, BKC, GB, NW>;
  constexpr int NL = LA::NI + LB::NI;                 // glds instructions per thread per K-tile

  // XCD-aware bijective remap of the linear block id; with split-K the slices of
  // one tile are consecutive ids, i.e. (mostly) on one XCD, next to their reducer
  const int S = P.splitk > 1 ? P.splitk : 1;
  const int ntile = P.tiles_m * P.tiles_n;
  const int nwg = ntile * S;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = wg / S, slice = wg - tile * S;
  const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int z = blockIdx.z;
  const bf16_t* A = P.a + (long)z * P.sa;
  const bf16_t* B = P.b + (long)z * P.sb;

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w / NWN, wn = w % NWN;

  LA la;
  LB lb;
  la.init(m0, P.m, P.lda, P.ga);
  lb.init(n0, P.n, P.ldb, P.gb);
  using FA = FragAddr<BM, AKC, TM>;
  using FB = FragAddr<BN, BKC, TN>;
  FA fra;
  FB frb;
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

  const int nk_all = (P.k + BK - 1) / BK;
  const int kb = S > 1 ? slice * P.kper : 0;                  // this slice's first k-tile
  const int nk = S > 1 ? min(nk_all - kb, P.kper) : nk_all;   // >= 1 (host checks)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (s < nk) {
      la.issue(A, P.lda, smem + s * ST_BYTES, (kb + s) * BK, P.k, P.ga);
      lb.issue(B, P.ldb, smem + s * ST_BYTES + A_BYTES, (kb + s) * BK, P.k, P.gb);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + STAGES - 2) - kt;
    wait_tiles<NL, STAGES>(ahead);
    barrier();
    const int nt = kt + STAGES - 1;
    if (nt < nk) {
      char* st = smem + (nt % STAGES) * ST_BYTES;
      la.issue(A, P.lda, st, (kb + nt) * BK, P.k, P.ga);
      lb.issue(B, P.ldb, st + A_BYTES, (kb + nt) * BK, P.k, P.gb);
    }
    const uint32_t cur = lds0 + (kt % STAGES) * ST_BYTES;
    constexpr int R = FA::READS + FB::READS;
    i32x4_t fa[2][TM], fb[2][TN];
    fra.read(cur, 0, fa[0]);
    frb.read(cur + A_BYTES, 0, fb[0]);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      if (s + 1 < BK / 16) {
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
    // __syncthreads (waits for this wave's LDS ops, then barriers); no LDS-DMA is in flight now
    __syncthreads();                                    // every wave is done with the ring
#pragma unroll
    for (int pass = 0; pass < NWM * GPW; ++pass) {
      const int pw = pass / GPW, pg = pass % GPW;
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
      for (int r0 = 0; r0 < HALF; r0 += RPP) {
        const int r = r0 + tid / TPR, row = m0 + pw * WM + pg * HALF + r;
        if (HALF % RPP != 0 && r >= HALF) continue;
        if (NT % TPR != 0 && tid >= RPP * TPR) continue;   // BN = 192: 24 threads per row, 10 rows per sweep
        if (row >= P.m || col >= P.n) continue;
        const float4 x0 = *reinterpret_cast<const float4*>(img + r * LDR + c);
        const float4 x1 = *reinterpret_cast<const float4*>(img + r * LDR + c + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        float kf[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) kf[t] = 1.f;
        if (MK) {
          const uint4 m4 = *reinterpret_cast<const uint4*>(MK + (long)row * P.ldmask + col);
          const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
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
          const float4 a0 = *reinterpret_cast<const float4*>(R32 + (long)row * P.ldres + col);
          const float4 a1 = *reinterpret_cast<const float4*>(R32 + (long)row * P.ldres + col + 4);
          v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w;
          v[4] += a1.x; v[5] += a1.y; v[6] += a1.z; v[7] += a1.w;
        }
        if (R16) {
          const uint4 q = *reinterpret_cast<const uint4*>(R16 + (long)row * P.ldres + col);
          const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += bf2f((t & 1) ? (qw[t >> 1] >> 16) : (qw[t >> 1] & 0xffff));
        }
        if (P.relu) {
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
        }
        if (C32) {
          float4* cp = reinterpret_cast<float4*>(C32 + (long)row * P.ldc32 + col);
          float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
          if (beta) {
            const float4 c0 = cp[0], c1 = cp[1];
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
          if (row >= P.m || col >= P.n) continue;
          float kf = 1.f;
          if (MK && !(bf2f(MK[(long)row * P.ldmask + col]) > 0.f)) kf = 0.f;
          if (dk.on) kf *= drop_mul(dk, (ebase + (uint32_t)row) * (uint32_t)P.n + (uint32_t)col);
          float v = kf * (acc[i][j][e] * P.alpha + (BIAS ? BIAS[col] : 0.f));
          if (R32) v += R32[(long)row * P.ldres + col];
          if (R16) v += bf2f(R16[(long)row * P.ldres + col]);
          if (P.relu) v = fmaxf(v, 0.f);
          if (C32) {
            float* cp = C32 + (long)row * P.ldc32 + col;
            *cp = beta ? v + P.beta * *cp : v;
          }
          if (C16) C16[(long)row * P.ldc16 + col] = f2bf(v);
        }
  }
}

template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB>
__global__ __launch_bounds__(64 * NWM * NWN) void gemm_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<BM, BN, STAGES>::LDS];
  gemm_body<BM, BN, STAGES, NWM, NWN, AKC, BKC, GA, GB>(P, blockIdx.x, smem);
}

// Two independent problems in one launch (the backward's dX and dW of one
// layer share dY): blocks [0, t1) run problem 1, the padding up to a multiple
// of 8 exits (keeps problem 2's XCD remap aligned), the rest run problem 2.
// Fills the chip where either GEMM alone leaves CUs idle and saves a launch.
template <int BM1, int BN1, int S1, int BM2, int BN2, int S2>
__global__ __launch_bounds__(256) void gemm_pair_kernel(GemmParams P1, GemmParams P2, int t1pad) {
  constexpr int L1 = TileCfg<BM1, BN1, S1>::LDS, L2 = TileCfg<BM2, BN2, S2>::LDS;
  __shared__ __attribute__((aligned(1024))) char smem[L1 > L2 ? L1 : L2];
  const int t1 = P1.tiles_m * P1.tiles_n;
  const int bid = blockIdx.x;
  if (bid < t1) {
    gemm_body<BM1, BN1, S1, 2, 2, true, false, false, false>(P1, bid, smem);       // dX: A k-contig, B n-contig
  } else if (bid >= t1pad) {
    gemm_body<BM2, BN2, S2, 2, 2, false, false, false, false>(P2, bid - t1pad, smem);   // dW: both m/n-contig
  }
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

template <int BM, int BN, int STAGES, int NWM, int NWN, bool AKC, bool BKC, bool GA, bool GB>
int launch(GemmParams& P, int batch, hipStream_t s) {
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  if (P.splitk > 1) {                                   // workspace = [counters | slabs]
    const long long tiles = (long long)P.tiles_m * P.tiles_n * batch;
    if (tiles > SPLITK_MAX_TILES) return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: split-K needs <= %lld tiles", SPLITK_MAX_TILES);
    P.cnt = reinterpret_cast<unsigned*>(P.slab);
    P.slab = reinterpret_cast<float*>(reinterpret_cast<char*>(P.slab) + SPLITK_CNT_BYTES);
  }
  dim3 grid(P.tiles_m * P.tiles_n * (P.splitk > 1 ? P.splitk : 1), 1, batch);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, STAGES, NWM, NWN, AKC, BKC, GA, GB>), grid, dim3(64 * NWM * NWN), 0, s, P);
  return vqa::check_launch("vqa_gemm");
}

// config: 0 = auto; 1 = 128x128 (3 stages); 2 = 128x64 (4); 3 = 64x64 (4); 4 = 64x64 (2);
//         5 = 64x64 (3); 6 = 128x64 (2); 7 = 64x128 (2); 8 = 128x128 (2)  -- 4 waves (2x2);
//         9 = 256x128 (2, 8 waves 4x2); 10 = 128x256 (2, 8 waves 2x4); 11 = 256x256 (2, 8 waves 2x4);
//         12 = 256x128 (3, 8 waves 4x2); 13 = 64x192 (2); 14 = 128x192 (2); 15 = 64x192 (3);
//         16 = 128x192 (3) -- 4 waves, k-contiguous B only.
// Every config accumulates each output element in the same K order (BK = 64
// k-tiles, 16-deep MFMA steps), so the choice changes speed, never the bits.
// Auto (measured on MI355X, tools/callprof.py): fewer stages = less LDS = more
// resident blocks, which beats a deep ring at this model's sizes; 128-wide
// tiles only pay for narrow-N, long-K convolutions.  Engines autotune per call.
int auto_config(int m, int n, int k, int batch) {
  const long t128 = (long)vqa::cdiv(m, 128) * vqa::cdiv(n, 128) * batch;
  const int nk = vqa::cdiv(k, BK);
  if (nk <= 2) return 4;
  if (n <= 256 && k >= 1024 && t128 >= 128) return 1;
  if (k >= 2048) return 3;
  return 4;
}

template <bool AKC, bool BKC, bool GA, bool GB>
int dispatch_tile(GemmParams& P, int batch, int config, hipStream_t s) {
  if (config == 0) config = auto_config(P.m, P.n, P.k, batch);
  switch (config) {
    case 1: return launch<128, 128, 3, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 2: return launch<128, 64, 4, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 4: return launch<64, 64, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 5: return launch<64, 64, 3, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 6: return launch<128, 64, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 7: return launch<64, 128, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 8: return launch<128, 128, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 9: return launch<256, 128, 2, 4, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 10: return launch<128, 256, 2, 2, 4, AKC, BKC, GA, GB>(P, batch, s);
    case 11: return launch<256, 256, 2, 2, 4, AKC, BKC, GA, GB>(P, batch, s);
    case 12: return launch<256, 128, 3, 4, 2, AKC, BKC, GA, GB>(P, batch, s);
    case 13: case 14: case 15: case 16:
      // 192-column tiles: one tile per CU for the transformer shapes (2048 x 3072 = 16 x 16 tiles
      // of 128 x 192); the n-contig (transposed-B) LDS image has no 192-row form
      if constexpr (BKC) {
        if (config == 13) return launch<64, 192, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
        if (config == 14) return launch<128, 192, 2, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
        if (config == 15) return launch<64, 192, 3, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
        return launch<128, 192, 3, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
      } else {
        return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: tile config %d needs a k-contiguous B operand (b_trans=0)", config);
      }
    default: return launch<64, 64, 4, 2, 2, AKC, BKC, GA, GB>(P, batch, s);
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// (BM, BN) of a tile config (dispatch_tile's table)
void tile_of(int config, int& bm, int& bn) {
  static const int T[VQA_GEMM_CONFIGS + 1][2] = {{64, 64},   {128, 128}, {128, 64}, {64, 64},  {64, 64},
                                                 {64, 64},   {128, 64},  {64, 128}, {128, 128}, {256, 128},
                                                 {128, 256}, {256, 256}, {256, 128}, {64, 192}, {128, 192},
                                                 {64, 192},  {128, 192}};
  bm = T[config][0];
  bn = T[config][1];
}

// slices actually launched: whole k-tiles per slice, no empty slice
int effective_splitk(int k, int splitk, int* kper) {
  const int nk = vqa::cdiv(k, BK);
  if (splitk <= 1 || nk <= 1) { *kper = nk; return 1; }
  const int per = vqa::cdiv(nk, splitk < nk ? splitk : nk);
  *kper = per;
  return vqa::cdiv(nk, per);
}

}  // namespace

extern "C" int vqa_gemm_select(const vqa_gemm_desc* d) {
  if (!d) return 0;
  return d->config ? d->config : auto_config(d->m, d->n, d->k, d->batch);
}

extern "C" long long vqa_gemm_workspace_bytes(const vqa_gemm_desc* d) {
  if (!d || d->splitk <= 1) return 0;
  int bm, bn, kper;
  tile_of(vqa_gemm_select(d), bm, bn);
  const int S = effective_splitk(d->k, d->splitk, &kper);
  return splitk_bytes(bm, bn, d->m, d->n, d->batch < 1 ? 1 : d->batch, S);
}

static int prepare(const vqa_gemm_desc* d, GemmParams& P) {
  VQA_REQUIRE(d != nullptr, "vqa_gemm: null descriptor");
  VQA_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "vqa_gemm: empty problem m=%d n=%d k=%d", d->m, d->n, d->k);
  VQA_REQUIRE(d->a && d->b, "vqa_gemm: null operand");
  VQA_REQUIRE(d->c32 || d->c16, "vqa_gemm: no output");
  VQA_REQUIRE(aligned16(d->a) && aligned16(d->b), "vqa_gemm: operands must be 16-byte aligned");
  VQA_REQUIRE(d->lda % 8 == 0 && d->ldb % 8 == 0, "vqa_gemm: lda/ldb must be multiples of 8");
  VQA_REQUIRE((d->a_trans && d->b_trans) || d->k % 8 == 0, "vqa_gemm: k must be a multiple of 8 for a k-contig operand");
  VQA_REQUIRE(!d->a_trans || d->m % 8 == 0, "vqa_gemm: m must be a multiple of 8 for m-contig A");
  VQA_REQUIRE(!d->b_trans || d->n % 8 == 0, "vqa_gemm: n must be a multiple of 8 for n-contig B");
  VQA_REQUIRE(!(d->a_conv && d->a_trans), "vqa_gemm: a_conv needs a_trans=0");
  VQA_REQUIRE(!(d->b_conv && !d->b_trans), "vqa_gemm: b_conv needs b_trans=1");
  VQA_REQUIRE(!d->a_conv || d->ga.c % 8 == 0, "vqa_gemm: conv input channels must be a multiple of 8");
  VQA_REQUIRE(!d->b_conv || d->gb.c % 8 == 0, "vqa_gemm: conv input channels must be a multiple of 8");
  VQA_REQUIRE(d->batch >= 1, "vqa_gemm: batch must be >= 1");
  VQA_REQUIRE(d->config >= 0 && d->config <= VQA_GEMM_CONFIGS, "vqa_gemm: config must be 0..%d", VQA_GEMM_CONFIGS);
  VQA_REQUIRE(d->drop.p >= 0.f && d->drop.p < 1.f, "vqa_gemm: dropout p must be in [0, 1)");
  VQA_REQUIRE(!(d->drop.p > 0.f && d->drop.rng && d->relu && (d->res32 || d->res16)),
              "vqa_gemm: relu + residual + dropout is not a supported epilogue");
  P.a = (const bf16_t*)d->a; P.lda = d->lda;
  P.b = (const bf16_t*)d->b; P.ldb = d->ldb;
  P.m = d->m; P.n = d->n; P.k = d->k;
  P.c32 = d->c32; P.ldc32 = d->ldc32;
  P.c16 = (bf16_t*)d->c16; P.ldc16 = d->ldc16;
  P.bias = d->bias; P.res32 = d->res32; P.res16 = (const bf16_t*)d->res16; P.ldres = d->ldres;
  P.mask16 = (const bf16_t*)d->mask16; P.ldmask = d->ldmask;
  P.alpha = d->alpha; P.beta = d->beta; P.relu = d->relu;
  P.ga = d->ga; P.gb = d->gb;
  P.sa = d->stride_a; P.sb = d->stride_b; P.sc32 = d->stride_c32; P.sc16 = d->stride_c16; P.sres = d->stride_res;
  P.drop = d->drop;
  P.sbias = d->stride_bias;
  P.dsite = d->drop_site_stride;
  P.splitk = 1;
  P.kper = 0;
  P.slab = nullptr;
  P.cnt = nullptr;
  VQA_REQUIRE(d->splitk >= 0 && d->splitk <= 64, "vqa_gemm: splitk must be 0..64");
  if (d->splitk > 1) {
    int kper;
    const int S = effective_splitk(d->k, d->splitk, &kper);
    if (S > 1) {
      const long long need = vqa_gemm_workspace_bytes(d);
      VQA_REQUIRE(d->workspace && aligned16(d->workspace), "vqa_gemm: splitk needs a 16-byte aligned workspace");
      VQA_REQUIRE(d->workspace_bytes >= need, "vqa_gemm: workspace %lld bytes < %lld needed for splitk=%d",
                  d->workspace_bytes, need, d->splitk);
      P.splitk = S;
      P.kper = kper;
      P.slab = (float*)d->workspace;
    }
  }
  auto al = [](const void* p, int bytes) { return p == nullptr || ((uintptr_t)p % bytes) == 0; };
  P.vec = d->n % 8 == 0 && (!d->c32 || (d->ldc32 % 8 == 0 && al(d->c32, 16) && d->stride_c32 % 8 == 0)) &&
          (!d->c16 || (d->ldc16 % 8 == 0 && al(d->c16, 16) && d->stride_c16 % 8 == 0)) &&
          (!d->res32 || (d->ldres % 8 == 0 && al(d->res32, 16))) && (!d->res16 || (d->ldres % 8 == 0 && al(d->res16, 16))) &&
          (!d->mask16 || (d->ldmask % 8 == 0 && al(d->mask16, 16))) &&
          (!(d->res32 || d->res16 || d->mask16) || d->stride_res % 8 == 0) && al(d->bias, 16) &&
          d->stride_bias % 4 == 0;
  return VQA_OK;
}

extern "C" int vqa_gemm(const vqa_gemm_desc* d, hipStream_t stream) {
  GemmParams P;
  if (int rc = prepare(d, P)) return rc;
  const int batch = d->batch, cfg = d->config;
  const bool akc = !d->a_trans, bkc = !d->b_trans;
  if (akc && bkc && !d->a_conv) return dispatch_tile<true, true, false, false>(P, batch, cfg, stream);
  if (akc && bkc && d->a_conv) return dispatch_tile<true, true, true, false>(P, batch, cfg, stream);
  if (akc && !bkc && !d->a_conv && !d->b_conv) return dispatch_tile<true, false, false, false>(P, batch, cfg, stream);
  if (!akc && !bkc && !d->b_conv) return dispatch_tile<false, false, false, false>(P, batch, cfg, stream);
  if (!akc && !bkc && d->b_conv) return dispatch_tile<false, false, false, true>(P, batch, cfg, stream);
  if (!akc && bkc) return dispatch_tile<false, true, false, false>(P, batch, cfg, stream);
  return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: unsupported layout combination");
}

namespace {
// tile configs available to the paired launch (a subset of dispatch_tile's)
template <int C> struct CfgOf;
template <> struct CfgOf<3> { static constexpr int BM = 64, BN = 64, S = 4; };
template <> struct CfgOf<4> { static constexpr int BM = 64, BN = 64, S = 2; };
template <> struct CfgOf<6> { static constexpr int BM = 128, BN = 64, S = 2; };
template <> struct CfgOf<7> { static constexpr int BM = 64, BN = 128, S = 2; };

template <int C1, int C2>
int launch_pair(GemmParams& P1, GemmParams& P2, hipStream_t s) {
  using X = CfgOf<C1>;
  using Y = CfgOf<C2>;
  P1.tiles_m = vqa::cdiv(P1.m, X::BM); P1.tiles_n = vqa::cdiv(P1.n, X::BN);
  P2.tiles_m = vqa::cdiv(P2.m, Y::BM); P2.tiles_n = vqa::cdiv(P2.n, Y::BN);
  const int t1 = P1.tiles_m * P1.tiles_n, t1pad = (t1 + 7) / 8 * 8;
  const int grid = t1pad + P2.tiles_m * P2.tiles_n;
  hipLaunchKernelGGL((gemm_pair_kernel<X::BM, X::BN, X::S, Y::BM, Y::BN, Y::S>), dim3(grid), dim3(256), 0, s, P1, P2,
                     t1pad);
  return vqa::check_launch("vqa_gemm_pair");
}

template <int C1>
int pair_second(int c2, GemmParams& P1, GemmParams& P2, hipStream_t s) {
  switch (c2) {
    case 3: return launch_pair<C1, 3>(P1, P2, s);
    case 6: return launch_pair<C1, 6>(P1, P2, s);
    case 7: return launch_pair<C1, 7>(P1, P2, s);
    default: return launch_pair<C1, 4>(P1, P2, s);
  }
}

int pair_cfg(int c) { return (c == 3 || c == 6 || c == 7) ? c : 4; }
}  // namespace

extern "C" int vqa_gemm_pair(const vqa_gemm_desc* dx, const vqa_gemm_desc* dw, hipStream_t stream) {
  GemmParams P1, P2;
  if (int rc = prepare(dx, P1)) return rc;
  if (int rc = prepare(dw, P2)) return rc;
  const bool shape_ok = !dx->a_trans && dx->b_trans && !dx->a_conv && !dx->b_conv && dx->batch == 1 &&
                        dw->a_trans && dw->b_trans && !dw->a_conv && !dw->b_conv && dw->batch == 1 &&
                        P1.splitk == 1 && P2.splitk == 1;
  if (!shape_ok) {                                       // not a (dX, dW) pair: run them one after the other
    if (int rc = vqa_gemm(dx, stream)) return rc;
    return vqa_gemm(dw, stream);
  }
  const int c1 = pair_cfg(vqa_gemm_select(dx)), c2 = pair_cfg(vqa_gemm_select(dw));
  switch (c1) {
    case 3: return pair_second<3>(c2, P1, P2, stream);
    case 6: return pair_second<6>(c2, P1, P2, stream);
    case 7: return pair_second<7>(c2, P1, P2, stream);
    default: return pair_second<4>(c2, P1, P2, stream);
  }
}
