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
// from 32x32 v_mfma_f32_32x32x16_bf16 tiles.  Operands are register-staged
// into a double-buffered LDS image:
//   k-contig operand  -> [rows][64] (128-B rows), XOR swizzle chunk^((row>>1)&7),
//                        fragments by ds_read_b128 (conflict-free on the 4x16 lane groups);
//   m/n-contig operand-> [64 k][rows], XOR swizzle per T10 image (b),
//                        fragments by ds_read_b64_tr_b16 (hardware transpose).
// Block ids are remapped so that the blocks sharing an XCD (b % 8) get a
// contiguous range of tiles (bijective form, cdna_hip_programming.md §5).
#include "common.h"

namespace {

constexpr int BK = 64;
constexpr int NT = 256;

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
};

// byte offset of 16-B chunk `ch` of row `row` in a k-contig image ([rows][64 bf16])
__device__ __forceinline__ int kc_off(int row, int ch) {
  return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
}
// byte offset of chunk `ch` of k-row `kr` in an m/n-contig image ([64][ROWLEN bf16])
template <int ROWLEN>
__device__ __forceinline__ int mn_off(int kr, int ch) {
  if constexpr (ROWLEN == 128) {
    return kr * 256 + ((ch ^ (((kr & 3) << 2) | ((kr >> 2) & 3))) << 4);
  } else {
    static_assert(ROWLEN == 64, "row length");
    return kr * 128 + ((ch ^ ((((kr >> 1) & 1) << 2) | ((kr >> 2) & 3))) << 4);
  }
}

// ---------------------------------------------------------------- staging
// One operand tile: ROWS x 64 (k-contig) or 64 x ROWS (m/n-contig), ROWS*8 chunks.
template <int ROWS, bool KC, bool GATHER>
struct Stager {
  static constexpr int NCH = ROWS * 8 / NT;     // 16-B chunks per thread
  static constexpr int CPR = ROWS / 8;          // chunks per k-row in the m/n-contig image
  uint4 r[NCH];
  // gather state (KC: per-chunk output pixel; MN: per-thread (kh,kw,c))
  int img[GATHER && KC ? NCH : 1], ih0[GATHER && KC ? NCH : 1], iw0[GATHER && KC ? NCH : 1];
  int fkh, fkw, fc;

  __device__ __forceinline__ void init(int row0, int nrows, const vqa_conv_geom& g) {
    const int tid = threadIdx.x;
    if constexpr (GATHER && KC) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        int row = row0 + ((i * NT + tid) >> 3);
        if (row < nrows) {
          int hw = g.oh * g.ow;
          int im = row / hw, rem = row - im * hw;
          int oh = rem / g.ow, ow = rem - oh * g.ow;
          img[i] = im; ih0[i] = oh * g.stride - g.pad; iw0[i] = ow * g.stride - g.pad;
        } else {
          img[i] = 0; ih0[i] = -(1 << 28); iw0[i] = -(1 << 28);
        }
      }
    }
    if constexpr (GATHER && !KC) {
      int col = row0 + (tid % CPR) * 8;       // feature index (kh,kw,c)
      int tap = col / g.c;
      fc = col - tap * g.c;
      fkh = tap / g.kw;
      fkw = tap - fkh * g.kw;
    }
  }

  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int row0, int nrows,
                                       int k0, int K, const vqa_conv_geom& g) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = i * NT + tid;
      bool ok;
      const bf16_t* p;
      if constexpr (KC) {
        const int row = row0 + (idx >> 3);
        const int kk = k0 + (idx & 7) * 8;
        ok = (row < nrows) & (kk < K);
        if constexpr (!GATHER) {
          p = base + (long)row * ld + kk;
        } else {
          int tap = kk / g.c;
          int c = kk - tap * g.c;
          int kh = tap / g.kw, kw = tap - kh * g.kw;
          int ih = ih0[i] + kh, iw = iw0[i] + kw;
          ok = ok & (ih >= 0) & (ih < g.h) & (iw >= 0) & (iw < g.w);
          p = base + (((long)img[i] * g.h + ih) * g.w + iw) * g.c + c;
        }
      } else {
        const int kr = idx / CPR;
        const int col = row0 + (idx % CPR) * 8;
        const int kk = k0 + kr;
        ok = (kk < K) & (col < nrows);
        if constexpr (!GATHER) {
          p = base + (long)kk * ld + col;
        } else {
          int hw = g.oh * g.ow;
          int im = kk / hw, rem = kk - im * hw;
          int oh = rem / g.ow, ow = rem - oh * g.ow;
          int ih = oh * g.stride - g.pad + fkh, iw = ow * g.stride - g.pad + fkw;
          ok = ok & (ih >= 0) & (ih < g.h) & (iw >= 0) & (iw < g.w);
          p = base + (((long)im * g.h + ih) * g.w + iw) * g.c + fc;
        }
      }
      r[i] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
    }
  }

  __device__ __forceinline__ void store(char* lds) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = i * NT + tid;
      int off;
      if constexpr (KC) off = kc_off(idx >> 3, idx & 7);
      else off = mn_off<ROWS>(idx / CPR, idx % CPR);
      *reinterpret_cast<uint4*>(lds + off) = r[i];
    }
  }
};

// fragment of one 32-row MFMA operand tile at k-step s (16 deep)
template <int ROWS, bool KC>
__device__ __forceinline__ bf16x8_t read_frag(const char* lds, int row_base, int s) {
  const int l = threadIdx.x & 63;
  if constexpr (KC) {
    const int row = row_base + (l & 31);
    const int ch = 2 * s + (l >> 5);
    uint4 v = *reinterpret_cast<const uint4*>(lds + kc_off(row, ch));
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    const int h = l >> 5, g1 = (l >> 4) & 1, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
    const int col = row_base + 16 * g1 + 4 * p;
    const int ch = col >> 3, half = (col >> 2) & 1;
    const int kr0 = 16 * s + 8 * h + q;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4_t*)(lds + mn_off<ROWS>(kr0, ch) + 8 * half));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4_t*)(lds + mn_off<ROWS>(kr0 + 4, ch) + 8 * half));
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

template <int BM, int BN, bool AKC, bool BKC, bool GA, bool GB>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmParams P) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  // XCD-aware bijective remap of the linear block id
  const int nwg = P.tiles_m * P.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / P.tiles_n, tn = wg - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int z = blockIdx.z;
  const bf16_t* A = P.a + (long)z * P.sa;
  const bf16_t* B = P.b + (long)z * P.sb;

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w >> 1, wn = w & 1;

  Stager<BM, AKC, GA> sa;
  Stager<BN, BKC, GB> sb;
  sa.init(m0, P.m, P.ga);
  sb.init(n0, P.n, P.gb);

  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = (P.k + BK - 1) / BK;
  sa.load(A, P.lda, m0, P.m, 0, P.k, P.ga);
  sb.load(B, P.ldb, n0, P.n, 0, P.k, P.gb);
  sa.store(smem);
  sb.store(smem + A_BYTES);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * (A_BYTES + B_BYTES);
    char* nxt = smem + ((kt + 1) & 1) * (A_BYTES + B_BYTES);
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, P.lda, m0, P.m, (kt + 1) * BK, P.k, P.ga);
      sb.load(B, P.ldb, n0, P.n, (kt + 1) * BK, P.k, P.gb);
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<BM, AKC>(cur, wm * WM + i * 32, s);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<BN, BKC>(cur + A_BYTES, wn * WN + j * 32, s);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(nxt);
      sb.store(nxt + A_BYTES);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][e] -> row m0+wm*WM+i*32+(e&3)+8*(e>>2)+4*(l>>5), col n0+wn*WN+j*32+(l&31)
  float* C32 = P.c32 ? P.c32 + (long)z * P.sc32 : nullptr;
  bf16_t* C16 = P.c16 ? P.c16 + (long)z * P.sc16 : nullptr;
  const float* R32 = P.res32 ? P.res32 + (long)z * P.sres : nullptr;
  const bf16_t* R16 = P.res16 ? P.res16 + (long)z * P.sres : nullptr;
  const bf16_t* MK = P.mask16 ? P.mask16 + (long)z * P.sres : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 32 + (l & 31);
    if (col >= P.n) continue;
    const float bias = P.bias ? P.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
        if (row >= P.m) continue;
        float v = acc[i][j][e] * P.alpha + bias;
        if (R32) v += R32[(long)row * P.ldres + col];
        if (R16) v += bf2f(R16[(long)row * P.ldres + col]);
        if (P.relu) v = fmaxf(v, 0.f);
        if (MK && !(bf2f(MK[(long)row * P.ldmask + col]) > 0.f)) v = 0.f;
        if (C32) {
          float* cp = C32 + (long)row * P.ldc32 + col;
          *cp = P.beta != 0.f ? v + P.beta * *cp : v;
        }
        if (C16) C16[(long)row * P.ldc16 + col] = f2bf(v);
      }
    }
  }
}

template <int BM, int BN, bool AKC, bool BKC, bool GA, bool GB>
int launch(GemmParams& P, int batch, hipStream_t s) {
  P.tiles_m = vqa::cdiv(P.m, BM);
  P.tiles_n = vqa::cdiv(P.n, BN);
  dim3 grid(P.tiles_m * P.tiles_n, 1, batch);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AKC, BKC, GA, GB>), grid, dim3(NT), 0, s, P);
  return vqa::check_launch("vqa_gemm");
}

template <bool AKC, bool BKC, bool GA, bool GB>
int dispatch_tile(GemmParams& P, int batch, hipStream_t s) {
  // Largest tile that still gives >= ~1 wave of blocks over 256 CUs.
  const long t128 = (long)vqa::cdiv(P.m, 128) * vqa::cdiv(P.n, 128) * batch;
  const long t12864 = (long)vqa::cdiv(P.m, 128) * vqa::cdiv(P.n, 64) * batch;
  if (t128 >= 256) return launch<128, 128, AKC, BKC, GA, GB>(P, batch, s);
  if (t12864 >= 256) return launch<128, 64, AKC, BKC, GA, GB>(P, batch, s);
  return launch<64, 64, AKC, BKC, GA, GB>(P, batch, s);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int vqa_gemm(const vqa_gemm_desc* d, hipStream_t stream) {
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
  GemmParams P;
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
  const int batch = d->batch;
  const bool akc = !d->a_trans, bkc = !d->b_trans;
  if (akc && bkc && !d->a_conv) return dispatch_tile<true, true, false, false>(P, batch, stream);
  if (akc && bkc && d->a_conv) return dispatch_tile<true, true, true, false>(P, batch, stream);
  if (akc && !bkc && !d->a_conv && !d->b_conv) return dispatch_tile<true, false, false, false>(P, batch, stream);
  if (!akc && !bkc && !d->b_conv) return dispatch_tile<false, false, false, false>(P, batch, stream);
  if (!akc && !bkc && d->b_conv) return dispatch_tile<false, false, false, true>(P, batch, stream);
  if (!akc && bkc) return dispatch_tile<false, true, false, false>(P, batch, stream);
  return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: unsupported layout combination");
}
