// 3x3 / stride-1 / pad-1 convolution of an NHWC bf16 activation as an implicit GEMM whose
// A operand comes from an input PATCH staged once per 64-channel chunk in LDS -- the
// frozen ResNet's 3x3 convolutions except the three stride-2 ones
// (torchvision Bottleneck.conv2 / BasicBlock.conv1-2, run at resnet_vqa_model.py:126-132).
//
// gemm.hip's implicit im2col (a_conv = 1) DMA-gathers the A tile of every (tap, channel
// chunk) k-tile from L2: each input pixel crosses the L2 -> LDS path 9 times, and that
// path (~60 GB/s per CU) is what bounds the convolution.  Here a tile is R whole output
// rows of ONE image (R = min(BM / W, H); m rows R*W..BM-1 are padding, never stored), its
// input patch is (R + 2) x (W + 2) pixels (zero border) x 64 channels, and the nine taps
// of a chunk read their A fragments straight out of that patch at a per-tap pixel offset:
//   A(row r, tap (kh, kw), c) = patch[(r / W + kh) * (W + 2) + r % W + kw][c].
// K is ordered (chunk, tap, c) -- the weights are stored [Cout][C / 64][9][64] -- so a
// chunk's nine k-tiles follow each other.  With more than one chunk the patch is double
// buffered: the next chunk's patch streams in, in parts, alongside the B loads of taps
// S-1..8 of the current chunk (earlier issue slots still overlap the previous chunk's last
// reads).  B (the weights) streams through an S-stage LDS-DMA ring with counted waits as
// in gemm.hip (padding DMAs keep every k-tile's count equal).
// Per chunk the L2 -> LDS bytes drop from 9 * BM * 128 to (R + 2)(W + 2) * 128 for A.
//
// Numerics: the same bf16 products, fp32 accumulation in 64-deep k-tiles and 16-deep MFMA
// steps as gemm.hip; only the order of the k-tiles differs (chunk-major), so the result
// equals the a_conv = 1 path up to fp32 summation order.
// Included by gemm.hip (one translation unit: it shares gemm.hip's GemmParams and prepare()).
#pragma once
#include "gemm_common.h"

namespace {

struct PatchGeom {
  int R;        // output rows per tile
  int rbs;      // row blocks per image: ceil(H / R)
  int npix;     // patch pixels (R + 2) * (W + 2)
  int pins;     // 1-KiB DMA instructions per patch: ceil(npix / 8)
  int chunks;   // C / 64
  int ppart;    // patch instructions per part (double-buffered: ceil(pins / 8))
};

// one 1-KiB DMA instruction q of the patch of chunk `cc` (pixels 8q .. 8q+7) into `pb`
__device__ __forceinline__ void patch_issue(const bf16_t* __restrict__ x, const vqa_conv_geom& g, const PatchGeom& G,
                                            int q, int b, int rb, int cc, char* pb, float iw2) {
  const int l = threadIdx.x & 63;
  const int pp = q * 8 + (l >> 3);
  const int W2 = g.w + 2;
  const int srow = fdiv(pp, W2, iw2), pcol = pp - srow * W2;
  const int ih = rb * G.R + srow - 1, iw = pcol - 1;
  const int ch = (l & 7) ^ kc_swz(pp);
  const void* src = vqa_zero_page;
  if (pp < G.npix && ih >= 0 && ih < g.h && iw >= 0 && iw < g.w)
    src = x + (((long)b * g.h + ih) * g.w + iw) * g.c + cc * 64 + ch * 8;
  glds16(src, pb + q * 1024);
}

template <int BM, int BN, int NWM, int NWN, int PMAX, bool DB, int S>
struct PatchCfg {
  static constexpr int NW = NWM * NWN;
  static constexpr int PATCH = PMAX * 128;                   // bytes of one patch buffer
  static constexpr int NPB = DB ? 2 : 1;
  static constexpr int B_STAGE = BN * BK * 2;
  static constexpr int B_OFF = NPB * PATCH;
  static constexpr int DUMMY = B_OFF + S * B_STAGE;           // 1 KiB per wave: target of the padding DMAs
  static constexpr int EPI = 2 * (BM + BN) * BK * 2;          // the epilogue's staging image (tile_epilogue)
  static constexpr int BODY = DUMMY + NW * 1024;
  static constexpr int LDS = BODY > EPI ? BODY : EPI;
  // double-buffered: the next chunk's patch rides in parts on the issue slots of taps S-1..8
  // (earlier slots still overlap the previous chunk's reads); every slot carries exactly NIP
  // patch DMAs per wave (real or padding), so the counted waits see NL loads per k-tile
  static constexpr int PARTS = 10 - S;
  static constexpr int NIP = DB ? ((PMAX / 8 + PARTS - 1) / PARTS + NW - 1) / NW : 0;
};

template <int BM, int BN, int NWM, int NWN, int PMAX, bool DB, int S>
__global__ __launch_bounds__(64 * NWM * NWN) void conv_patch_kernel(GemmParams P, PatchGeom G) {
  using C = PatchCfg<BM, BN, NWM, NWN, PMAX, DB, S>;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  constexpr int NW = NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN, TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "wave sub-tile must be whole 32x32 blocks");
  static_assert(S >= 2 && S <= 4, "2..4 B stages");
  using LB = Loader<BN, true, false, NW>;
  using FB = FragAddr<BN, true, TN>;
  constexpr int NL = LB::NI + C::NIP;                         // DMA instructions per wave per k-tile
  const vqa_conv_geom& g = P.ga;

  // tile -> (image, row block, column tile); XCD-aware bijective remap as in gemm_body
  const int ntile = P.tiles_m * P.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = ntile >> 3, r8 = ntile & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
  const int b = tm / G.rbs, rb = tm - b * G.rbs;
  const int rows = min(G.R, g.h - rb * G.R) * g.w;             // valid output rows of this tile
  const int m0 = (b * g.h + rb * G.R) * g.w, n0 = tn * BN;

  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = w / NWN, wn = w % NWN;
  LB lb;
  lb.init(n0, P.n, P.ldb, P.gb);
  FB frb;
  frb.init(wn * WN);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const float iw2 = 1.f / (float)(g.w + 2);
  char* dummy = smem + C::DUMMY + w * 1024;

  // A fragments: this lane's output row of fragment i -> its patch pixel at tap (0, 0)
  int pbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WM + i * 32 + (l & 31);
    const int orow = r / g.w, ocol = r - orow * g.w;
    pbase[i] = r < rows ? orow * (g.w + 2) + ocol : -1;
  }

  f32x16_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = 9 * G.chunks;
  // the loads of k-tile slot nt: its B tile, and (double-buffered) NIP patch DMAs per wave
  auto issue_slot = [&](int nt) {
    lb.issue(P.b, P.ldb, smem + C::B_OFF + (nt % S) * C::B_STAGE, nt * BK, P.k, P.gb);
    if constexpr (DB) {
      const int cc = nt / 9, t = nt - cc * 9;
      const bool live = t >= S - 1 && cc + 1 < G.chunks;
      char* pb = smem + ((cc + 1) & 1) * C::PATCH;
#pragma unroll
      for (int u = 0; u < C::NIP; ++u) {
        const int qi = w + u * NW;                         // this wave's u-th DMA of the part
        const int q = (t - (S - 1)) * G.ppart + qi;
        if (live && qi < G.ppart && q < G.pins) patch_issue(P.a, g, G, q, b, rb, cc + 1, pb, iw2);
        else glds16(vqa_zero_page, dummy);
      }
    }
  };
  // prologue: the whole patch of chunk 0 (older than every counted load), then S-1 slots
  for (int q = w; q < G.pins; q += NW) patch_issue(P.a, g, G, q, b, rb, 0, smem, iw2);
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue_slot(s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + S - 2) - kt;
    wait_tiles<NL, S>(ahead);                           // k-tile kt (and everything before it) landed
    barrier();
    const int nt = kt + S - 1;
    if (nt < nk) issue_slot(nt);
    const int cc = kt / 9, tap = kt - cc * 9;
    const int kh = tap / 3, kw = tap - kh * 3;
    const uint32_t pa = lds0 + (DB ? (cc & 1) * C::PATCH : 0);
    const uint32_t pbB = lds0 + C::B_OFF + (kt % S) * C::B_STAGE;
    uint32_t pp[TM], sw[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int p = pbase[i] < 0 ? 0 : pbase[i] + kh * (g.w + 2) + kw;
      pp[i] = pa + p * 128;
      sw[i] = kc_swz(p);
    }
    constexpr int R_ = TM + FB::READS;
    i32x4_t fa[2][TM], fb[2][TN];
    auto read_a = [&](int s, i32x4_t (&f)[TM]) {
#pragma unroll
      for (int i = 0; i < TM; ++i) f[i] = ds_b128(pp[i] + (((2 * s + (l >> 5)) ^ sw[i]) << 4));
    };
    read_a(0, fa[0]);
    frb.read(pbB, 0, fb[0]);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      if (s + 1 < BK / 16) {
        read_a(s + 1, fa[(s + 1) & 1]);
        frb.read(pbB, s + 1, fb[(s + 1) & 1]);
        wait_lgkm<R_>();
      } else {
        wait_lgkm<0>();
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[s & 1][j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[s & 1][i]),
                                                              acc[i][j], 0, 0, 0);
    }
  }
  tile_epilogue<BM, BN, 2, NWM, NWN>(P, acc, 0, m0, n0, m0 + rows, smem);
}

constexpr int PMAX_SB = 272;     // single chunk (C = 64): W = 56 / 64 at R = 2 -> 232 / 264 pixels
constexpr int PMAX_DB = 208;     // double-buffered chunks: W <= 32 at BM = 128 -> <= 204 pixels

template <int BM, int BN, int NWM = 2, int NWN = 2>
int launch_patch(GemmParams& P, const PatchGeom& G, hipStream_t s) {
  P.tiles_m = P.ga.n * G.rbs;
  P.tiles_n = vqa::cdiv(P.n, BN);
  const dim3 grid(P.tiles_m * P.tiles_n);
  if (G.chunks == 1) {
    if (G.npix > PMAX_SB) return vqa::fail(VQA_ERR_INVALID, "vqa_gemm(a_conv=2): patch of %d pixels > %d", G.npix, PMAX_SB);
    // one chunk: 2 B stages keep the block small (3 blocks / CU at BN = 64; measured 29.7 vs
    // 37.5 us at 3 stages for the layer1 3x3 conv, 44.6 us for the implicit-im2col path)
    hipLaunchKernelGGL((conv_patch_kernel<BM, BN, NWM, NWN, PMAX_SB, false, 2>), grid, dim3(64 * NWM * NWN), 0, s, P, G);
  } else {
    if (G.npix > PMAX_DB) return vqa::fail(VQA_ERR_INVALID, "vqa_gemm(a_conv=2): patch of %d pixels > %d", G.npix, PMAX_DB);
    hipLaunchKernelGGL((conv_patch_kernel<BM, BN, NWM, NWN, PMAX_DB, true, 3>), grid, dim3(64 * NWM * NWN), 0, s, P, G);
  }
  return vqa::check_launch("vqa_gemm(a_conv=2)");
}

}  // namespace

// does the (R + 2) x (W + 2) input patch of a bm-row tile fit the kernel's LDS patch buffer?
static bool patch_fits(const vqa_conv_geom& g, int bm) {
  const int R = bm / g.w < g.h ? bm / g.w : g.h;
  if (R < 1) return false;
  return (R + 2) * (g.w + 2) <= (g.c == 64 ? PMAX_SB : PMAX_DB);
}

// called by vqa_gemm for a_conv == 2 (gemm.hip has validated the descriptor and filled P)
static int conv_patch_dispatch(GemmParams& P, int config, hipStream_t s) {
  const vqa_conv_geom& g = P.ga;
  VQA_REQUIRE(g.kh == 3 && g.kw == 3 && g.stride == 1 && g.pad == 1 && g.oh == g.h && g.ow == g.w,
              "vqa_gemm(a_conv=2): a 3x3 / stride-1 / pad-1 convolution is required");
  VQA_REQUIRE(g.c % 64 == 0 && P.k == 9 * g.c && P.m == g.n * g.h * g.w, "vqa_gemm(a_conv=2): C %% 64, K = 9C, M = NHW");
  VQA_REQUIRE(P.splitk <= 1 && P.alpha == 1.f, "vqa_gemm(a_conv=2): no split-K, alpha = 1");
  int bm = (config == 19 || config == 20) ? 64 : 128;
  const int bn = (config == 18 || config == 20 || config == 25) ? 128 : 64;
  // a 128-row tile whose input patch exceeds the LDS buffer (e.g. C >= 128 at W 40-42 or 51-64,
  // where R = 128 / W leaves (R + 2)(W + 2) > PMAX_DB) runs as the 64-row tile: the tile
  // configs give the same bits, so this changes speed only
  if (bm == 128 && !patch_fits(g, 128)) bm = 64;
  VQA_REQUIRE(patch_fits(g, bm), "vqa_gemm(a_conv=2): no patch tile fits W = %d, C = %d", g.w, g.c);
  PatchGeom G;
  G.R = bm / g.w < g.h ? bm / g.w : g.h;
  G.rbs = vqa::cdiv(g.h, G.R);
  G.npix = (G.R + 2) * (g.w + 2);
  G.pins = vqa::cdiv(G.npix, 8);
  G.chunks = g.c / 64;
  G.ppart = vqa::cdiv(G.pins, 10 - 3);          // double-buffered: parts on taps S-1..8 at S = 3 stages
  // config 25: 8 waves -- 4 x 2 on the 128 x 128 tile (the layer2 / layer3 3x3 convs: 31.8 vs
  // 36.6 us at 14 x 14 x 256, 35.7 vs 38.5 at 28 x 28 x 128, profiles/r05_conv_patch_micro.txt),
  // 2 x 4 when the patch needs the 64-row tile
  if (config == 25) return bm == 128 ? launch_patch<128, 128, 4, 2>(P, G, s) : launch_patch<64, 128, 2, 4>(P, G, s);
  if (bm == 128 && bn == 64) return launch_patch<128, 64>(P, G, s);
  if (bm == 128) return launch_patch<128, 128>(P, G, s);
  if (bn == 64) return launch_patch<64, 64>(P, G, s);
  return launch_patch<64, 128>(P, G, s);
}
