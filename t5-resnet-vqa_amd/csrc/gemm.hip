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
#include "gemm_body.h"

namespace {

// GELU / tanh epilogues (vqa_gemm_desc.relu 2 / 3: the ViT intermediate and pooler of
// config 4) in ONE tile config (64x128, 2 stages, k-contiguous A and B = X W^T), so the
// extra epilogue code is not instantiated into every config (a 256x256 variant measured
// 1 ms slower per config-4 step: 600 tiles leave 2.3 rounds per CU)
template <int BM, int BN, int NWM, int NWN>
__global__ __launch_bounds__(64 * NWM * NWN) void gemm_ext_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<BM, BN, 2>::LDS];
  gemm_body<BM, BN, 2, NWM, NWN, true, true, false, false, true>(P, blockIdx.x, smem);
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

// config: 0 = auto; 1 = 128x128 (3 stages); 2 = 128x64 (4); 3 = 64x64 (4); 4 = 64x64 (2);
//         5 = 64x64 (3); 6 = 128x64 (2); 7 = 64x128 (2); 8 = 128x128 (2)  -- 4 waves (2x2);
//         9 = 256x128 (2, 8 waves 4x2); 10 = 128x256 (2, 8 waves 2x4); 11 = 256x256 (2, 8 waves 2x4);
//         12 = 256x128 (3, 8 waves 4x2); 13 = 64x192 (2); 14 = 128x192 (2); 15 = 64x192 (3);
//         16 = 128x192 (3) -- 4 waves, k-contiguous B only;
//         17..20 = the LDS-patch 3x3 convolution (a_conv = 2, conv_patch.inl): 128x64, 128x128,
//         64x64, 64x128; 21..23 = 64x64 / 64x128 / 128x64 with 128-deep k-tiles (4 waves);
//         24 = 64x128 with 128-deep k-tiles on 8 waves (2x4); 26 / 27 / 28 = 64x128 / 128x64 /
//         64x64 for k <= 64 (one k-tile, single-stage ring: 4 / 4 / 5 workgroups per CU).
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
    case 21: case 22: case 23: case 24:
      // 128-deep k-tiles: twice the bytes per ring slot and per barrier (the per-k-tile fixed
      // cost of the L2 -> LDS fill is amortised over 32-48 KB instead of 16-24 KB); plain
      // (non-gathered) operands, no split-K.  24: config 22's 64x128 tile on 8 waves (2x4, each
      // 32x32): twice the waves issuing the ring's DMA pieces (r04 stamps: 7 % faster on the
      // 2048 x 2304 x 768 q|k|v projection)
      if constexpr (!GA && !GB) {
        if (config == 21) return launch<64, 64, 2, 2, 2, AKC, BKC, GA, GB, 128>(P, batch, s);
        if (config == 22) return launch<64, 128, 2, 2, 2, AKC, BKC, GA, GB, 128>(P, batch, s);
        if (config == 24) return launch<64, 128, 2, 2, 4, AKC, BKC, GA, GB, 128>(P, batch, s);
        return launch<128, 64, 2, 2, 2, AKC, BKC, GA, GB, 128>(P, batch, s);
      } else {
        return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: tile config %d takes no implicit-im2col operand", config);
      }
    case 26: case 27: case 28:
      // one k-tile in a single-stage ring (gemm_k1_kernel): k <= 64, plain operands
      if constexpr (!GA && !GB) {
        if (config == 26) return launch_k1<64, 128, 4, AKC, BKC, GA, GB>(P, batch, s);
        if (config == 27) return launch_k1<128, 64, 4, AKC, BKC, GA, GB>(P, batch, s);
        return launch_k1<64, 64, 5, AKC, BKC, GA, GB>(P, batch, s);
      } else {
        return vqa::fail(VQA_ERR_INVALID, "vqa_gemm: tile config %d takes no implicit-im2col operand", config);
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
                                                 {64, 192},  {128, 192}, {128, 64}, {128, 128}, {64, 64},
                                                 {64, 128},  {64, 64},   {64, 128}, {128, 64}, {64, 128},
                                                 {128, 128}, {64, 128},  {128, 64}, {64, 64}};
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

#ifndef VQA_GEMM_MICRO
#include "conv_patch.inl"
#endif

namespace {
// auto tile for the patch convolution: 64-column tiles for 64 output channels, 64-row tiles
// for the 7 / 8-wide maps (a 128-row tile would be mostly padding)
int patch_auto_config(const vqa_gemm_desc* d) {
  const int bm64 = d->ga.w <= 8;
  return d->n <= 64 ? (bm64 ? 19 : 17) : (bm64 ? 20 : 18);
}
}  // namespace

extern "C" int vqa_gemm_select(const vqa_gemm_desc* d) {
  if (!d) return 0;
  if (d->config) return d->config;
  return d->a_conv == 2 ? patch_auto_config(d) : auto_config(d->m, d->n, d->k, d->batch);
}

extern "C" long long vqa_gemm_workspace_bytes(const vqa_gemm_desc* d) {
  if (!d || d->splitk <= 1 || d->a_conv == 2) return 0;
  int bm, bn, kper;
  tile_of(vqa_gemm_select(d), bm, bn);
  const int S = effective_splitk(d->fp8 ? d->k / 2 : d->k, d->splitk, &kper);   // fp8: k in 2-byte units
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
  VQA_REQUIRE(d->relu >= 0 && d->relu <= 3, "vqa_gemm: activation must be 0..3");
  VQA_REQUIRE(d->relu <= 1 || (!(d->drop.p > 0.f && d->drop.rng) && !d->mask16),
              "vqa_gemm: GELU / tanh epilogues take no dropout or mask (act(k*t) != k*act(t))");
  P.alpha = d->alpha; P.beta = d->beta; P.relu = d->relu;
  P.ga = d->ga; P.gb = d->gb;
  P.sa = d->stride_a; P.sb = d->stride_b; P.sc32 = d->stride_c32; P.sc16 = d->stride_c16; P.sres = d->stride_res;
  P.drop = d->drop;
  P.sbias = d->stride_bias;
  P.dsite = d->drop_site_stride;
  P.qsa = P.qsb = nullptr;
  P.sqa = P.sqb = 0;
  if (d->fp8) {
    // e4m3 operands: bytes, staged by the bf16 loaders as 2-byte units (128 fp8 per 64-unit k-tile)
    VQA_REQUIRE(!d->a_trans && !d->b_trans && !d->a_conv && !d->b_conv && d->relu <= 1,
                "vqa_gemm(fp8): k-contiguous A and B, no conv operand, ReLU at most");
    VQA_REQUIRE(d->k % 16 == 0 && d->lda % 16 == 0 && d->ldb % 16 == 0 && d->stride_a % 2 == 0 &&
                    d->stride_b % 2 == 0 && d->n % 4 == 0,
                "vqa_gemm(fp8): k, lda, ldb multiples of 16 bytes, even strides, n %% 4 == 0");
    VQA_REQUIRE(d->scale_a && d->scale_b && aligned16(d->scale_b) && d->stride_scale_b % 4 == 0,
                "vqa_gemm(fp8): row scales of A and B (scale_b 16-byte aligned)");
    P.k = d->k / 2;
    P.lda = d->lda / 2;
    P.ldb = d->ldb / 2;
    P.sa = d->stride_a / 2;
    P.sb = d->stride_b / 2;
    P.qsa = d->scale_a;
    P.qsb = d->scale_b;
    P.sqa = d->stride_scale_a;
    P.sqb = d->stride_scale_b;
  }
  P.splitk = 1;
  P.kper = 0;
  P.slab = nullptr;
  P.cnt = nullptr;
  VQA_REQUIRE(d->splitk >= 0 && d->splitk <= 64, "vqa_gemm: splitk must be 0..64");
  if (d->splitk > 1) {
    int kper;
    const int S = effective_splitk(P.k, d->splitk, &kper);
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

#ifndef VQA_GEMM_MICRO
int vqa_gemm_fp8_dispatch(void* P, int batch, int config, hipStream_t s);   // gemm_fp8.hip

extern "C" int vqa_gemm(const vqa_gemm_desc* d, hipStream_t stream) {
  GemmParams P;
  if (int rc = prepare(d, P)) return rc;
  const int batch = d->batch, cfg = d->config;
  if (d->fp8) return vqa_gemm_fp8_dispatch(&P, batch, cfg, stream);
  const bool akc = !d->a_trans, bkc = !d->b_trans;
  const bool patch_cfg = (cfg >= VQA_GEMM_PATCH_FIRST && cfg <= VQA_GEMM_PATCH_LAST) || cfg == VQA_GEMM_PATCH_WIDE;
  if (d->a_conv == 2) {                                   // LDS-patch 3x3 convolution (conv_patch.inl)
    VQA_REQUIRE(akc && bkc && !d->b_conv && batch == 1, "vqa_gemm(a_conv=2): k-contiguous B, batch 1");
    VQA_REQUIRE(cfg == 0 || patch_cfg, "vqa_gemm(a_conv=2): tile config %d is not a patch config (%d..%d)", cfg,
                VQA_GEMM_PATCH_FIRST, VQA_GEMM_PATCH_LAST);
    return conv_patch_dispatch(P, vqa_gemm_select(d), stream);
  }
  VQA_REQUIRE(!patch_cfg, "vqa_gemm: tile config %d is for a_conv = 2 only", cfg);
  if (d->relu >= 2) {                                     // GELU / tanh: gemm_ext_kernel only
    VQA_REQUIRE(akc && bkc && !d->a_conv && !d->b_conv && P.splitk <= 1,
                "vqa_gemm: GELU / tanh epilogues need k-contiguous A and B, no conv operand, no split-K");
    P.tiles_m = vqa::cdiv(P.m, 64);
    P.tiles_n = vqa::cdiv(P.n, 128);
    hipLaunchKernelGGL((gemm_ext_kernel<64, 128, 2, 2>), dim3(P.tiles_m * P.tiles_n, 1, batch), dim3(256), 0, stream,
                       P);
    return vqa::check_launch("vqa_gemm (ext epilogue)");
  }
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
#endif  // VQA_GEMM_MICRO
