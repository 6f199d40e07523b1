// GEMM + attention in one launch: the T5 self-attention's projection and attention, with the
// attention computed by the workgroup that produced its operands (no kernel boundary, no
// second launch reading them back).
//
//   forward  (TF modeling_t5.py:498-560, T5Attention.forward): one tile = 64 token rows (64 / L
//            samples) x the 3 x 64 columns of ONE head's q, k and v (GemmParams.hd, the B rows
//            gathered head by head from the stacked [q|k|v] weight); the epilogue writes them to
//            the usual [T, 3D] buffer, then waves 0 .. 64/L - 1 run the attention of (sample,
//            head) pairs of the tile (attention_mfma.h attn_fwd_body: rel-bias, key mask,
//            softmax, saved P, dropout, O).
//   backward (the o projection's input gradient + the attention backward): one tile = 64 rows
//            x the 64 columns of ONE head of dContext = dY Wo; the epilogue writes them, then
//            the attention backward of the tile's (sample, head) pairs (attn_bwd_body: dQ, dK,
//            dV, per-sample dS for the rel-bias gradient).
// The GEMM tile and the attention body are the library's own code, so the results are the
// unfused launches' bit for bit (tests/test_kernels_gpu.py).  Everything the attention reads
// from the GEMM was written by the same workgroup: a workgroup barrier orders it.
#include "gemm_body.h"
#include "attention_mfma.h"

int vqa_gemm_prepare(const vqa_gemm_desc* d, void* P);   // gemm.hip
bool vqa_attn_mfma_ok(const vqa_attn_desc* d);          // attention_mfma.hip

namespace {

constexpr int FT = 64;                                   // token rows per tile
constexpr int FDH = 64;                                  // head dim (T5: 12 x 64)
constexpr int FL = 32;                                   // tokens per sample (lq = lk)
constexpr int FUNITS = FT / FL;                          // (sample, head) pairs per tile

// forward tile: 64 x 192, 2 stages, 4 waves (config 13's shape), k-contiguous A and B
constexpr int FWD_LDS = TileCfg<FT, 3 * FDH, 2>::LDS;
static_assert(4 * 32 * Geo<FDH>::ROWB <= FWD_LDS, "attention V images must fit the GEMM ring");

__global__ __launch_bounds__(256) void qkv_attn_fwd_kernel(GemmParams P, AttnM A) {
  __shared__ __attribute__((aligned(1024))) char smem[FWD_LDS];
  gemm_body<FT, 3 * FDH, 2, 2, 2, true, true, false, false>(P, blockIdx.x, smem);
  int tile, slice, tm, tn;
  tile_coords<3 * FDH, false>(P, blockIdx.x, tile, slice, tm, tn);
  __threadfence_block();
  __syncthreads();                                       // q|k|v of the tile stored; the ring is free
  const int w = threadIdx.x >> 6;
  const int pair = w < FUNITS ? (tm * FUNITS + w) * A.heads + tn : A.pairs;   // others: not live
  attn_fwd_body<FDH, 1>(A, pair, smem);
}

// backward tile: 64 x 64 with 128-deep k-tiles, 2 stages (config 21's shape): dContext = dY Wo
// (A = dY k-contiguous, B = Wo read n-contiguous)
constexpr int BWD_LDS = TileCfg<FT, FDH, 2, 128>::LDS;
static_assert(FUNITS * BwdLds<FDH, 1>::PER_WAVE <= BWD_LDS, "attention backward images must fit the GEMM ring");

__global__ __launch_bounds__(256) void odx_attn_bwd_kernel(GemmParams P, AttnM A) {
  __shared__ __attribute__((aligned(1024))) char smem[BWD_LDS];
  gemm_body<FT, FDH, 2, 2, 2, true, false, false, false, false, 128>(P, blockIdx.x, smem);
  int tile, slice, tm, tn;
  tile_coords<FDH, false>(P, blockIdx.x, tile, slice, tm, tn);
  __threadfence_block();
  __syncthreads();                                       // dContext of the tile stored; the ring is free
  const int w = threadIdx.x >> 6;
  if (w < FUNITS) {
    attn_bwd_body<FDH, 1>(A, (tm * FUNITS + w) * A.heads + tn, smem);
  } else {
    __syncthreads();                                     // the body's one barrier
  }
}

}  // namespace

extern "C" int vqa_gemm_attn(const vqa_gemm_desc* g, const vqa_attn_desc* a, int backward, hipStream_t s) {
  VQA_REQUIRE(g && a, "vqa_gemm_attn: null descriptor");
  GemmParams P;
  if (int rc = vqa_gemm_prepare(g, &P)) return rc;
  const int D = a->heads * a->dh;
  VQA_REQUIRE(a->dh == FDH && a->lq == FL && a->lk == FL && g->batch == 1 && P.splitk == 1 && !g->fp8 &&
                  !g->a_conv && !g->b_conv && !g->a_trans && g->m == a->batch * FL && g->m % FT == 0 && g->c16 &&
                  !g->c32 && P.vec,
              "vqa_gemm_attn: T5 shapes only (dh %d, lq = lk = %d, m = batch * lq multiple of %d, bf16 output)", FDH,
              FL, FT);
  VQA_REQUIRE(vqa_attn_mfma_ok(a), "vqa_gemm_attn: attention descriptor outside the MFMA kernel's shapes");
  AttnM A;
  fillm(A, a);
  const bf16_t* c16 = (const bf16_t*)g->c16;
  if (!backward) {
    // q|k|v projection [T, 3D] (k-contiguous weight [3D, D]) feeding the attention in place
    VQA_REQUIRE(!g->b_trans && g->n == 3 * D && g->ldc16 == 3 * D && a->q == c16 && a->k == c16 + D &&
                    a->v == c16 + 2 * D && a->ldq == 3 * D && a->ldk == 3 * D && a->ldv == 3 * D && a->o,
                "vqa_gemm_attn(forward): the attention must read q, k, v from the projection's output");
    P.hd = FDH;
    P.tiles_m = g->m / FT;
    P.tiles_n = a->heads;
    hipLaunchKernelGGL(qkv_attn_fwd_kernel, dim3(P.tiles_m * P.tiles_n), dim3(256), 0, s, P, A);
    return vqa::check_launch("vqa_gemm_attn (forward)");
  }
  // dContext = dY Wo (Wo [D, D] read n-contiguous) feeding the attention backward as dO
  VQA_REQUIRE(g->b_trans && g->n == D && a->dout == c16 && a->lddo == g->ldc16 && a->dq && a->dk && a->dv && a->p,
              "vqa_gemm_attn(backward): the attention backward must read dO from the GEMM's output");
  P.tiles_m = g->m / FT;
  P.tiles_n = a->heads;
  hipLaunchKernelGGL(odx_attn_bwd_kernel, dim3(P.tiles_m * P.tiles_n), dim3(256), 0, s, P, A);
  return vqa::check_launch("vqa_gemm_attn (backward)");
}
