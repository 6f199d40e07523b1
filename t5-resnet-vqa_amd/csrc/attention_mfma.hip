// Attention kernels over the MFMA bodies of attention_mfma.h (one wave per (batch, head)),
// the long-sequence forward, and their host-side dispatch.
#include "attention_mfma.h"

namespace {

template <int DH, int NT>
__global__ __launch_bounds__(64 * wpb_for(NT)) void attn_fwd_mfma(AttnM P) {
  constexpr int WPB = wpb_for(NT);
  __shared__ __attribute__((aligned(16))) char smem[WPB * 32 * NT * Geo<DH>::ROWB];
  attn_fwd_body<DH, NT>(P, blockIdx.x * WPB + (threadIdx.x >> 6), smem);
}

template <int DH, int NT>
__global__ __launch_bounds__(64 * wpb_for(NT)) void attn_bwd_mfma(AttnM P) {
  constexpr int WPB = wpb_for(NT);
  __shared__ __attribute__((aligned(16))) char smem[WPB * BwdLds<DH, NT>::PER_WAVE];
  attn_bwd_body<DH, NT>(P, blockIdx.x * WPB + (threadIdx.x >> 6), smem);
}

// ------------------------------------------------------------------ long forward
// ViT-base self-attention (BASELINE config 4: vision_model of VitVQAModel, run under
// no_grad, vit_vqa_model.py:183-186; HF ViTSelfAttention: softmax(QK^T / sqrt(64)) V,
// 197 tokens, no mask, no dropout): forward only, any lq, lk <= 1024.  One wave per
// (batch, head, 32-query block); the keys stream through in 32-key tiles with an
// online softmax (running max m and sum z per query, the O^T accumulators rescaled by
// exp(m_old - m_new)), so nothing of size lk is kept.  Same MFMA layouts as above:
// S^T tile in X layout (lane = query), O^T = V^T P^T with V through an LDS image.
template <int DH>
__global__ __launch_bounds__(64) void attn_fwd_long(AttnM P) {
  using G = Geo<DH>;
  __shared__ __attribute__((aligned(16))) char smem[32 * G::ROWB];
  const int l = threadIdx.x, h5 = l >> 5, l31 = l & 31;
  const int lq = P.lq, lk = P.lk;
  const int qblocks = (lq + 31) >> 5;
  const int pair = blockIdx.x / qblocks, qb = blockIdx.x - pair * qblocks;
  const int b = pair / P.heads, hh = pair - b * P.heads;
  const int nq = min(32, lq - 32 * qb);
  lds_char* vimg = (lds_char*)smem;
  const bf16_t* Q = P.q + ((long)b * lq + 32 * qb) * P.ldq + hh * DH;
  const bf16_t* K = P.k + (long)b * lk * P.ldk + hh * DH;
  const bf16_t* V = P.v + (long)b * lk * P.ldv + hh * DH;
  bf16x8_t qf[G::KS];
#pragma unroll
  for (int s = 0; s < G::KS; ++s) qf[s] = ld_frag(Q + (long)min(l31, nq - 1) * P.ldq + 16 * s + 8 * h5, l31 < nq);
  f32x16_t oa[G::ET];
#pragma unroll
  for (int et = 0; et < G::ET; ++et)
#pragma unroll
    for (int e = 0; e < 16; ++e) oa[et][e] = 0.f;
  float m = -INFINITY, z = 0.f;
  const int ntiles = (lk + 31) >> 5;
  for (int t = 0; t < ntiles; ++t) {
    const int nk = min(32, lk - 32 * t);
    const bf16_t* Kt = K + (long)32 * t * P.ldk;
    bf16x8_t kf[G::KS];
#pragma unroll
    for (int s = 0; s < G::KS; ++s) kf[s] = ld_frag(Kt + (long)min(l31, nk - 1) * P.ldk + 16 * s + 8 * h5, l31 < nk);
    __syncthreads();                                             // the previous tile's V reads are done
    stage_img<DH, 32, G::ROWB>(vimg, V + (long)32 * t * P.ldv, P.ldv, nk);
    f32x16_t sa;
#pragma unroll
    for (int e = 0; e < 16; ++e) sa[e] = 0.f;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) sa = mfma(kf[s], qf[s], sa);
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = (r & 3) + 8 * (r >> 2) + 4 * h5;
      const float v = key < nk ? sa[r] * P.scale : -INFINITY;
      sa[r] = v;
      mt = fmaxf(mt, v);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float corr = __expf(m - mn);                           // 0 on the first tile (m = -inf)
    float zt = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = sa[r] == -INFINITY ? 0.f : __expf(sa[r] - mn);
      sa[r] = e;
      zt += e;
    }
    zt += __shfl_xor(zt, 32, 64);
    z = z * corr + zt;
    m = mn;
    __syncthreads();                                             // V image complete
#pragma unroll
    for (int et = 0; et < G::ET; ++et) {
#pragma unroll
      for (int e = 0; e < 16; ++e) oa[et][e] *= corr;
#pragma unroll
      for (int s = 0; s < 2; ++s) oa[et] = mfma(tr_frag<G::ROWB>(vimg, s, et * 32), regs_frag(sa, s), oa[et]);
    }
  }
  const float iz = 1.f / z;
#pragma unroll
  for (int et = 0; et < G::ET; ++et)
    store_tr(P.o + ((long)b * lq + 32 * qb) * P.ldo + hh * DH, P.ldo, l31, l31 < nq, et * 32, oa[et], iz);
}

}  // namespace

// host side: the long forward (vqa_attn_fwd for lq > 32 or lk > 64; no P, bias, mask, dropout)
bool vqa_attn_long_ok(const vqa_attn_desc* d) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return d->lq >= 1 && d->lk >= 1 && d->lk <= 1024 && (d->dh == 64 || d->dh == 96) && !d->p && !d->bias &&
         !d->key_mask && !(d->drop.p > 0.f && d->drop.rng) && d->ldq % 8 == 0 && d->ldk % 8 == 0 &&
         d->ldv % 8 == 0 && al16(d->q) && al16(d->k) && al16(d->v) && d->o && d->ldo % 4 == 0 &&
         ((uintptr_t)d->o & 7) == 0;
}

int vqa_attn_fwd_long(const vqa_attn_desc* d, hipStream_t s) {
  AttnM M;
  M.q = (const bf16_t*)d->q; M.k = (const bf16_t*)d->k; M.v = (const bf16_t*)d->v;
  M.ldq = d->ldq; M.ldk = d->ldk; M.ldv = d->ldv;
  M.o = (bf16_t*)d->o; M.ldo = d->ldo; M.p = nullptr; M.bias = nullptr; M.mask = nullptr;
  M.pairs = d->batch * d->heads; M.heads = d->heads; M.lq = d->lq; M.lk = d->lk; M.scale = d->scale;
  const long grid = (long)M.pairs * ((d->lq + 31) / 32);
  VQA_REQUIRE(grid > 0 && grid < (1l << 31), "vqa_attn_fwd (long): bad grid");
  if (d->dh == 64) hipLaunchKernelGGL((attn_fwd_long<64>), dim3((unsigned)grid), dim3(64), 0, s, M);
  else hipLaunchKernelGGL((attn_fwd_long<96>), dim3((unsigned)grid), dim3(64), 0, s, M);
  return vqa::check_launch("vqa_attn_fwd (long)");
}

// host side: called by vqa_attn_fwd / vqa_attn_bwd (attention.hip) when the shape fits
bool vqa_attn_mfma_ok(const vqa_attn_desc* d) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return d->lq >= 1 && d->lq <= 32 && d->lk >= 1 && d->lk <= 32 * MAX_NT &&
         (d->dh == 64 || d->dh == 96 || d->dh == 128) && (d->lk <= 64 || !d->key_mask) &&
         d->ldq % 8 == 0 && d->ldk % 8 == 0 && d->ldv % 8 == 0 && al16(d->q) && al16(d->k) && al16(d->v) &&
         (!d->o || (d->ldo % 4 == 0 && ((uintptr_t)d->o & 7) == 0)) &&
         (!d->dout || (d->lddo % 8 == 0 && al16(d->dout))) &&
         (!d->dq || (d->lddq % 4 == 0 && ((uintptr_t)d->dq & 7) == 0)) &&
         (!d->dk || (d->lddk % 4 == 0 && ((uintptr_t)d->dk & 7) == 0)) &&
         (!d->dv || (d->lddv % 4 == 0 && ((uintptr_t)d->dv & 7) == 0));
}


template <int DH, int NT>
int launch_fwd(AttnM& M, hipStream_t s) {
  constexpr int W = wpb_for(NT);
  hipLaunchKernelGGL((attn_fwd_mfma<DH, NT>), dim3(vqa::cdiv(M.pairs, W)), dim3(64 * W), 0, s, M);
  return vqa::check_launch("vqa_attn_fwd (mfma)");
}
template <int DH, int NT>
int launch_bwd(AttnM& M, hipStream_t s) {
  constexpr int W = wpb_for(NT);
  hipLaunchKernelGGL((attn_bwd_mfma<DH, NT>), dim3(vqa::cdiv(M.pairs, W)), dim3(64 * W), 0, s, M);
  return vqa::check_launch("vqa_attn_bwd (mfma)");
}
template <int DH>
int dispatch_nt(AttnM& M, int nt, bool bwd, hipStream_t s) {
  switch (nt) {
    case 1: return bwd ? launch_bwd<DH, 1>(M, s) : launch_fwd<DH, 1>(M, s);
    case 2: return bwd ? launch_bwd<DH, 2>(M, s) : launch_fwd<DH, 2>(M, s);
    case 3: return bwd ? launch_bwd<DH, 3>(M, s) : launch_fwd<DH, 3>(M, s);
    case 4: return bwd ? launch_bwd<DH, 4>(M, s) : launch_fwd<DH, 4>(M, s);
    default: return bwd ? launch_bwd<DH, 5>(M, s) : launch_fwd<DH, 5>(M, s);
  }
}
int dispatch_dh(const vqa_attn_desc* d, bool bwd, hipStream_t s) {
  AttnM M;
  fillm(M, d);
  const int nt = (d->lk + 31) / 32;
  if (d->dh == 64) return dispatch_nt<64>(M, nt, bwd, s);
  if (d->dh == 96) return dispatch_nt<96>(M, nt, bwd, s);
  return dispatch_nt<128>(M, nt, bwd, s);
}

int vqa_attn_fwd_mfma(const vqa_attn_desc* d, hipStream_t s) { return dispatch_dh(d, false, s); }

int vqa_attn_bwd_mfma(const vqa_attn_desc* d, hipStream_t s) { return dispatch_dh(d, true, s); }
