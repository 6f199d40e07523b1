// The AdamW-amsgrad element update (torch.optim.AdamW(amsgrad=True) with the trainer's groups,
// faster_rcnn_vqa_trainer.py:231-267), shared by the fused optimiser pass (optim.hip) and the
// embedding gather that reads a deferred update's result on the fly (elementwise.hip,
// vqa_embedding_fwd_pending): both run this one function, so the gathered rows equal the rows
// the deferred pass writes later, bit for bit.
#pragma once
#include "common.h"

namespace {

struct AdamArgs {
  float* p; const float* g; float* m; float* v; float* vm; bf16_t* p16;
  long n4;
  int ngroups; long gend4[VQA_MAX_GROUPS]; float glr[VQA_MAX_GROUPS];
  float b1, b2, eps, wd, gscale;
  const float* st;
};

inline int adam_args(const vqa_adamw_desc* d, AdamArgs& A) {
  VQA_REQUIRE(d && d->param && d->grad && d->exp_avg && d->exp_avg_sq && d->max_exp_avg_sq && d->state,
              "vqa_adamw: null argument");
  VQA_REQUIRE(d->n % 4 == 0 && d->ngroups >= 1 && d->ngroups <= VQA_MAX_GROUPS, "vqa_adamw: bad sizes");
  A.p = d->param; A.g = d->grad; A.m = d->exp_avg; A.v = d->exp_avg_sq; A.vm = d->max_exp_avg_sq;
  A.p16 = (bf16_t*)d->param16;
  A.n4 = d->n / 4;
  A.ngroups = d->ngroups;
  for (int i = 0; i < VQA_MAX_GROUPS; ++i) {
    VQA_REQUIRE(i >= d->ngroups || d->group_end[i] % 4 == 0, "vqa_adamw: group ends must be multiples of 4");
    A.gend4[i] = i < d->ngroups ? d->group_end[i] / 4 : A.n4;
    A.glr[i] = i < d->ngroups ? d->group_lr[i] : 0.f;
  }
  A.b1 = d->beta1; A.b2 = d->beta2; A.eps = d->eps; A.wd = d->weight_decay; A.gscale = d->grad_scale;
  A.st = d->state;
  return VQA_OK;
}

// float4 i of the range: p, m, v, vm updated in place from g, with the clip coefficient, LR
// schedule multiplier and bias corrections given (adamw_update4 reads them from the device state
// written by vqa_optim_finalize; the embedding table's row-split update, vqa_adamw_rows, computes
// them for the coming step itself)
__device__ __forceinline__ void adamw_update4_with(const AdamArgs& A, long i, f32x4_t& p, const f32x4_t g4,
                                                   f32x4_t& m, f32x4_t& v, f32x4_t& vm, const float coef,
                                                   const float lam, const float bc1, const float bc2s) {
  // no FMA contraction: the kernels that inline this must round every operation alike
#pragma clang fp contract(off)
  const float gmul = A.gscale * coef;
  const float omb1 = 1.f - A.b1, omb2 = 1.f - A.b2;
  int gi = 0;
#pragma unroll
  for (int k = 0; k < VQA_MAX_GROUPS - 1; ++k) gi += (k < A.ngroups - 1 && i >= A.gend4[k]) ? 1 : 0;
  const float lr = A.glr[gi] * lam;
  const float decay = 1.f - lr * A.wd, step_size = lr / bc1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gr = g4[j] * gmul;
    p[j] *= decay;                                      // decoupled weight decay
    m[j] = m[j] + omb1 * (gr - m[j]);                   // exp_avg.lerp_(grad, 1-beta1)
    v[j] = v[j] * A.b2 + omb2 * gr * gr;                // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    vm[j] = fmaxf(vm[j], v[j]);                         // amsgrad running max
    const float denom = sqrtf(vm[j]) / bc2s + A.eps;
    p[j] = p[j] - step_size * (m[j] / denom);
  }
}

__device__ __forceinline__ void adamw_update4(const AdamArgs& A, long i, f32x4_t& p, const f32x4_t g4, f32x4_t& m,
                                              f32x4_t& v, f32x4_t& vm) {
  adamw_update4_with(A, i, p, g4, m, v, vm, A.st[VQA_ST_CLIP_COEF], A.st[VQA_ST_LR_SCALE], A.st[VQA_ST_BC1],
                     A.st[VQA_ST_BC2_SQRT]);
}

}  // namespace
