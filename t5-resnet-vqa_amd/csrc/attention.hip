// Fused multi-head attention core, forward and backward, for the two short
// attention shapes of the step (Lq, Lk <= 64):
//   SGA  MHAtt.att   softmax(QK^T/sqrt(96)) V, 8 heads x 96     multi_head_vision_text_attn.py:73-86
//   T5   attention   softmax(QK^T + relbias + mask) V, 12 x 64  TF/models/t5/modeling_t5.py:144-173
// One workgroup per (batch, head).  Q/K/V/dO are staged in LDS as packed bf16
// pairs ([rows][D/2+1] dwords, conflict-free for both the row-dot and the
// column-axpy access), scores/probabilities in fp32, one wave per softmax row.
// The whole (b,h) problem is at most 64x64x96, so everything stays on-chip; Q,
// K and V are read straight out of the fused QKV projection output through
// row strides (no head transposes in HBM).
#include "common.h"

namespace {

constexpr float MASK_MIN = -3.4028234663852886e38f;     // torch.finfo(float32).min (additive key mask)

struct AttnP {
  const bf16_t *q, *k, *v; long ldq, ldk, ldv;
  bf16_t* o; long ldo;
  float* p;
  const float* bias;
  const long long* mask;
  int heads, lq, lk, dh;
  float scale;
  const bf16_t* dout; long lddo;
  bf16_t *dq, *dk, *dv; long lddq, lddk, lddv;
  float* dbias;
  vqa_dropout drop;        // attention-probability dropout (MHAtt.att :84, T5 :168)
};

__device__ __forceinline__ float2 unpack(uint32_t u) {
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}
__device__ __forceinline__ uint32_t pack(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// stage rows [n][dh] bf16 (row stride ld, head offset) into LDS [n][dh/2+1] dwords
__device__ __forceinline__ void stage(uint32_t* dst, const bf16_t* src, long ld, int n, int dh) {
  const int w2 = dh / 2, st = w2 + 1, c8 = dh / 8;
  for (int idx = threadIdx.x; idx < n * c8; idx += blockDim.x) {
    const int r = idx / c8, c = idx - r * c8;
    const uint4 u = *reinterpret_cast<const uint4*>(src + (long)r * ld + c * 8);
    uint32_t* d = dst + r * st + c * 4;
    d[0] = u.x; d[1] = u.y; d[2] = u.z; d[3] = u.w;
  }
}

__device__ __forceinline__ float rowdot(const uint32_t* a, const uint32_t* b, int w2) {
  float s0 = 0.f, s1 = 0.f;
  for (int e = 0; e < w2; ++e) {
    const float2 x = unpack(a[e]), y = unpack(b[e]);
    s0 = fmaf(x.x, y.x, s0);
    s1 = fmaf(x.y, y.y, s1);
  }
  return s0 + s1;
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnP P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int b = blockIdx.x / P.heads, h = blockIdx.x - b * P.heads;
  const int lq = P.lq, lk = P.lk, dh = P.dh, w2 = dh / 2, st = w2 + 1, sst = lk + 1;
  uint32_t* Qs = sm;
  uint32_t* Ks = Qs + lq * st;
  uint32_t* Vs = Ks + lk * st;
  float* S = reinterpret_cast<float*>(Vs + lk * st);
  stage(Qs, P.q + (long)b * lq * P.ldq + h * dh, P.ldq, lq, dh);
  stage(Ks, P.k + (long)b * lk * P.ldk + h * dh, P.ldk, lk, dh);
  stage(Vs, P.v + (long)b * lk * P.ldv + h * dh, P.ldv, lk, dh);
  __syncthreads();
  for (int idx = threadIdx.x; idx < lq * lk; idx += blockDim.x) {
    const int i = idx / lk, j = idx - i * lk;
    float s = rowdot(Qs + i * st, Ks + j * st, w2) * P.scale;
    if (P.bias) s += P.bias[((long)h * lq + i) * lk + j];
    if (P.mask && P.mask[(long)b * lk + j] == 0 && !(P.bias && P.bias[((long)h * lq + i) * lk + j] <= 0.5f * MASK_MIN))
      s += MASK_MIN;                                   // one finfo.min per masked pair (see attention_mfma.hip)
    S[i * sst + j] = s;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const DropK dk = drop_init(P.drop);
  for (int i = wv; i < lq; i += 4) {
    const float s = l < lk ? S[i * sst + l] : -INFINITY;
    const float m = wave_max(s);
    const float e = l < lk ? __expf(s - m) : 0.f;
    const float z = wave_sum(e);
    const float pr = e / z;
    if (l < lk) {
      const long idx = (((long)b * P.heads + h) * lq + i) * lk + l;
      S[i * sst + l] = dk.on ? pr * drop_mul(dk, (uint32_t)idx) : pr;      // O uses dropout(P)
      if (P.p) P.p[idx] = pr;                                               // saved pre-dropout
    }
  }
  __syncthreads();
  // O[i][2e..2e+1] = sum_j P[i][j] V[j][2e..2e+1]
  for (int idx = threadIdx.x; idx < lq * w2; idx += blockDim.x) {
    const int i = idx / w2, e = idx - i * w2;
    float a0 = 0.f, a1 = 0.f;
    for (int j = 0; j < lk; ++j) {
      const float pr = S[i * sst + j];
      const float2 v = unpack(Vs[j * st + e]);
      a0 = fmaf(pr, v.x, a0);
      a1 = fmaf(pr, v.y, a1);
    }
    reinterpret_cast<uint32_t*>(P.o + ((long)b * lq + i) * P.ldo + h * dh)[e] = pack(a0, a1);
  }
}

__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnP P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int b = blockIdx.x / P.heads, h = blockIdx.x - b * P.heads;
  const int lq = P.lq, lk = P.lk, dh = P.dh, w2 = dh / 2, st = w2 + 1, sst = lk + 1;
  uint32_t* Qs = sm;
  uint32_t* Ks = Qs + lq * st;
  uint32_t* Vs = Ks + lk * st;
  uint32_t* Os = Vs + lk * st;                       // dO
  float* Ps = reinterpret_cast<float*>(Os + lq * st);
  float* dS = Ps + lq * sst;
  stage(Qs, P.q + (long)b * lq * P.ldq + h * dh, P.ldq, lq, dh);
  stage(Ks, P.k + (long)b * lk * P.ldk + h * dh, P.ldk, lk, dh);
  stage(Vs, P.v + (long)b * lk * P.ldv + h * dh, P.ldv, lk, dh);
  stage(Os, P.dout + (long)b * lq * P.lddo + h * dh, P.lddo, lq, dh);
  const float* Pg = P.p + ((long)b * P.heads + h) * lq * lk;
  for (int idx = threadIdx.x; idx < lq * lk; idx += blockDim.x) {
    const int i = idx / lk, j = idx - i * lk;
    Ps[i * sst + j] = Pg[idx];
  }
  __syncthreads();
  // dP = dO V^T
  for (int idx = threadIdx.x; idx < lq * lk; idx += blockDim.x) {
    const int i = idx / lk, j = idx - i * lk;
    dS[i * sst + j] = rowdot(Os + i * st, Vs + j * st, w2);
  }
  __syncthreads();
  // with dropout: dP = mask * dP(dropped);  dS = P (dP - sum_j P dP);  Ps <- dropout(P) for dV
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const DropK dk = drop_init(P.drop);
  for (int i = wv; i < lq; i += 4) {
    const long idx = (((long)b * P.heads + h) * lq + i) * lk + l;
    const float km = (dk.on && l < lk) ? drop_mul(dk, (uint32_t)idx) : 1.f;
    const float pr = l < lk ? Ps[i * sst + l] : 0.f;
    const float dp = l < lk ? dS[i * sst + l] * km : 0.f;
    const float di = wave_sum(pr * dp);
    if (l < lk) {
      const float ds = pr * (dp - di);
      dS[i * sst + l] = ds;
      if (dk.on) Ps[i * sst + l] = pr * km;
      if (P.dbias) P.dbias[idx] = ds;                                       // per-sample dS
    }
  }
  __syncthreads();
  // dQ = scale * dS K
  for (int idx = threadIdx.x; idx < lq * w2; idx += blockDim.x) {
    const int i = idx / w2, e = idx - i * w2;
    float a0 = 0.f, a1 = 0.f;
    for (int j = 0; j < lk; ++j) {
      const float d = dS[i * sst + j];
      const float2 kv = unpack(Ks[j * st + e]);
      a0 = fmaf(d, kv.x, a0);
      a1 = fmaf(d, kv.y, a1);
    }
    reinterpret_cast<uint32_t*>(P.dq + ((long)b * lq + i) * P.lddq + h * dh)[e] = pack(a0 * P.scale, a1 * P.scale);
  }
  // dK = scale * dS^T Q ; dV = dropout(P)^T dO
  for (int idx = threadIdx.x; idx < lk * w2; idx += blockDim.x) {
    const int j = idx / w2, e = idx - j * w2;
    float k0 = 0.f, k1 = 0.f, v0 = 0.f, v1 = 0.f;
    for (int i = 0; i < lq; ++i) {
      const float d = dS[i * sst + j], pr = Ps[i * sst + j];
      const float2 qv = unpack(Qs[i * st + e]);
      const float2 ov = unpack(Os[i * st + e]);
      k0 = fmaf(d, qv.x, k0);
      k1 = fmaf(d, qv.y, k1);
      v0 = fmaf(pr, ov.x, v0);
      v1 = fmaf(pr, ov.y, v1);
    }
    reinterpret_cast<uint32_t*>(P.dk + ((long)b * lk + j) * P.lddk + h * dh)[e] = pack(k0 * P.scale, k1 * P.scale);
    reinterpret_cast<uint32_t*>(P.dv + ((long)b * lk + j) * P.lddv + h * dh)[e] = pack(v0, v1);
  }
}

size_t fwd_smem(int lq, int lk, int dh) { return 4ul * ((lq + 2 * lk) * (dh / 2 + 1) + lq * (lk + 1)); }
size_t bwd_smem(int lq, int lk, int dh) {
  return 4ul * ((2 * lq + 2 * lk) * (dh / 2 + 1) + 2 * lq * (lk + 1));
}

int fill(AttnP& P, const vqa_attn_desc* d) {
  VQA_REQUIRE(d && d->q && d->k && d->v, "attention: null q/k/v");
  VQA_REQUIRE(d->lq > 0 && d->lk > 0 && d->lq <= 64 && d->lk <= 64, "attention: lq, lk must be in [1, 64]");
  VQA_REQUIRE(d->dh % 8 == 0 && d->dh <= 256, "attention: head dim must be a multiple of 8");
  VQA_REQUIRE(d->ldq % 8 == 0 && d->ldk % 8 == 0 && d->ldv % 8 == 0, "attention: strides must be multiples of 8");
  P.q = (const bf16_t*)d->q; P.k = (const bf16_t*)d->k; P.v = (const bf16_t*)d->v;
  P.ldq = d->ldq; P.ldk = d->ldk; P.ldv = d->ldv;
  P.o = (bf16_t*)d->o; P.ldo = d->ldo;
  P.p = d->p; P.bias = d->bias; P.mask = d->key_mask;
  P.heads = d->heads; P.lq = d->lq; P.lk = d->lk; P.dh = d->dh; P.scale = d->scale;
  P.dout = (const bf16_t*)d->dout; P.lddo = d->lddo;
  P.dq = (bf16_t*)d->dq; P.dk = (bf16_t*)d->dk; P.dv = (bf16_t*)d->dv;
  P.lddq = d->lddq; P.lddk = d->lddk; P.lddv = d->lddv;
  P.dbias = d->dbias;
  P.drop = d->drop;
  VQA_REQUIRE(d->drop.p >= 0.f && d->drop.p < 1.f, "attention: dropout p must be in [0, 1)");
  return VQA_OK;
}

// Attention probabilities only (output_attentions=True of HF ViTModel, vit_vqa_model.py:238-240):
// P[b, h, i, :] = softmax_j(scale * q_i . k_j (+ bias[h, i, j]) (+ finfo.min where key_mask[b, j] == 0)),
// fp32, one 256-thread workgroup per (b, h, query i); the q row sits in LDS, each thread takes keys
// j = tid, tid + 256, ...  An eval-time readout (the heat-map caller), not on the training path.
__global__ __launch_bounds__(256) void attn_probs_kernel(AttnP P, int pairs) {
  __shared__ float qs[1024];
  __shared__ float red[8];
  const int blk = blockIdx.x, i = blk % P.lq, pair = blk / P.lq;
  const int b = pair / P.heads, hh = pair - b * P.heads;
  const bf16_t* q = P.q + ((long)b * P.lq + i) * P.ldq + (long)hh * P.dh;
  for (int c = threadIdx.x; c < P.dh; c += 256) qs[c] = bf2f(q[c]);
  __syncthreads();
  float* prow = P.p + (((long)b * P.heads + hh) * P.lq + i) * P.lk;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < P.lk; j += 256) {
    const bf16_t* k = P.k + ((long)b * P.lk + j) * P.ldk + (long)hh * P.dh;
    float acc = 0.f;
    for (int c = 0; c < P.dh; c += 2) {
      const float2 kv = unpack(*reinterpret_cast<const uint32_t*>(k + c));
      acc = fmaf(qs[c], kv.x, fmaf(qs[c + 1], kv.y, acc));
    }
    float v = acc * P.scale;
    if (P.bias) v += P.bias[((long)hh * P.lq + i) * P.lk + j];
    if (P.mask && P.mask[(long)b * P.lk + j] == 0) v += MASK_MIN;
    prow[j] = v;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float z = 0.f;
  for (int j = threadIdx.x; j < P.lk; j += 256) {         // each thread re-reads only its own entries
    const float e = __expf(prow[j] - mx);
    prow[j] = e;
    z += e;
  }
  z = wave_sum(z);
  if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = z;
  __syncthreads();
  const float iz = 1.f / (red[4] + red[5] + red[6] + red[7]);
  for (int j = threadIdx.x; j < P.lk; j += 256) prow[j] *= iz;
}

}  // namespace

bool vqa_attn_mfma_ok(const vqa_attn_desc* d);           // attention_mfma.hip
int vqa_attn_fwd_mfma(const vqa_attn_desc* d, hipStream_t s);
int vqa_attn_bwd_mfma(const vqa_attn_desc* d, hipStream_t s);

bool vqa_attn_long_ok(const vqa_attn_desc* d);
int vqa_attn_fwd_long(const vqa_attn_desc* d, hipStream_t s);

extern "C" int vqa_attn_path(const vqa_attn_desc* d, int backward) {
  if (!d) return -1;
  if (!backward && d->groups <= 1 && (d->lq > 32 || d->lk > 64) && vqa_attn_long_ok(d)) return VQA_ATTN_LONG;
  return vqa_attn_mfma_ok(d) ? VQA_ATTN_MFMA : VQA_ATTN_VALU;
}

extern "C" int vqa_attn_fwd(const vqa_attn_desc* d, hipStream_t s) {
  VQA_REQUIRE(d && d->q && d->k && d->v, "attention: null q/k/v");
  if (d->groups <= 1 && (d->lq > 32 || d->lk > 64) && vqa_attn_long_ok(d))
    return vqa_attn_fwd_long(d, s);                                // ViT (config 4)
  VQA_REQUIRE(d->o, "vqa_attn_fwd: null output");
  VQA_REQUIRE(d->drop.p >= 0.f && d->drop.p < 1.f, "attention: dropout p must be in [0, 1)");
  VQA_REQUIRE(d->batch > 0 && d->heads > 0, "attention: empty batch");
  VQA_REQUIRE(d->groups <= 1 || ((long)d->groups * d->batch * d->heads < (1l << 30) && vqa_attn_mfma_ok(d) &&
                                 !d->bias && !d->dbias && !d->key_mask),
              "attention: groups > 1 needs the MFMA shapes and no bias / key mask");
  if (vqa_attn_mfma_ok(d)) return vqa_attn_fwd_mfma(d, s);        // the step's shapes (lk <= 160)
  AttnP P;
  if (int rc = fill(P, d)) return rc;
  const size_t sm = fwd_smem(d->lq, d->lk, d->dh);
  VQA_REQUIRE(sm <= 65536, "vqa_attn_fwd: shape needs %zu B of LDS (> 64 KiB)", sm);
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(d->batch * d->heads), dim3(256), sm, s, P);
  return vqa::check_launch("vqa_attn_fwd");
}

extern "C" int vqa_attn_bwd(const vqa_attn_desc* d, hipStream_t s) {
  VQA_REQUIRE(d && d->q && d->k && d->v, "attention: null q/k/v");
  VQA_REQUIRE(d->p && d->dout && d->dq && d->dk && d->dv, "vqa_attn_bwd: null P / dO / dQ / dK / dV");
  VQA_REQUIRE(d->lddo % 8 == 0, "vqa_attn_bwd: dO stride must be a multiple of 8");
  VQA_REQUIRE(d->drop.p >= 0.f && d->drop.p < 1.f, "attention: dropout p must be in [0, 1)");
  VQA_REQUIRE(d->batch > 0 && d->heads > 0, "attention: empty batch");
  VQA_REQUIRE(d->groups <= 1 || ((long)d->groups * d->batch * d->heads < (1l << 30) && vqa_attn_mfma_ok(d) &&
                                 !d->bias && !d->dbias && !d->key_mask),
              "attention: groups > 1 needs the MFMA shapes and no bias / key mask");
  if (vqa_attn_mfma_ok(d)) return vqa_attn_bwd_mfma(d, s);        // lk <= 160
  AttnP P;
  if (int rc = fill(P, d)) return rc;
  const size_t sm = bwd_smem(d->lq, d->lk, d->dh);
  VQA_REQUIRE(sm <= 65536, "vqa_attn_bwd: shape needs %zu B of LDS (> 64 KiB)", sm);
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(d->batch * d->heads), dim3(256), sm, s, P);
  return vqa::check_launch("vqa_attn_bwd");
}

extern "C" int vqa_attn_probs(const vqa_attn_desc* d, hipStream_t s) {
  VQA_REQUIRE(d && d->q && d->k && d->p, "vqa_attn_probs: null q / k / p");
  VQA_REQUIRE(d->batch > 0 && d->heads > 0 && d->lq > 0 && d->lk > 0 && d->dh > 0 && d->dh <= 1024 && d->dh % 2 == 0,
              "vqa_attn_probs: bad shape (dh even, <= 1024)");
  VQA_REQUIRE(d->ldk % 2 == 0 && ((uintptr_t)d->k & 3) == 0, "vqa_attn_probs: k rows must be 4-byte aligned");
  VQA_REQUIRE(d->groups <= 1, "vqa_attn_probs: one attention per call (groups <= 1)");
  AttnP P{};                                              // (fill() is for the lq, lk <= 64 kernels)
  P.q = (const bf16_t*)d->q; P.k = (const bf16_t*)d->k; P.ldq = d->ldq; P.ldk = d->ldk;
  P.p = d->p; P.bias = d->bias; P.mask = d->key_mask;
  P.heads = d->heads; P.lq = d->lq; P.lk = d->lk; P.dh = d->dh; P.scale = d->scale;
  const long grid = (long)d->batch * d->heads * d->lq;
  VQA_REQUIRE(grid < (1l << 31), "vqa_attn_probs: grid too large");
  hipLaunchKernelGGL(attn_probs_kernel, dim3((unsigned)grid), dim3(256), 0, s, P, d->batch * d->heads);
  return vqa::check_launch("vqa_attn_probs");
}
