// MFMA attention core for the step's two attention shapes, one wave per (batch, head):
//   SGA  MHAtt.att   softmax(QK^T/sqrt(96)) V, 8 heads x 96   multi_head_vision_text_attn.py:73-86
//   T5   attention   softmax(QK^T + relbias + mask) V, 12 x 64 TF/models/t5/modeling_t5.py:144-173
// Lq <= 32 queries (one 32-wide MFMA tile), Lk <= 64 keys (two), dh in {64, 96}.
//
// Layouts (v_mfma_f32_32x32x16_bf16: D[i][j] += a[i][k] b[k][j]; lane l holds
// a[l&31][8(l>>5)+0..7], b[8(l>>5)+0..7][l&31]; D lane l = column j = l&31,
// register r = row i = (r&3) + 8(r>>2) + 4(l>>5)):
//   * "X" = S^T tile: lane = query, registers = 16 keys of a 32-key tile.  Row
//     softmax / row sums are in-lane + one lane^32 exchange.  The registers of a
//     16-key step, in order, are keys 16s + 4h + {0..3, 8..11} (h = l>>5) -- an
//     MFMA k-order that the other operand reproduces with ds_read_b64_tr_b16
//     rows 16s+4h and 16s+8+4h, so P / dS feed the next MFMA straight from
//     registers (no shuffles).
//   * "Y" = S tile: lane = key, registers = queries (backward only, for dV / dK).
//   * Q, K, V, dO fragments with k = head dim are 16-B row loads from global;
//     fragments with k = key / query come from small LDS images via
//     ds_read_b64_tr_b16 (the transposing read).
//   * outputs (O, dQ, dK, dV) are produced transposed (lane = token, registers =
//     4 consecutive head-dim columns) so every store is 8 contiguous bytes.
// Forward stores the pre-dropout P (fp32) for backward (and the T5 rel-bias
// gradient needs per-sample dS anyway); backward recomputes nothing else.
#include "common.h"

namespace {

constexpr float MASK_MIN = -3.4028234663852886e38f;     // torch.finfo(float32).min
typedef __attribute__((address_space(3))) char lds_char;
typedef short s16x8_t __attribute__((ext_vector_type(8)));

struct AttnM {
  const bf16_t *q, *k, *v; long ldq, ldk, ldv;
  bf16_t* o; long ldo;
  float* p;
  const float* bias;
  const long long* mask;
  int pairs, heads, lq, lk;
  float scale;
  const bf16_t* dout; long lddo;
  bf16_t *dq, *dk, *dv; long lddq, lddk, lddv;
  float* dbias;
  vqa_dropout drop;
  int pg;                                               // pairs per group (batch * heads)
  long gq, go, gp, gdo;                                 // group strides (vqa_attn_desc.gstride_*)
  int gsite;                                            // dropout site stride per group
};

// group of `pair` (vqa_attn_desc.groups): its (batch, head) index inside the group, the
// group's operand offsets applied to a copy of the parameters, its dropout site
__device__ __forceinline__ int group_pair(AttnM& P, int pair) {
  if (P.pg <= 0 || pair >= P.pairs) return pair;
  const int g = pair / P.pg;
  if (g == 0) return pair;
  P.q += g * P.gq; P.k += g * P.gq; P.v += g * P.gq;
  if (P.o) P.o += g * P.go;
  if (P.p) P.p += g * P.gp;
  if (P.dout) P.dout += g * P.gdo;
  if (P.dq) P.dq += g * P.gq;
  if (P.dk) P.dk += g * P.gq;
  if (P.dv) P.dv += g * P.gq;
  P.drop.site += (unsigned)(g * P.gsite);
  return pair - g * P.pg;
}

// Every global load below is issued UNconditionally at a clamped (valid) address
// and zeroed afterwards by an AND mask / multiply: "if (ok) load" or "ok ? load : 0"
// makes hipcc branch around each load and wait for it (one L2 round trip per
// load, cdna_hip_programming.md §5 'Three .s-level traps' (c)).
__device__ __forceinline__ uint32_t okmask(bool ok) { return ok ? 0xffffffffu : 0u; }

// `row` must point at a valid row (callers clamp the index); ok = 0 zeroes the fragment
__device__ __forceinline__ bf16x8_t ld_frag(const bf16_t* row, bool ok) {
  uint4 u = *reinterpret_cast<const uint4*>(row);
  const uint32_t m = okmask(ok);
  u.x &= m; u.y &= m; u.z &= m; u.w &= m;
  return __builtin_bit_cast(bf16x8_t, u);
}

__device__ __forceinline__ f32x16_t mfma(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// tr-read fragment of an LDS image [rows][ROWB bytes] (bf16, row-major): lane gets
// column c0 + (l & 31) at rows kb0 + 0..3 (j = 0..3) and kb1 + 0..3 (j = 4..7),
// kb0 = 16s + 4h, kb1 = kb0 + 8 (the X-layout k order).
template <int ROWB>
__device__ __forceinline__ bf16x8_t tr_frag(const lds_char* img, int s, int c0) {
  const int l = threadIdx.x & 63, h = l >> 5, g1 = (l >> 4) & 1, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
  const int col = c0 + 16 * g1 + 4 * p;
  const int r0 = 16 * s + 4 * h + q;
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + r0 * ROWB + col * 2));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + (r0 + 8) * ROWB + col * 2));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// stage rows [n][DH] bf16 (global row stride ld) into an LDS image [ROWS][ROWB]; rows >= n are zero
template <int DH, int ROWS, int ROWB>
__device__ __forceinline__ void stage_img(lds_char* img, const bf16_t* src, long ld, int n) {
  const int l = threadIdx.x & 63;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int CPR = DH / 8;                           // 16-B chunks per row
  constexpr int PER = ROWS * CPR / 64;                  // chunks per lane (exact for DH 64 / 96)
  static_assert(ROWS * CPR % 64 == 0, "image chunks must split evenly over the wave");
  u32x4 u[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {                       // all loads first, then all LDS writes
    const int idx = l + 64 * j, r = idx / CPR, c = idx - r * CPR;
    u[j] = *reinterpret_cast<const u32x4*>(src + (long)max(min(r, n - 1), 0) * ld + c * 8);
    u[j] &= u32x4{okmask(r < n), okmask(r < n), okmask(r < n), okmask(r < n)};
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int idx = l + 64 * j, r = idx / CPR, c = idx - r * CPR;
    *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(img + r * ROWB + c * 16) = u[j];
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// X-layout accumulator registers [8s'..8s'+7] (s' = s & 1) as a bf16 MFMA k-fragment
__device__ __forceinline__ bf16x8_t regs_frag(const f32x16_t& a, int s) {
  const int o = 8 * (s & 1);
  uint4 u;
  u.x = pack2(a[o], a[o + 1]); u.y = pack2(a[o + 2], a[o + 3]);
  u.z = pack2(a[o + 4], a[o + 5]); u.w = pack2(a[o + 6], a[o + 7]);
  return __builtin_bit_cast(bf16x8_t, u);
}

// store a transposed output tile: lane = token row (l&31), registers = columns
// c0 + (r&3) + 8(r>>2) + 4h -> 4 bf16 (8 B) per register group
__device__ __forceinline__ void store_tr(bf16_t* base, long ld, int row, bool ok, int c0, const f32x16_t& a,
                                         float mul) {
  if (!ok) return;
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint2 u;
    u.x = pack2(a[4 * g] * mul, a[4 * g + 1] * mul);
    u.y = pack2(a[4 * g + 2] * mul, a[4 * g + 3] * mul);
    *reinterpret_cast<uint2*>(base + (long)row * ld + c0 + 8 * g + 4 * h) = u;
  }
}

// waves (= (b, h) pairs) per block: two for the short key ranges; one from 3 key tiles on
// (SGA cross-attention over larger layer4 maps, e.g. 144 keys at 384^2), whose LDS images
// and saved-P transposes take up to ~100 KB per wave
constexpr int wpb_for(int nt) { return nt <= 2 ? 2 : 1; }
constexpr int MAX_NT = 5;                               // lk <= 160

// Values row[key] for this lane's 16 X-layout keys of 32-key tile t (keys 32t + 8g +
// 4h + 0..3 for register group g), loaded unconditionally at clamped keys: 4 float4
// loads when the row is 16-B aligned and lk % 4 == 0, else 16 scalar loads.
__device__ __forceinline__ void load_xrow(const float* row, int lk, int t, bool vec, float (&out)[16]) {
  const int h5 = (threadIdx.x & 63) >> 5;
  if (vec) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = *reinterpret_cast<const float4*>(row + min(32 * t + 8 * g + 4 * h5, lk - 4));
      out[4 * g] = v.x; out[4 * g + 1] = v.y; out[4 * g + 2] = v.z; out[4 * g + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) out[r] = row[min(32 * t + (r & 3) + 8 * (r >> 2) + 4 * h5, lk - 1)];
  }
}

// bit k = key k is kept by the padding mask (one load + one ballot per wave; lk <= 64)
__device__ __forceinline__ unsigned long long key_bits(const long long* mrow, int lk) {
  const int l = threadIdx.x & 63;
  const long long m = mrow[min(l, lk - 1)];
  return __ballot(m != 0 && l < lk);
}

template <int DH>
struct Geo {
  static constexpr int KS = DH / 16;                    // k-steps over the head dim
  static constexpr int ET = DH / 32;                    // 32-wide head-dim tiles
  static constexpr int ROWB = DH * 2 + 16;              // LDS image row (16-B aligned, banks spread)
};

// ------------------------------------------------------------------ forward
// NT = number of 32-key tiles (1: lk <= 32, 2: lk <= 64, ... MAX_NT), a template parameter
// so the lk <= 32 shapes (T5, SGA blocks 1-2) issue no work for a second tile.
template <int DH, int NT>
__global__ __launch_bounds__(64 * wpb_for(NT)) void attn_fwd_mfma(AttnM P) {
  using G = Geo<DH>;
  constexpr int WPB = wpb_for(NT);
  constexpr int KR = 32 * NT;                            // key rows of the V image
  __shared__ __attribute__((aligned(16))) char smem[WPB * KR * G::ROWB];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h5 = l >> 5, l31 = l & 31;
  const bool live = blockIdx.x * WPB + w < P.pairs;
  const int pair = group_pair(P, blockIdx.x * WPB + w);
  const int b = live ? pair / P.heads : 0, hh = live ? pair - b * P.heads : 0;
  const int lq = P.lq, lk = P.lk;
  lds_char* vimg = (lds_char*)smem + w * KR * G::ROWB;
  const bf16_t* Q = P.q + (long)b * lq * P.ldq + hh * DH;
  const bf16_t* K = P.k + (long)b * lk * P.ldk + hh * DH;
  const bf16_t* V = P.v + (long)b * lk * P.ldv + hh * DH;

  // fragments with k = head dim straight from global (16 B per lane per k-step)
  bf16x8_t qf[G::KS], kf[NT][G::KS];
  const int qr = min(l31, lq - 1);                                  // clamped rows
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
    qf[s] = ld_frag(Q + (long)qr * P.ldq + 16 * s + 8 * h5, live && l31 < lq);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      kf[t][s] = ld_frag(K + (long)min(32 * t + l31, lk - 1) * P.ldk + 16 * s + 8 * h5, live && 32 * t + l31 < lk);
  }
  stage_img<DH, KR, G::ROWB>(vimg, V, P.ldv, live ? lk : 0);
  // additive score terms for this lane's keys: rel-bias row (float4 row loads) and the
  // key-padding mask (one ballot)
  const int i = l31;
  float add[NT][16];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) add[t][r] = 0.f;
  if (P.bias) {
    const float* brow = P.bias + ((long)hh * lq + min(i, lq - 1)) * lk;
    const bool vec = (lk & 3) == 0 && ((uintptr_t)P.bias & 15) == 0;
#pragma unroll
    for (int t = 0; t < NT; ++t) load_xrow(brow, lk, t, vec, add[t]);
  }
  if (NT <= 2 && P.mask) {                              // lk <= 64 (host check for the mask)
    // one finfo.min per masked pair, as HF's combined extended mask has it: a pair the bias
    // already masks (the causal decoder's bucket < 0) does not take a second one (which
    // would give -inf and, for a fully masked query, a one-hot instead of a uniform row)
    const unsigned long long kb = key_bits(P.mask + (long)b * lk, lk);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool keep = (kb >> ((32 * t + (r & 3) + 8 * (r >> 2) + 4 * h5) & 63)) & 1ull;
        add[t][r] = (keep || add[t][r] <= 0.5f * MASK_MIN) ? add[t][r] : add[t][r] + MASK_MIN;
      }
  }

  // S^T tiles (X layout: lane = query, registers = keys)
  f32x16_t sa[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int e = 0; e < 16; ++e) sa[t][e] = 0.f;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) sa[t] = mfma(kf[t][s], qf[s], sa[t]);
  }
  // softmax over keys for query i = l31
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h5;
      const float v = key < lk ? sa[t][r] * P.scale + add[t][r] : -INFINITY;
      sa[t][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float z = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = sa[t][r] == -INFINITY ? 0.f : __expf(sa[t][r] - mx);
      sa[t][r] = e;
      z += e;
    }
  z += __shfl_xor(z, 32, 64);
  const float iz = 1.f / z;
  const DropK dk = drop_init(P.drop);
  const long prow = (((long)b * P.heads + hh) * lq + i) * lk;   // element index of P[b, h, i, 0]
  const bool qok = live && i < lq;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int key0 = 32 * t + 8 * g + 4 * h5;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = 4 * g + u, key = key0 + u;
        const float pr = sa[t][r] * iz;
        if (qok && key < lk && P.p) P.p[prow + key] = pr;          // saved pre-dropout P
        sa[t][r] = dk.on ? pr * drop_mul(dk, (uint32_t)(prow + key)) : pr;
      }
    }
  __syncthreads();                                                  // V image complete
  // O^T = V^T P^T: a = V^T (tr reads, k = key in X order), b = P from registers
#pragma unroll
  for (int et = 0; et < G::ET; ++et) {
    f32x16_t oa;
#pragma unroll
    for (int e = 0; e < 16; ++e) oa[e] = 0.f;
#pragma unroll
    for (int s = 0; s < 2 * NT; ++s) oa = mfma(tr_frag<G::ROWB>(vimg, s, et * 32), regs_frag(sa[s >> 1], s), oa);
    store_tr(P.o + (long)b * lq * P.ldo + hh * DH, P.ldo, i, qok, et * 32, oa, 1.f);
  }
}

// ------------------------------------------------------------------ backward
template <int DH, int NT>
__global__ __launch_bounds__(64 * wpb_for(NT)) void attn_bwd_mfma(AttnM P) {
  using G = Geo<DH>;
  constexpr int WPB = wpb_for(NT);
  constexpr int KR = 32 * NT;
  constexpr int IMG = (KR + 32 + 32) * G::ROWB;         // K [32*NT], dO [32], Q [32] images
  constexpr int PR = KR + 1;                             // row stride of the P / mask transposes (bank spread)
  constexpr int TRB = 2 * 32 * PR * 4;                   // saved P and dropout multipliers, [query][key] fp32
  __shared__ __attribute__((aligned(16))) char smem[WPB * (IMG + 32 * 4 + TRB)];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h5 = l >> 5, l31 = l & 31;
  const bool live = blockIdx.x * WPB + w < P.pairs;
  const int pair = group_pair(P, blockIdx.x * WPB + w);
  const int b = live ? pair / P.heads : 0, hh = live ? pair - b * P.heads : 0;
  const int lq = P.lq, lk = P.lk;
  lds_char* kimg = (lds_char*)smem + w * (IMG + 128 + TRB);
  lds_char* oimg = kimg + KR * G::ROWB;
  lds_char* qimg = oimg + 32 * G::ROWB;
  float* dis = (float*)(qimg + 32 * G::ROWB);           // D_i per query
  float* plds = dis + 32;                               // P[query][key] (masked, pre-dropout)
  float* mlds = plds + 32 * PR;                         // dropout multiplier [query][key]
  const bf16_t* Q = P.q + (long)b * lq * P.ldq + hh * DH;
  const bf16_t* K = P.k + (long)b * lk * P.ldk + hh * DH;
  const bf16_t* V = P.v + (long)b * lk * P.ldv + hh * DH;
  const bf16_t* dO = P.dout + (long)b * lq * P.lddo + hh * DH;
  const float* Pg = P.p + ((long)b * P.heads + hh) * lq * lk;

  bf16x8_t of[G::KS], vf[NT][G::KS];
  const int qr = min(l31, lq - 1);                      // clamped rows
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
    of[s] = ld_frag(dO + (long)qr * P.lddo + 16 * s + 8 * h5, live && l31 < lq);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      vf[t][s] = ld_frag(V + (long)min(32 * t + l31, lk - 1) * P.ldv + 16 * s + 8 * h5, live && 32 * t + l31 < lk);
  }
  stage_img<DH, KR, G::ROWB>(kimg, K, P.ldk, live ? lk : 0);
  stage_img<DH, 32, G::ROWB>(oimg, dO, P.lddo, live ? lq : 0);
  stage_img<DH, 32, G::ROWB>(qimg, Q, P.ldq, live ? lq : 0);
  const DropK dk = drop_init(P.drop);
  const long pbase = ((long)b * P.heads + hh) * lq * lk;  // dropout / dbias element base of (b, h)

  // ---- X layout (lane = query): dP^T, D_i, dS^T -> dQ^T
  const int i = l31;
  const bool qok = live && i < lq;
  f32x16_t xa[NT];
  float di = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int e = 0; e < 16; ++e) xa[t][e] = 0.f;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) xa[t] = mfma(vf[t][s], of[s], xa[t]);     // dP^T[key][query]
  }
  float px[NT][16];
  const float* prow = Pg + (long)min(i, lq - 1) * lk;   // saved P of this lane's query (clamped row)
  const bool pvec = (lk & 3) == 0 && ((uintptr_t)P.p & 15) == 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) load_xrow(prow, lk, t, pvec, px[t]);   // unconditional loads, masked below
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h5;
      const bool ok = qok && key < lk;
      const float pr = px[t][r] * (ok ? 1.f : 0.f);
      const float m = ok ? drop_mul(dk, (uint32_t)(pbase + (long)i * lk + key)) : 0.f;
      const float dp = xa[t][r] * m;
      plds[i * PR + key] = pr;                          // transposed for the Y-layout phase
      mlds[i * PR + key] = m;
      px[t][r] = pr;
      xa[t][r] = dp;                                    // dP (gradient w.r.t. the pre-dropout P)
      di += pr * dp;
    }
  di += __shfl_xor(di, 32, 64);
  if (h5 == 0) dis[i] = di;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float ds = px[t][r] * (xa[t][r] - di);
      xa[t][r] = ds;
      const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h5;
      if (P.dbias && qok && key < lk) P.dbias[pbase + (long)i * lk + key] = ds;   // per-sample dS
    }
  __syncthreads();                                      // images + D_i complete
  // dQ^T = scale K^T dS^T: a = K^T (tr reads of the K image, k = key), b = dS^T registers
#pragma unroll
  for (int et = 0; et < G::ET; ++et) {
    f32x16_t acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < 2 * NT; ++s) acc = mfma(tr_frag<G::ROWB>(kimg, s, et * 32), regs_frag(xa[s >> 1], s), acc);
    store_tr(P.dq + (long)b * lq * P.lddq + hh * DH, P.lddq, i, qok, et * 32, acc, P.scale);
  }

  // ---- Y layout (lane = key, registers = queries): dP, dS, dropout(P) -> dV^T, dK^T
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int key = 32 * t + l31;
    const bool kok = live && key < lk;
    f32x16_t ya;
#pragma unroll
    for (int e = 0; e < 16; ++e) ya[e] = 0.f;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) ya = mfma(of[s], vf[t][s], ya);        // dP[query][key]
    f32x16_t pd, dsy;
#pragma unroll
    for (int r = 0; r < 16; ++r) {                        // P and its dropout multiplier from the X phase
      const int qi = (r & 3) + 8 * (r >> 2) + 4 * h5;     // (zero outside the valid (query, key) range)
      const float pr = plds[qi * PR + key];
      const float m = mlds[qi * PR + key];
      pd[r] = pr * m;                                   // dropout(P)
      dsy[r] = pr * (ya[r] * m - dis[qi]);              // dS
    }
#pragma unroll
    for (int et = 0; et < G::ET; ++et) {
      f32x16_t va, ka;
#pragma unroll
      for (int e = 0; e < 16; ++e) { va[e] = 0.f; ka[e] = 0.f; }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        va = mfma(tr_frag<G::ROWB>(oimg, s, et * 32), regs_frag(pd, s), va);     // dV^T = dO^T dropout(P)
        ka = mfma(tr_frag<G::ROWB>(qimg, s, et * 32), regs_frag(dsy, s), ka);    // dK^T = Q^T dS
      }
      store_tr(P.dv + (long)b * lk * P.lddv + hh * DH, P.lddv, key, kok, et * 32, va, 1.f);
      store_tr(P.dk + (long)b * lk * P.lddk + hh * DH, P.lddk, key, kok, et * 32, ka, P.scale);
    }
  }
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

static void fillm(AttnM& M, const vqa_attn_desc* d) {
  M.q = (const bf16_t*)d->q; M.k = (const bf16_t*)d->k; M.v = (const bf16_t*)d->v;
  M.ldq = d->ldq; M.ldk = d->ldk; M.ldv = d->ldv;
  M.o = (bf16_t*)d->o; M.ldo = d->ldo; M.p = d->p; M.bias = d->bias; M.mask = d->key_mask;
  M.pairs = d->batch * d->heads; M.heads = d->heads; M.lq = d->lq; M.lk = d->lk; M.scale = d->scale;
  M.dout = (const bf16_t*)d->dout; M.lddo = d->lddo;
  M.dq = (bf16_t*)d->dq; M.dk = (bf16_t*)d->dk; M.dv = (bf16_t*)d->dv;
  M.lddq = d->lddq; M.lddk = d->lddk; M.lddv = d->lddv;
  M.dbias = d->dbias; M.drop = d->drop;
  M.pg = 0;
  M.gq = M.go = M.gp = M.gdo = 0;
  M.gsite = 0;
  if (d->groups > 1) {                                  // groups x (batch, head) pairs in one grid
    M.pg = M.pairs;
    M.pairs *= d->groups;
    M.gq = d->gstride_qkv; M.go = d->gstride_o; M.gp = d->gstride_p; M.gdo = d->gstride_dout;
    M.gsite = d->gdrop_site_stride;
  }
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
