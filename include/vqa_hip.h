/* libvqa_hip — MI355X (gfx950) kernels for the ResNet+T5+SGA VQA training step.
 *
 * Drop-in boundary.  The reference
 * (shiv-vignesh/T5-Resnet-VQA) has no FFI: its hot path is PyTorch eager
 * ops under `ResnetVQAModel.forward` (model/resnet_vqa_model.py:101-165),
 * `SGA.forward` (model/multi_head_vision_text_attn.py:145-158) and
 * `train_one_step` (trainer/faster_rcnn_vqa_trainer.py:391-406).  Each export
 * below replaces the ATen/cuDNN/cuBLAS calls of one op of that path (cited per
 * function).  Conventions:
 *   - plain C ABI: raw device pointers, sizes, an explicit hipStream_t;
 *   - every call returns 0 on success, else a VQA_ERR_* / hipError_t code; the
 *     message is in vqa_last_error() (thread-local); nothing throws;
 *   - the caller owns every buffer; the library allocates nothing per call,
 *     so every call is safe inside hipStream capture (hipGraph);
 *   - bf16 tensors are passed as void* (raw bfloat16 bits), fp32 as float*.
 */
#ifndef VQA_HIP_H
#define VQA_HIP_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VQA_ABI_VERSION 18
#define VQA_OK 0
#define VQA_ERR_INVALID 1000

int vqa_abi_version(void);
const char* vqa_last_error(void);

/* --------------------------------------------------------------- dropout ---
 * nn.Dropout(p) in training mode at the reference's 12 dropout sites of the
 * step (T5 encoder: embeddings, attention probabilities, attention/FF residual
 * branches, FF inner activation, final output -- TF modeling_t5.py:86, 140,
 * 168, 400, 725, 745; SGA: MHAtt.att probabilities, dropout1..3 and the MLP
 * inner activation -- multi_head_vision_text_attn.py:84, 99, 146-156).
 * Masks are counter-based, so the backward regenerates the forward mask and
 * nothing is stored: element e (the flat row-major index of the tensor the
 * dropout applies to) of site `site` is kept iff
 *   mix32(e * 0x9E3779B9 + key) >= (uint32)(p * 2^32)
 *   key = mix32(k1 ^ (site*0xC2B2AE35 + 0x27D4EB2F)),
 *   k1  = mix32(k0 ^ (rng[1]*0x85EBCA6B + 0x632BE5AB)), k0 = mix32(rng[0] + 0x9E3779B9),
 * mix32 = the lowbias32 finaliser; kept values are scaled by 1/(1-p).
 * rng is a device uint32[3] {seed, counter, training}; vqa_rng_advance()
 * increments the counter (once per step, first call of the forward), so a
 * replayed hipGraph draws fresh masks; training == 0 (model.eval()) turns every
 * dropout into the identity without re-planning or re-capturing.  p == 0 or
 * rng == NULL also means identity. */
typedef struct vqa_dropout {
  float p;
  unsigned site;
  const unsigned* rng;
} vqa_dropout;

int vqa_rng_advance(unsigned* rng, hipStream_t stream);
/* out[e] = keep(e) ? 1/(1-p) : 0 for e < n (tests / debugging) */
int vqa_dropout_mask(const vqa_dropout* d, float* out, long long n, hipStream_t stream);

/* ------------------------------------------------------------------ GEMM ---
 * C[m,n] = epilogue( alpha * sum_k A(m,k) * B(k,n) ), bf16 operands, fp32 MFMA
 * accumulation (v_mfma_f32_32x32x16_bf16).  Replaces every nn.Linear
 * (multi_head_vision_text_attn.py:31-34, 92-93; TF t5 q/k/v/o/wi/wo;
 * resnet_vqa_model.py:19, 85) forward, input-grad and weight-grad, and the
 * implicit-GEMM convolutions (torchvision conv layers, ConvTranspose2d
 * resnet_vqa_model.py:72-78).
 *   a_trans = 0: A(m,k) = a[m*lda + k]   a_trans = 1: A(m,k) = a[k*lda + m]
 *   b_trans = 0: B(k,n) = b[n*ldb + k]   b_trans = 1: B(k,n) = b[k*ldb + n]
 * a_conv = 1: A(m,k) is the implicit im2col of an NHWC bf16 activation
 *   (m = output pixel (img,oh,ow), k = (kh,kw,c)); requires a_trans = 0.
 * a_conv = 2: the same 3x3 / stride-1 / pad-1 convolution read from input patches staged
 *   once per 64-channel chunk in LDS (each input pixel crosses L2 -> LDS once, not 9x):
 *   k = (c / 64, kh, kw, c % 64), i.e. weights stored [Cout][C/64][3][3][64]; C % 64 == 0,
 *   b_trans = 0, batch 1, no split-K; tile configs VQA_GEMM_PATCH_FIRST..VQA_GEMM_PATCH_LAST.
 * b_conv: B(k,n) is the implicit im2col with k = output pixel, n = (kh,kw,c);
 *   requires b_trans = 1 (weight-gradient of a convolution).
 * Epilogue: k = [mask(m,n) > 0] * dropout multiplier of element (z*m+row)*n+col
 *   (1 when neither is given); v = k*(alpha*acc + bias[n]) + res(m,n); relu;
 *   c32 = v + beta*c32 (c32 may be NULL); c16 = bf16(v) (may be NULL).
 *   With res, relu acts after the residual (ResNet); relu with dropout needs no res.
 *   `relu` is the epilogue activation: 0 none, 1 ReLU, 2 GELU (erf form), 3 tanh;
 *   GELU / tanh take no dropout and no mask16 (ViT intermediate / pooler, config 4).
 * batch > 1 offsets a, b, c32, c16 by their strides and res/mask by stride_res. */
typedef struct vqa_conv_geom {
  int n, h, w, c;          /* NHWC input */
  int oh, ow;              /* output spatial size */
  int kh, kw, stride, pad;
} vqa_conv_geom;

typedef struct vqa_gemm_desc {
  const void* a; long long lda; int a_trans;
  const void* b; long long ldb; int b_trans;
  int m, n, k;
  float* c32; long long ldc32;
  void* c16; long long ldc16;
  const float* bias;
  const float* res32; const void* res16; long long ldres;
  const void* mask16; long long ldmask;
  float alpha, beta; int relu;
  int a_conv; vqa_conv_geom ga;
  int b_conv; vqa_conv_geom gb;
  int batch; long long stride_a, stride_b, stride_c32, stride_c16, stride_res;
  int config;              /* 0 auto, else a tile config 1..VQA_GEMM_CONFIGS (speed only: results are identical) */
  vqa_dropout drop;        /* dropout of the (alpha*acc + bias) branch, before the residual */
  /* split-K: splitk > 1 cuts K into splitk slices of whole 64-deep k-tiles computed by
   * separate workgroups; the last slice of a tile to finish sums all slices' fp32
   * partials in slice order (deterministic: same bits for every tile config at a
   * given splitk, different rounding from splitk = 1) and runs the epilogue.
   * workspace: >= vqa_gemm_workspace_bytes(d) bytes = a 64 KiB block of arrival
   * counters (<= 16384 tiles x batch) then the fp32 partial slabs; zero-filled
   * before its first use (the counters are left zero after every launch, so calls
   * on one stream may share a workspace); one in-flight launch per workspace.
   * splitk <= 1 ignores it. */
  int splitk;
  void* workspace;
  long long workspace_bytes;
  /* batched launches of distinct layers (the 3 SGA blocks' self-attention halves):
   * bias of batch z at bias + z*stride_bias; drop_site_stride != 0 gives batch z its
   * own dropout site (drop.site + z*drop_site_stride) with element indices restarting
   * at 0, i.e. exactly the masks of z separate launches (0: one site, index (z*m+row)*n+col) */
  long long stride_bias;
  int drop_site_stride;
  /* fp8 != 0: e4m3 (OCP float8_e4m3fn) operands for the forward weight GEMMs of BASELINE
   * configs[4] ("fp8 MFMA weights"): a = X8 [m][k] bytes (lda in bytes), b = W8 [n][k] bytes
   * (a_trans = b_trans = 0), both row-wise quantised by vqa_quant_rows_fp8; the accumulator
   * is scaled by scale_a[z*stride_scale_a + row] * scale_b[z*stride_scale_b + col] before the
   * epilogue (bias / residual / ReLU / dropout as usual).  k and lda / ldb multiples of 16,
   * n % 4 == 0, no conv operand, no GELU / tanh.  Products of e4m3 values are
   * exact in fp32, so the result differs from an fp32 GEMM of the dequantised operands only
   * by accumulation order. */
  int fp8;
  const float* scale_a;
  const float* scale_b;
  long long stride_scale_a, stride_scale_b;
} vqa_gemm_desc;

/* tile configs: 1 128x128/3 stages, 2 128x64/4, 3 64x64/4, 4 64x64/2, 5 64x64/3, 6 128x64/2,
 * 7 64x128/2, 8 128x128/2 (4 waves); 9 256x128/2, 10 128x256/2, 11 256x256/2, 12 256x128/3 (8 waves);
 * 13..16 64x192 / 128x192 (k-contiguous B only); 17..20 the LDS-patch convolution;
 * 21 64x64/2, 22 64x128/2, 23 128x64/2 with 128-deep k-tiles (no implicit im2col, no split-K);
 * 24 64x128/2 with 8 waves (2x4) and 128-deep k-tiles; 25 the LDS-patch convolution's 128x128 tile
 * with 8 waves (4x2); 26 64x128, 27 128x64, 28 64x64 for k <= 64 only (one k-tile in a single-stage
 * ring: more workgroups per CU; no implicit im2col) */
#define VQA_GEMM_CONFIGS 28
#define VQA_GEMM_PATCH_FIRST 17    /* configs 17..20 and VQA_GEMM_PATCH_WIDE: a_conv = 2 only */
#define VQA_GEMM_PATCH_LAST 20
#define VQA_GEMM_PATCH_WIDE 25
int vqa_gemm(const vqa_gemm_desc* d, hipStream_t stream);
/* Row-wise e4m3 quantisation for vqa_gemm_desc.fp8: per row r of x (fp32, or bf16 when
 * x_bf16), scale[r] = max_c |x[r][c]| / 448 (1 for an all-zero row) and
 * q[r][c] = e4m3(x[r][c] / scale[r]) (round to nearest even).  cols, ldx, ldq multiples of 8. */
int vqa_quant_rows_fp8(const void* x, int x_bf16, long long ldx, int rows, int cols, void* q, long long ldq,
                       float* scale, hipStream_t stream);
/* tile configuration (1..VQA_GEMM_CONFIGS) that vqa_gemm would run for this descriptor */
int vqa_gemm_select(const vqa_gemm_desc* d);
/* workspace bytes vqa_gemm needs for d (its config and splitk; 0 when splitk <= 1) */
long long vqa_gemm_workspace_bytes(const vqa_gemm_desc* d);
/* Two independent GEMMs in one launch: a layer's input gradient dX (a_trans=0,
 * b_trans=1) and weight gradient dW (a_trans=1, b_trans=1), both batch 1, no
 * conv.  Each keeps its own epilogue and tile config (configs 3, 4, 6, 7; others
 * map to 4).  Any other pair of descriptors runs as two vqa_gemm calls. */
int vqa_gemm_pair(const vqa_gemm_desc* dx, const vqa_gemm_desc* dw, hipStream_t stream);

/* ------------------------------------------------------------- attention ---
 * Multi-head attention core for Lq, Lk <= 64 (one workgroup per (b, head)):
 *   S = scale * Q K^T (+ bias[h,i,j]) (+ finfo(f32).min where key_mask[b,j]==0)
 *   P = softmax_j(S), O = P V.
 * Replaces MHAtt.att (multi_head_vision_text_attn.py:73-86; scale 1/sqrt(96),
 * 8 heads, no mask) and T5 eager attention (TF modeling_t5.py:144-173; scale 1,
 * 12 heads, relative bias, key mask).  Element (b, i, h, e) of Q lives at
 * q[(b*lq + i)*ldq + h*dh + e] (likewise K, V, O, dO, dQ, dK, dV), so Q/K/V are
 * read in place from fused projection outputs.  p: saved P [B, H, Lq, Lk].
 * Backward: dS = P (dP - rowsum(P dP)), dQ = scale dS K, dK = scale dS^T Q,
 * dV = P^T dO; when dbias != NULL the per-sample dS is written to
 * dbias[b, h, i, j] (reduce with vqa_batch_sum; no atomics -> deterministic).
 * drop: dropout on P (element index ((b*H + h)*Lq + i)*Lk + j): O = drop(P) V;
 * p keeps the pre-dropout P and the backward regenerates the mask.
 * Long forward (lq > 32 or lk > 64, up to lk = 1024; dh 64 / 96; no p, bias, mask or
 * dropout): ViTSelfAttention of BASELINE config 4 (vit_vqa_model.py:183-186, frozen,
 * no_grad), an online-softmax MFMA kernel; there is no long backward.
 * Causal T5 decoder self-attention (vit_vqa_model.py:199-205): the bias rows carry
 * finfo.min where j > i (vqa_t5_relbias_fwd with bucket < 0). */
typedef struct vqa_attn_desc {
  const void* q; long long ldq;
  const void* k; long long ldk;
  const void* v; long long ldv;
  void* o; long long ldo;
  float* p;
  const float* bias;
  const long long* key_mask;
  int batch, heads, lq, lk, dh;
  float scale;
  const void* dout; long long lddo;
  void* dq; long long lddq;
  void* dk; long long lddk;
  void* dv; long long lddv;
  float* dbias;
  vqa_dropout drop;
  /* groups > 1 (MFMA path): `groups` independent attentions of the same shape in ONE launch
   * (the SGA blocks' self-attention halves): group g reads / writes q, k, v, dq, dk, dv at
   * + g*gstride_qkv, o at + g*gstride_o, p at + g*gstride_p, dout at + g*gstride_dout
   * (elements), with dropout site drop.site + g*gdrop_site_stride and element indices from 0 --
   * the results of `groups` separate launches.  0 / 1: one attention (strides unused). */
  int groups;
  long long gstride_qkv, gstride_o, gstride_p, gstride_dout;
  int gdrop_site_stride;
} vqa_attn_desc;

int vqa_attn_fwd(const vqa_attn_desc* d, hipStream_t stream);
int vqa_attn_bwd(const vqa_attn_desc* d, hipStream_t stream);
/* which kernel vqa_attn_fwd (backward = 0) / vqa_attn_bwd (1) runs for d: the MFMA kernels
 * (lq <= 32, lk <= 160, dh 64 / 96 / 128; key mask only with lk <= 64), the long
 * online-softmax forward, or the scalar VALU kernel every other shape falls back to (an
 * order of magnitude slower: callers that plan a step check this and say so). */
#define VQA_ATTN_MFMA 0
#define VQA_ATTN_LONG 1
#define VQA_ATTN_VALU 2
int vqa_attn_path(const vqa_attn_desc* d, int backward);
/* The attention probabilities alone, d->p = [batch, heads, lq, lk] fp32:
 * softmax_j(scale q_i.k_j (+ bias) (+ finfo.min at masked keys)) for any lq, lk (dh <= 1024):
 * HF ViTModel(output_attentions=True), the `attentions` that VitVQAModel.generate_answers
 * returns (model/vit_vqa_model.py:238-240, 285-290).  Eval-time readout; o / v / dropout unused. */
int vqa_attn_probs(const vqa_attn_desc* d, hipStream_t stream);

/* ----------------------------------------------------------------- norms ---
 * Rows of width d (d % 256 == 0, d <= 1024), fp32 in, fp32 and/or bf16 out.
 * RMS: T5LayerNorm (TF modeling_t5.py:50-72): y = w * x * rsqrt(mean(x^2)+eps).
 * LN:  nn.LayerNorm (multi_head_vision_text_attn.py:120-126), post-LN of SGA.
 * Backward adds the residual gradient dres (may be NULL) into dx and reduces
 * the weight gradients deterministically through ws
 * (vqa_norm_bwd_workspace_floats(rows, d) floats).
 * Dropout hooks (NULL = none; element index row*d + col):
 *   rmsnorm_fwd drop: y = drop(norm(x))            (T5 final dropout, TF :745)
 *   rmsnorm_bwd drop_dy: the incoming dy is masked (backward of that dropout);
 *     drop_dx32 / drop_dx16: mask applied to that output only (the residual
 *     branch gradient of `h + dropout(f(h))`, or the embedding dropout)
 *   layernorm_bwd: dres is added into dx32 only (a running sum of residual
 *     gradients, e.g. the text gradient of the SGA blocks); dx16 and dsum see
 *     the LayerNorm input gradient alone.
 *   layernorm_bwd drop_dx16: mask on the bf16 output only (SGA dropout1..3);
 *     dsum (may be NULL) = column sums of that masked branch gradient in fp32,
 *     i.e. the bias gradient of the Linear feeding the dropout (fused). */
int vqa_rmsnorm_fwd(const float* x, const float* w, float* y32, void* y16, float* rstd, int rows, int d, float eps,
                    const vqa_dropout* drop, hipStream_t stream);
int vqa_rmsnorm_bwd(const float* dy, const float* x, const float* rstd, const float* w, const float* dres,
                    float* dx32, void* dx16, float* dw, float dw_beta, float* ws, int rows, int d,
                    const vqa_dropout* drop_dy, const vqa_dropout* drop_dx32, const vqa_dropout* drop_dx16,
                    hipStream_t stream);
int vqa_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y32, void* y16, float* mean,
                      float* rstd, int rows, int d, float eps, hipStream_t stream);
int vqa_layernorm_bwd(const float* dy, const float* x, const float* mean, const float* rstd, const float* gamma,
                      const float* dres, float* dx32, void* dx16, float* dgamma, float* dbeta, float* ws, int rows,
                      int d, const vqa_dropout* drop_dx16, float* dsum, hipStream_t stream);
int vqa_norm_bwd_workspace_floats(int rows, int d);
/* out[c] = beta*out[c] + sum_p ws[p*stride + c] (fixed order) */
int vqa_colsum_partials(const float* ws, int parts, long long stride, int cols, float* out, float beta,
                        hipStream_t stream);
/* Deferred reductions: vqa_rmsnorm_bwd with dw == NULL, vqa_layernorm_bwd with
 * dgamma == dbeta == NULL and vqa_colsum with out == NULL only write their per-block
 * partial rows into ws (rmsnorm: [vqa_norm_bwd_parts(rows)][d]; layernorm:
 * [parts][3][d] = dgamma, dbeta, dsum; colsum: [vqa_colsum_parts(rows)][cols]);
 * vqa_colsum_batched then finishes any number of such reductions in ONE launch.
 * jobs: DEVICE array; job j covers blocks [first_block, first_block + ceil(cols/64))
 * (first_block cumulative, nblocks = total), each computing
 * out[c] = beta*out[c] + sum_{p < parts} ws[p*stride + c] in fixed order. */
typedef struct vqa_colsum_job {
  const float* ws; float* out; long long stride; int parts; int cols; float beta; int first_block;
} vqa_colsum_job;
int vqa_norm_bwd_parts(int rows);
int vqa_colsum_parts(int rows);
int vqa_colsum_batched(const vqa_colsum_job* jobs, int njobs, int nblocks, hipStream_t stream);

/* ---------------------------------------------------------- elementwise ---
 * vqa_image_to_nhwc8: NCHW fp32 [N,3,H,W] (collate ToTensor,
 *   resnet_vqa_daquar_dataset.py:131-137) -> NHWC bf16 [N,H,W,8], ch 3..7 = 0.
 * vqa_image_to_s2d16: the same image as the stem's space-to-depth input
 *   Z [N,H/2+1,W/2+1,16] bf16, Z[b,u,v,(2p+q)*3+c] = img[b,c,2u+p-1,2v+q-1]
 *   (0 outside, ch 12..15 = 0); conv7x7/2 pad 3 over img == conv4x4/1 pad 1
 *   over Z with W'[o,a,e,(2p+q)*3+c] = W[o,c,2a+p,2e+q] (0 at index 7).
 *   H and W must be even.
 * vqa_maxpool3x3s2_nhwc: torchvision ResNet maxpool (3, 2, pad 1), bf16 NHWC.
 * vqa_subsample_nhwc: y[((b*oh + i)*ow + j)*ldy + c] = x[b, i*stride, j*stride, c] (bf16 NHWC,
 *   oh = (h-1)/stride + 1; c and ldy multiples of 8, y 16-B aligned): the input of a bottleneck's
 *   1x1 downsample placed beside conv2's output, so conv3 + downsample run as ONE GEMM over the
 *   concatenated K (torchvision Bottleneck: out = relu(bn3(conv3(t)) + bn(downsample(x)))).
 * vqa_colsum: out[c] = beta*out[c] + sum_r x[r*ld + c] (bias gradients of
 *   every nn.Linear / ConvTranspose2d), ws = vqa_colsum_workspace_floats().
 * vqa_embedding_fwd/bwd: T5 embed_tokens gather (TF modeling_t5.py:678) and
 *   its dense scatter-add gradient (dtable must be zeroed by the caller).
 * vqa_t5_relbias_fwd/bwd: compute_bias gather of the [buckets, H] table by a
 *   precomputed bucket map [Lq*Lk] (TF modeling_t5.py:217-279) and its
 *   scatter-add gradient (dtable zeroed by the caller).  bucket < 0 writes
 *   finfo(f32).min (a causally masked pair of the T5 decoder) and takes no gradient. */
int vqa_image_to_nhwc8(const float* img, void* out, int n, int h, int w, hipStream_t stream);
int vqa_image_to_s2d16(const float* img, void* out, int n, int h, int w, hipStream_t stream);
int vqa_maxpool3x3s2_nhwc(const void* x, void* y, int n, int h, int w, int c, int oh, int ow, hipStream_t stream);
int vqa_subsample_nhwc(const void* x, int n, int h, int w, int c, int stride, void* y, long long ldy,
                       hipStream_t stream);
/* vqa_stem_s2d_conv: the ResNet stem (conv1 7x7/2 pad 3 + folded bn1 + ReLU) as the 4x4 / stride-1 /
 *   pad-1 convolution over the space-to-depth image z [n][hz][hz][16] bf16 (vqa_image_to_s2d16) with
 *   weights w [64][4][4][16] bf16 and bias [64] fp32, into y [n][oh][oh][64] bf16; oh % 16 == 0,
 *   hz == oh + 1, 16-B aligned buffers.  The input patch of each 8 x 16 output block is staged in LDS
 *   once (the implicit GEMM re-reads every pixel per tap); bit-identical to vqa_gemm's a_conv = 1 form. */
int vqa_stem_s2d_conv(const void* z, const void* w, const float* bias, void* y, int n, int hz, int oh,
                      hipStream_t stream);
/* vqa_stem_pool_s2d: vqa_stem_s2d_conv followed by vqa_maxpool3x3s2_nhwc in one pass, bit-identical:
 *   y [n][oh/2][oh/2][64] bf16 (the pooled map only; the stem map is never stored); oh / 2 a multiple
 *   of 8, hz == oh + 1, 16-B aligned buffers. */
int vqa_stem_pool_s2d(const void* z, const void* w, const float* bias, void* y, int n, int hz, int oh,
                      hipStream_t stream);
/* vqa_stem_pool_img: vqa_image_to_s2d16 + vqa_stem_pool_s2d in one pass, bit-identical: the input
 *   patches are staged from the fp32 NCHW image img [n][3][h][h] directly (the space-to-depth image is
 *   never stored); y [n][h/4][h/4][64] bf16; h a multiple of 32, 16-B aligned w, bias and y. */
int vqa_stem_pool_img(const float* img, const void* w, const float* bias, void* y, int n, int h, hipStream_t stream);
int vqa_colsum(const void* x, int x_bf16, int rows, int cols, long long ld, float* out, float beta, float* ws,
               hipStream_t stream);
int vqa_colsum_workspace_floats(int rows, int cols);
/* drop: T5 embedding dropout (TF :725) on out (element token*d + col); NULL = none */
int vqa_embedding_fwd(const long long* ids, const float* table, float* out, int tokens, int d, int vocab,
                      const vqa_dropout* drop, hipStream_t stream);
/* ---------------------------------------------------------- input pipeline ---
 * The collate's image path (dataset_utils/resnet_vqa_daquar_dataset.py:145-163:
 * cv2.resize(INTER_LINEAR) to oh x ow, then ToTensor) for a whole batch: `src`
 * holds the decoded uint8 RGB images (HWC, row-major) back to back, desc[b] (device
 * memory) says where image b starts and its size; out = [batch, 3, oh, ow] fp32 in
 * [0, 1].  OpenCV's 8-bit fixed-point bilinear arithmetic (image.hip). */
typedef struct {
  long long offset;        /* byte offset of the image in src */
  int h, w;                /* source size (>= 1) */
} vqa_image_desc;
int vqa_resize_linear_u8(const void* src, const vqa_image_desc* desc, int batch, int oh, int ow, float* out,
                         hipStream_t stream);
/* deterministic, no atomics: each touched row gets its tokens' dh rows summed in token order
 * and ADDED to it (the rows must be zero, or hold an earlier partial sum); any number of
 * tokens (slices of 16384, in order); ws = 3*min(tokens, 16384) ints */
int vqa_embedding_bwd(const long long* ids, const float* dh, float* dtable, int tokens, int d, int vocab, int* ws,
                      hipStream_t stream);
/* zero the dtable rows named by ids_prev[0, tokens) (the rows the previous vqa_embedding_bwd
 * wrote), then ids_prev = ids_cur when ids_cur != NULL: keeps the dense gradient zero outside
 * the touched rows without clearing all vocab*d floats every step */
int vqa_embedding_zero_rows(long long* ids_prev, const long long* ids_cur, int tokens, float* dtable, int d,
                            int vocab, hipStream_t stream);
int vqa_t5_relbias_fwd(const float* table, const int* bucket, float* out, int heads, int lq, int lk,
                       hipStream_t stream);
/* dtable[b, h] = sum_{(i,j): bucket = b} dbias[h, i, j] (overwrites, fixed order) */
int vqa_t5_relbias_bwd(const float* dbias, const int* bucket, float* dtable, int heads, int lq, int lk,
                       int nbuckets, hipStream_t stream);
/* out[i] = beta*out[i] + sum_b x[b*n + i] (fixed order; reduces per-sample attention dS) */
int vqa_batch_sum(const float* x, int batch, long long n, float* out, float beta, hipStream_t stream);
int vqa_cast_f32_bf16(const float* x, void* y, long long n, hipStream_t stream);
int vqa_zero(void* p, long long bytes, hipStream_t stream);
/* dst <- src, 16-byte aligned (a kernel, so a captured step holds no runtime memcpy node) */
int vqa_copy(void* dst, const void* src, long long bytes, hipStream_t stream);
/* Tap-shifted copies of an NHWC bf16 map [n, h, w, c] (c % 8 == 0, 16-byte aligned):
 * out[t][(b*h + y)*w + x][:] = in[b][y - ky + pad][x - kx + pad][:] (0 outside), t = ky*kw + kx.
 * The ConvTranspose2d scaler's weight gradient (resnet_vqa_model.py:72-78, 135) as ONE GEMM
 * batched over the 9 taps: dW[:, t*C:(t+1)*C] = shift_t(dVIS)^T @ F4 -- plain operands in
 * place of the implicit im2col gather (127 -> 100 us at B=64, tools/convt_micro.py). */
int vqa_tap_shift(const void* in, void* out, int n, int h, int w, int c, int kh, int kw, int pad,
                  hipStream_t stream);

/* ------------------------------------------------ config 4: ViT + T5 enc-dec ---
 * VitVQAModel (model/vit_vqa_model.py:127-227) data movement (vit.hip):
 * vqa_vit_patchify: ViTPatchEmbeddings' Conv2d(3, 768, 16, stride 16) as an im2col:
 *   out[(b*np + p)][c*P*P + ky*P + kx] bf16 from NCHW fp32 pixel_values.
 * vqa_gather_rows / vqa_scatter_rows: dst[r] = src[row(r)] / dst[row(r)] = src[r],
 *   row(r) = idx ? idx[r] : offset + r*stride (stride 0 broadcasts one row); esz 2 or 4
 *   bytes, 16-byte rows: the CLS token rows, encoder_outputs[:, 0, :] into the fusing
 *   layer's concat (:189-195), the answer-token gather (:208-212) and its gradient.
 * vqa_last_index: out[b] = b*len + max{j : mask[b, j] == 1} (0 if none), (:208).
 * vqa_xattn1_fwd/bwd: the T5 decoder's EncDecAttention over its ONE encoder token
 *   (encoder_hidden_states = fused.unsqueeze(1), :199-205): context[b*len + i, h*dh + e]
 *   = drop(1)[b, h, i] * v[b, h*dh + e] (softmax over one key is 1; weight-dropout
 *   element ((b*H + h)*len + i)); backward dv[b] = sum_i drop * dctx[b*len + i]
 *   (query order), rows of dv lddv elements apart; q and k get no gradient. */
int vqa_vit_patchify(const float* img, void* out, int n, int h, int w, int patch, hipStream_t stream);
int vqa_gather_rows(const void* src, long long lds, const long long* idx, long long stride, long long offset,
                    void* dst, long long ldd, int rows, int cols, int esz, hipStream_t stream);
int vqa_scatter_rows(const void* src, long long lds, const long long* idx, long long stride, long long offset,
                     void* dst, long long ldd, int rows, int cols, int esz, hipStream_t stream);
int vqa_last_index(const long long* mask, int batch, int len, long long* out, hipStream_t stream);
int vqa_xattn1_fwd(const void* v, long long ldv, void* out, long long ldo, int batch, int len, int heads, int dh,
                   const vqa_dropout* drop, hipStream_t stream);
int vqa_xattn1_bwd(const void* dctx, long long ldd, float* dv32, void* dv16, long long lddv, int batch, int len,
                   int heads, int dh, const vqa_dropout* drop, hipStream_t stream);

/* ------------------------------------------------------------------ head ---
 * AttentionPooler (resnet_vqa_model.py:14-26) + classification_layer +
 * log_softmax + NLLLoss mean (:152-160).  fp32.  targets may be NULL in
 * forward (loss is then not computed, like annotation_ids=None).  A negative
 * target marks an ignored row, as nn.NLLLoss's ignore_index = -100: nll 0, no
 * gradient, and the mean runs over the rows with a target >= 0 (the engines pad a
 * loader's short final batch this way; ABI 17).  No valid row: loss = NaN (0/0),
 * as in torch.
 * Limits: seq <= 64, d <= 1024 (d % 4 == 0; 1024 = T5-large), batch <= 1024, answers <= 1024.
 * The forward writes the logits through logp.
 * ws = vqa_head_workspace_floats(batch, seq, d, answers) floats. */
int vqa_head_fwd(const float* x, const float* wp, const float* bp, const float* wc, const float* bc,
                 const long long* targets, float* att, float* pooled, float* logp, float* nll, float* loss,
                 int batch, int seq, int d, int answers, hipStream_t stream);
/* Backward.  row_total NULL: the NLL mean's divisor is this batch's valid-row count.  Data
 * parallel (ABI 18): row_total -> the valid-row count summed over the ranks (vqa_count_targets,
 * all-reduced) and row_scale = the world size; the divisor is then row_total[0] / row_scale, so
 * the ranks' gradients summed and scaled by 1/world are the global batch's mean however the rows
 * are split (a rank with no valid row gives zero), and loss[0] is rewritten as
 * sum(nll) * row_scale / row_total[0] (its mean over the ranks is the global batch's loss).
 * nll / loss are read / written only when row_total is set.  Replaces the DP form of
 * loss.backward() on a contiguously split global batch (NLLLoss mean, resnet_vqa_model.py:159). */
int vqa_head_bwd(const float* x, const float* att, const float* pooled, const float* logp, const long long* targets,
                 const float* wp, const float* wc, float* dx32, void* dx16, float* dwp, float* dbp, float* dwc,
                 float* dbc, float* ws, int batch, int seq, int d, int answers, const float* nll, float* loss,
                 const float* row_total, float row_scale, hipStream_t stream);
int vqa_head_workspace_floats(int batch, int seq, int d, int answers);
/* out[0] = (float) the number of targets >= 0 among targets[0..batch) (batch <= 1024). */
int vqa_count_targets(const long long* targets, int batch, float* out, hipStream_t stream);

/* ------------------------------------------------------------- optimiser ---
 * clip_grad_norm_(1.0) + AdamW(amsgrad) + linear warmup/decay schedule
 * (faster_rcnn_vqa_trainer.py:399-404, :231-287; TF optimization.py:101-107),
 * device-resident so a whole step is graph-capturable.  `state` is a float[16]
 * device block indexed by VQA_ST_*; vqa_optim_finalize reads STEP and writes
 * the rest, then advances STEP and sets PENDING = 1.  vqa_adamw_amsgrad is a
 * no-op while PENDING == 0: a caller that defers the update (the engine applies
 * it segment by segment inside the next forward, each parameter range just
 * before its first use) clears PENDING (16 bytes at state + 8, vqa_zero) once
 * every range is applied, so the update is applied exactly once. */
#define VQA_MAX_GROUPS 8
#define VQA_ST_STEP 0
#define VQA_ST_GRAD_NORM 1
#define VQA_ST_CLIP_COEF 2
#define VQA_ST_LR_SCALE 3
#define VQA_ST_BC1 4
#define VQA_ST_BC2_SQRT 5
#define VQA_ST_PENDING 8

typedef struct vqa_adamw_desc {
  float* param; const float* grad;
  float* exp_avg; float* exp_avg_sq; float* max_exp_avg_sq;
  void* param16;                      /* bf16 shadow written after the update (may be NULL) */
  long long n;
  int ngroups;
  long long group_end[VQA_MAX_GROUPS];/* exclusive end element of each contiguous group */
  float group_lr[VQA_MAX_GROUPS];
  float beta1, beta2, eps, weight_decay, grad_scale;
  const float* state;
} vqa_adamw_desc;

int vqa_grad_sqnorm(const float* g, long long n, double* ws, int parts, hipStream_t stream);
int vqa_optim_finalize(const double* ws, int parts, float grad_scale, float max_norm, int warmup, int total,
                       float beta1, float beta2, float* state, hipStream_t stream);
int vqa_adamw_amsgrad(const vqa_adamw_desc* d, hipStream_t stream);
/* The embedding table's AdamW split by rows (ABI 18; the dense table pass was the step's last,
 * exposed 0.9 GB).  vqa_embed_mark: mark[ids[i]] = the step counter (state[VQA_ST_STEP]) for the
 * step's n token ids (rows outside [0, rows) ignored); mark starts at -1.  vqa_adamw_rows over the
 * table d (n = rows x cols elements, its groups / state as vqa_adamw_amsgrad):
 *   touched = 0, BEFORE the step's vqa_optim_finalize: every row NOT marked with the counter gets
 *     the update with a zero gradient (exactly its gradient: no token touched it), using the LR
 *     multiplier and bias corrections that finalize is about to set (computed here from STEP,
 *     warmup, total); no clip coefficient is needed (0 * coef = 0).  Ignores PENDING.
 *   touched > 1: the same as 0 on a grid of `touched` workgroups striding over the rows (the
 *     engine's pass beside the backward chain: a grid per row would hold CU slots it waits for).
 *   touched = 1, AFTER finalize (STEP advanced): the marked rows get the full update (no-op while
 *     PENDING == 0).
 * Together bit-identical to vqa_adamw_amsgrad over the table.  Replaces the embedding part of
 * optimizer.step() (faster_rcnn_vqa_trainer.py:399-404) for a dense-gradient table that a step
 * touches in <= batch x seq rows. */
int vqa_embed_mark(const long long* ids, int n, int rows, int* mark, const float* state, hipStream_t stream);
int vqa_adamw_rows(const vqa_adamw_desc* d, const int* mark, int rows, int cols, int touched, int warmup, int total,
                   hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VQA_HIP_H */
