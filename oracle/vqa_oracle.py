"""ORACLE — test infrastructure only, never the product path.

CPU fp32 restatement of one training step of the reference `ResnetVQAModel`
(shiv-vignesh/T5-Resnet-VQA), written from scratch in functional PyTorch-CPU
form.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg import this module, and only as the checker / the timed CPU
baseline.  The HIP engine in `t5-resnet-vqa_amd/` never imports it.

Pinning: the restatement is checked against golden vectors produced by the
reference modules themselves (imported in the build container by
`tests/golden/make_golden.py`; torchvision is absent there, so its ResNet is a
stub with torchvision's architecture — SURVEY.md Appendix A).  The ResNet
arithmetic is therefore pinned only by that architectural restatement; the T5
encoder (transformers 5.15 eager), SGA blocks, pooler, head, clip, AdamW and
scheduler are pinned by the real code.

Every function cites the reference line it restates.  State dicts use the
reference `state_dict()` key names.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

T5_EPS = 1e-6          # T5LayerNorm eps (t5-base config layer_norm_epsilon)
LN_EPS = 1e-5          # nn.LayerNorm default (multi_head_vision_text_attn.py:123)
BN_EPS = 1e-5          # torchvision BatchNorm2d default
SGA_HEADS, SGA_DHEAD = 8, 96     # multi_head_vision_text_attn.py:7-14 (t5-base width; head dim = width / 8)
T5_HEADS, T5_DKV = 12, 64        # t5-base; the encoder below reads heads / layers off the state dict
T5_BUCKETS, T5_MAX_DIST = 32, 128


# --------------------------------------------------------------------------- dropout
# nn.Dropout(p) in train mode draws its Bernoulli(1-p) keep mask from torch's
# RNG; a GPU path cannot reproduce that stream, so the build defines its masks
# by a stateless counter hash (include/vqa_hip.h, "dropout") and this oracle
# restates the same hash, which makes train-mode steps comparable element for
# element.  The mask law (keep prob 1-p, scale 1/(1-p)) is the reference's.
_M32 = 0xFFFFFFFF


def _mix32(x):
    """lowbias32 finaliser on uint64 arrays/ints holding 32-bit values."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_key(seed, counter, site):
    k0 = _mix32((seed + 0x9E3779B9) & _M32)
    k1 = _mix32(k0 ^ ((counter * 0x85EBCA6B + 0x632BE5AB) & _M32))
    return _mix32(k1 ^ ((site * 0xC2B2AE35 + 0x27D4EB2F) & _M32))


def dropout_multiplier(p, seed, counter, site, n):
    """float32 [n]: 1/(1-p) where element e is kept, 0 where dropped.  The 32-bit hash runs on
    int64 torch tensors (multi-threaded; products wrap mod 2^64 and are masked to their low 32
    bits, so every value equals the uint32 arithmetic of _mix32 -- tests/test_dropout_cpu.py)."""
    key = dropout_key(seed, counter, site)
    e = torch.arange(n, dtype=torch.int64)
    x = ((e * 0x9E3779B9) + key) & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    h = x ^ (x >> 16)
    thresh = int(float(np.float32(p)) * 4294967296.0)
    scale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
    return torch.where(h >= thresh, scale, 0.0).to(torch.float32).numpy()


def dropout_multiplier_np(p, seed, counter, site, n):
    """The same multipliers from the numpy uint64 form of the hash (tests compare the two)."""
    key = dropout_key(seed, counter, site)
    e = np.arange(n, dtype=np.uint64)
    h = _mix32(((e * np.uint64(0x9E3779B9)) + np.uint64(key)) & np.uint64(_M32))
    thresh = int(float(np.float32(p)) * 4294967296.0)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return np.where(h >= thresh, scale, np.float32(0.0)).astype(np.float32)


# site ids (same numbering as the engine: one per nn.Dropout application)
SITE_EMBED, SITE_FINAL = 1, 2


def t5_site(layer, kind):
    return 16 + 4 * layer + kind


def sga_site(block, kind):
    return 128 + 8 * block + kind


class HashDropout:
    """drop(site, x) -> x * mask(site) for one step (seed, counter); p = 0: identity."""

    def __init__(self, p, seed, counter):
        self.p, self.seed, self.counter = float(p), int(seed), int(counter)

    def __call__(self, site, x):
        if self.p <= 0.0:
            return x
        m = dropout_multiplier(self.p, self.seed, self.counter, site, x.numel())
        return x * torch.from_numpy(m).view(x.shape)


def _nodrop(site, x):
    return x


# --------------------------------------------------------------------------- fp8 (config 5)
# BASELINE configs[4] trains with "fp8 MFMA weights": the engine's forward weight GEMMs of the
# T5 layers and SGA blocks take row-wise e4m3 quantisations of the bf16 activation and of the
# fp32 weight (scale = row amax / 448, round to nearest even; include/vqa_hip.h
# vqa_quant_rows_fp8), the backward the unquantised operands.  No reference path computes in
# fp8, so this is the restatement of that arithmetic the fp8 engine is checked against, and
# the fp32 oracle (fp8=False) measures what the quantisation costs.
def fp8_rows(x):
    """Row-wise e4m3 quantise-dequantise: scale = amax / 448 and x / scale as correctly rounded
    fp32 divisions (computed in fp64, then rounded), then torch.float8_e4m3fn (nearest even)."""
    amax = x.detach().abs().amax(-1, keepdim=True).double()
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax)).float()
    q = (x.double() / s.double()).float().to(torch.float8_e4m3fn).float()
    return q * s


class _Fp8Matmul(torch.autograd.Function):
    """y = q(bf16(x)) q(w)^T; dx = dy w, dw = dy^T x (unquantised operands, as the engine)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return fp8_rows(x.bfloat16().float()) @ fp8_rows(w).T

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w
        dw = dy.reshape(-1, dy.shape[-1]).T @ x.reshape(-1, x.shape[-1])
        return dx, dw


def _mm(x, w, fp8=False):
    """x @ w^T (a Linear without bias), or its fp8 form."""
    return _Fp8Matmul.apply(x, w) if fp8 else x @ w.T


# --------------------------------------------------------------------------- ResNet
def _bn_eval(x, sd, p):
    """Frozen BatchNorm2d in eval mode (resnet_vqa_model.py:127 `vision_model.eval()`)."""
    w, b = sd[p + ".weight"], sd[p + ".bias"]
    rm, rv = sd[p + ".running_mean"], sd[p + ".running_var"]
    inv = torch.rsqrt(rv + BN_EPS)
    return (x - rm[None, :, None, None]) * (inv * w)[None, :, None, None] + b[None, :, None, None]


def resnet_features(sd, x, arch, prefix="vision_model."):
    """layer4 map of torchvision resnet18/34/50 run child-by-child, skipping
    avgpool/fc (resnet_vqa_model.py:115-121, 126-132)."""
    g = lambda k: sd[prefix + k]
    sdp = {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    x = x.float()
    x = F.conv2d(x, g("conv1.weight"), stride=2, padding=3)
    x = F.relu(_bn_eval(x, sdp, "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    nblocks = {"resnet18": (2, 2, 2, 2), "resnet34": (3, 4, 6, 3), "resnet50": (3, 4, 6, 3)}[arch]
    for li, nb in enumerate(nblocks):
        for bi in range(nb):
            p = f"layer{li + 1}.{bi}."
            stride = (1 if li == 0 else 2) if bi == 0 else 1
            idt = x
            if arch == "resnet50":        # Bottleneck v1.5: stride on the 3x3
                o = F.relu(_bn_eval(F.conv2d(x, sdp[p + "conv1.weight"]), sdp, p + "bn1"))
                o = F.relu(_bn_eval(F.conv2d(o, sdp[p + "conv2.weight"], stride=stride, padding=1), sdp, p + "bn2"))
                o = _bn_eval(F.conv2d(o, sdp[p + "conv3.weight"]), sdp, p + "bn3")
            else:                         # BasicBlock
                o = F.relu(_bn_eval(F.conv2d(x, sdp[p + "conv1.weight"], stride=stride, padding=1), sdp, p + "bn1"))
                o = _bn_eval(F.conv2d(o, sdp[p + "conv2.weight"], padding=1), sdp, p + "bn2")
            if (p + "downsample.0.weight") in sdp:
                idt = _bn_eval(F.conv2d(x, sdp[p + "downsample.0.weight"], stride=stride), sdp, p + "downsample.1")
            x = F.relu(o + idt)
    return x


# --------------------------------------------------------------------------- T5 encoder
def t5_relative_position_bucket(rel, num_buckets=T5_BUCKETS, max_distance=T5_MAX_DIST):
    """Bidirectional bucket (transformers T5Attention._relative_position_bucket,
    TF/models/t5/modeling_t5.py:217-262)."""
    num_buckets //= 2
    buckets = (rel > 0).long() * num_buckets
    rel = rel.abs()
    max_exact = num_buckets // 2
    is_small = rel < max_exact
    large = max_exact + (torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = torch.clamp(large, max=num_buckets - 1)
    return buckets + torch.where(is_small, rel, large)


def t5_position_bias(rel_emb, lq, lk):
    """compute_bias (modeling_t5.py:264-279): [1, H, Lq, Lk]."""
    ctx = torch.arange(lq)[:, None]
    mem = torch.arange(lk)[None, :]
    bucket = t5_relative_position_bucket(mem - ctx)
    return rel_emb[bucket].permute(2, 0, 1).unsqueeze(0)


def t5_rmsnorm(h, w):
    """T5LayerNorm (modeling_t5.py:50-72): w * h * rsqrt(mean(h^2) + eps), fp32 variance."""
    var = h.float().pow(2).mean(-1, keepdim=True)
    return w * (h * torch.rsqrt(var + T5_EPS))


def t5_encoder(sd, ids, mask, prefix="lang_model.", drop=_nodrop, fp8=False):
    """T5Stack encoder forward (modeling_t5.py:640-751), called from
    resnet_vqa_model.py:137-140.  Returns last_hidden_state [B, L, 768].
    `drop` applies the train-mode dropouts (identity = eval mode)."""
    g = lambda k: sd[prefix + k]
    B, L = ids.shape
    rel_emb = g("block.0.layer.0.SelfAttention.relative_attention_bias.weight")
    nh = rel_emb.shape[1]                                              # 12 (t5-base) / 16 (t5-large)
    dkv = g("block.0.layer.0.SelfAttention.q.weight").shape[0] // nh   # 64
    nl = sum(1 for k in sd if k.startswith(prefix + "block.") and k.endswith(".layer.0.layer_norm.weight"))
    h = drop(SITE_EMBED, g("embed_tokens.weight")[ids])                # :678, dropout :725
    ext = (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min   # bidirectional mask
    bias = t5_position_bias(rel_emb, L, L)
    for i in range(nl):
        p = f"block.{i}.layer."
        n = t5_rmsnorm(h, g(p + "0.layer_norm.weight"))                # T5LayerSelfAttention :384-401
        q = _mm(n, g(p + "0.SelfAttention.q.weight"), fp8).view(B, L, nh, dkv).transpose(1, 2)
        k = _mm(n, g(p + "0.SelfAttention.k.weight"), fp8).view(B, L, nh, dkv).transpose(1, 2)
        v = _mm(n, g(p + "0.SelfAttention.v.weight"), fp8).view(B, L, nh, dkv).transpose(1, 2)
        s = q @ k.transpose(2, 3)                                      # no 1/sqrt(d) (scaling = 1.0)
        s = s + bias + ext
        a = drop(t5_site(i, 0), torch.softmax(s.float(), dim=-1))     # :168
        o = (a @ v).transpose(1, 2).reshape(B, L, nh * dkv)
        h = h + drop(t5_site(i, 1), _mm(o, g(p + "0.SelfAttention.o.weight"), fp8))     # :400
        n = t5_rmsnorm(h, g(p + "1.layer_norm.weight"))                # T5LayerFF :126-141
        f = drop(t5_site(i, 2), F.relu(_mm(n, g(p + "1.DenseReluDense.wi.weight"), fp8)))  # :86
        h = h + drop(t5_site(i, 3), _mm(f, g(p + "1.DenseReluDense.wo.weight"), fp8))    # :140
    return drop(SITE_FINAL, t5_rmsnorm(h, g("final_layer_norm.weight")))         # :745


# --------------------------------------------------------------------------- SGA
def _linear(x, sd, p, fp8=False):
    return _mm(x, sd[p + ".weight"], fp8) + sd[p + ".bias"]


def sga_mhatt(sd, p, v, k, q, drop=_nodrop, site=0, fp8=False):
    """MHAtt.forward + att (multi_head_vision_text_attn.py:38-86), mask=None.  MULTI_HEAD = 8
    heads of HIDDEN_SIZE / 8 (96 at the reference's 768, 128 at config 5's 1024)."""
    B = q.shape[0]
    dh = sd[p + ".linear_q.weight"].shape[0] // SGA_HEADS
    V = _linear(v, sd, p + ".linear_v", fp8).view(B, -1, SGA_HEADS, dh).transpose(1, 2)
    K = _linear(k, sd, p + ".linear_k", fp8).view(B, -1, SGA_HEADS, dh).transpose(1, 2)
    Q = _linear(q, sd, p + ".linear_q", fp8).view(B, -1, SGA_HEADS, dh).transpose(1, 2)
    s = (Q @ K.transpose(-2, -1)) / math.sqrt(dh)
    a = drop(site, torch.softmax(s, dim=-1))                          # :83-84
    o = (a @ V).transpose(1, 2).contiguous().view(B, -1, SGA_HEADS * dh)
    return _linear(o, sd, p + ".linear_merge", fp8)


def _layernorm(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".norm.weight"], sd[p + ".norm.bias"], LN_EPS)


def sga_block(sd, p, x, y, drop=_nodrop, block=0, fp8=False):
    """SGA.forward (multi_head_vision_text_attn.py:145-158): post-LN; `drop` = train-mode dropouts."""
    st = lambda kind: sga_site(block, kind)
    x = _layernorm(x + drop(st(1), sga_mhatt(sd, p + ".mhatt1", x, x, x, drop, st(0), fp8)), sd, p + ".norm1")
    x = _layernorm(x + drop(st(3), sga_mhatt(sd, p + ".mhatt2", y, y, x, drop, st(2), fp8)), sd, p + ".norm2")
    f = _linear(drop(st(4), F.relu(_linear(x, sd, p + ".ffn.mlp.fc1", fp8))), sd, p + ".ffn.mlp.fc2", fp8)  # :97-101
    return _layernorm(x + drop(st(5), f), sd, p + ".norm3")


# --------------------------------------------------------------------------- full model
def model_forward(sd, batch, vision="resnet50", num_blocks=3, return_features=False, drop=_nodrop, fp8=False):
    """ResnetVQAModel.forward (resnet_vqa_model.py:101-165); eval mode unless
    `drop` (a HashDropout) supplies train-mode dropout.
    Returns (log_probs [B, A], loss scalar or None)."""
    with torch.no_grad():
        feat = resnet_features(sd, batch["image_tensors"], vision)
    scaler = "downscale_layer" if vision == "resnet50" else "upscale_layer"
    vis = F.conv_transpose2d(feat, sd[scaler + ".weight"], sd[scaler + ".bias"], stride=1, padding=1)
    txt = t5_encoder(sd, batch["question_input_ids"], batch["question_attention_masks"], drop=drop, fp8=fp8)
    y = vis.view(vis.shape[0], vis.shape[1], -1).permute(0, 2, 1)      # :142-143
    fused = None
    for n in range(num_blocks):                                        # :147-149 (Q4)
        fused = sga_block(sd, f"sga_modules.{n}", txt, y, drop, n, fp8)
        y = fused
    w = sd["attention_pooler.attention.0.weight"]                      # AttentionPooler :14-26
    a = torch.softmax(fused @ w.T + sd["attention_pooler.attention.0.bias"], dim=1)
    pooled = torch.bmm(a.transpose(1, 2), fused).squeeze(1)
    logits = pooled @ sd["classification_layer.weight"].T + sd["classification_layer.bias"]
    lp = F.log_softmax(logits, dim=-1)                                 # :156
    loss = None
    if batch.get("annotation_ids") is not None:
        loss = F.nll_loss(lp, batch["annotation_ids"])                 # :158-160 (mean)
    if return_features:
        return lp, loss, {"features": feat}
    return lp, loss


# --------------------------------------------------------------------------- optimiser
# faster_rcnn_vqa_trainer.py:231-267 with vit_daquar_config.json:37-48
GROUP_LRS = OrderedDict([
    ("vision_model", 0.008), ("lang_model", 0.005), ("scaler", 0.0005),
    ("sga_modules", 0.0005), ("attention_pooler", 0.0005), ("classification_layer", 1e-5)])
WEIGHT_DECAY, BETAS, ADAM_EPS, CLIP = 0.1, (0.9, 0.999), 1e-8, 1.0


def group_of(key, vision="resnet50"):
    top = key.split(".", 1)[0]
    if top in ("upscale_layer", "downscale_layer"):
        return "scaler"
    return top


def trainable_keys(sd, vision="resnet50"):
    """Parameters that receive gradients: not the frozen ResNet (Q1), not the
    unused scaler (Q3), not BN buffers."""
    unused = "upscale_layer" if vision == "resnet50" else "downscale_layer"
    return [k for k in sd if not k.startswith(("vision_model.", unused + "."))]


def lr_lambda(step, warmup, total):
    """get_linear_schedule_with_warmup (TF/optimization.py:101-107)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(total - step) / float(max(1, total - warmup)))


class OracleTrainer:
    """zero_grad -> fwd -> bwd -> clip_grad_norm_(1.0) -> AdamW(amsgrad) -> sched
    (faster_rcnn_vqa_trainer.py:391-406), all restated in fp32 on the CPU."""

    def __init__(self, sd, vision="resnet50", warmup=10, total=100, num_blocks=3, dropout=0.0, seed=0, fp8=False):
        self.vision, self.warmup, self.total, self.num_blocks = vision, warmup, total, num_blocks
        self.fp8 = bool(fp8)
        self.dropout, self.seed, self.rng_counter = float(dropout), int(seed), 0
        self.sd = OrderedDict((k, torch.as_tensor(v).clone()) for k, v in sd.items())
        self.keys = trainable_keys(self.sd, vision)
        for k in self.keys:
            self.sd[k].requires_grad_(True)
        self.m = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.v = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.vmax = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.step_count = 0        # LambdaLR last_epoch == AdamW state step before this step

    def forward_backward(self, batch):
        for k in self.keys:
            self.sd[k].grad = None
        drop = _nodrop
        if self.dropout > 0.0:                     # one draw per forward, like the engine's rng advance
            self.rng_counter += 1
            drop = HashDropout(self.dropout, self.seed, self.rng_counter)
        lp, loss = model_forward(self.sd, batch, self.vision, self.num_blocks, drop=drop, fp8=self.fp8)
        loss.backward()
        return lp.detach(), loss.detach()

    def grad_norm(self):
        """clip_grad_norm_ total norm: 2-norm of the per-parameter 2-norms."""
        norms = torch.stack([torch.linalg.vector_norm(self.sd[k].grad) for k in self.keys])
        return torch.linalg.vector_norm(norms)

    def group_grad_norms(self):
        out = OrderedDict()
        for k in self.keys:
            gname = group_of(k)
            out[gname] = out.get(gname, 0.0) + float(self.sd[k].grad.double().pow(2).sum())
        return OrderedDict((g, math.sqrt(v)) for g, v in out.items())

    @torch.no_grad()
    def clip_and_step(self):
        total = self.grad_norm()
        coef = torch.clamp(CLIP / (total + 1e-6), max=1.0)
        lam = lr_lambda(self.step_count, self.warmup, self.total)
        t = self.step_count + 1
        b1, b2 = BETAS
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        for k in self.keys:
            p, g = self.sd[k], self.sd[k].grad * coef
            lr = GROUP_LRS[group_of(k)] * lam
            p.mul_(1 - lr * WEIGHT_DECAY)                      # decoupled weight decay
            self.m[k].lerp_(g, 1 - b1)
            self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
            torch.maximum(self.vmax[k], self.v[k], out=self.vmax[k])
            denom = (self.vmax[k].sqrt() / math.sqrt(bc2)).add_(ADAM_EPS)
            p.addcdiv_(self.m[k], denom, value=-(lr / bc1))
        self.step_count += 1
        return total

    def train_one_step(self, batch):
        lp, loss = self.forward_backward(batch)
        gn = self.clip_and_step()
        return lp, loss, gn


def to_torch_batch(np_batch):
    out = {}
    for k, v in np_batch.items():
        out[k] = None if v is None else torch.as_tensor(v)
    return out
