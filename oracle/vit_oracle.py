"""ORACLE -- test infrastructure only, never the product path.

CPU fp32 restatement of one training step of BASELINE config 4, the reference's
`VitVQAModel` (model/vit_vqa_model.py:127-227): frozen ViT-base pooled output,
T5-base encoder CLS row, fusing MLP, T5-base decoder over the single fused token,
answer-token gather, classifier, NLL; trained by the ViT trainer's AdamW groups
(trainer/vit_vqa_trainer.py:300-322, train_one_step :450-464 = clip + step + sched).
Only `tests/` and `bench.py`'s CPU baseline import it.

Pinning: checked against fixtures written by `tests/golden/make_golden_vit.py`,
which imports the reference `VitVQAModel` itself (transformers' ViTModel and
T5ForConditionalGeneration built from configs, no network).  The dropouts use the
same counter-hash masks as the engine (vqa_oracle.py, "dropout") so train-mode steps
compare element for element; the reference fixtures are eval-mode.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

from .vqa_oracle import (ADAM_EPS, BETAS, CLIP, SITE_EMBED, SITE_FINAL, T5_DKV, T5_HEADS, WEIGHT_DECAY,
                         dropout_multiplier, lr_lambda, t5_position_bias, t5_rmsnorm, t5_site)

VIT_HEADS, VIT_DH, VIT_EPS, VIT_PATCH = 12, 64, 1e-12, 16
FUSE_P = 0.5
# dropout sites of config 4 beyond the encoder's (vqa_oracle numbering): decoder embedding /
# final, the fusing layer, and per decoder layer: 0 self probs, 1 self branch, 2 cross probs,
# 3 cross branch, 4 FF inner, 5 FF branch (T5LayerSelfAttention / CrossAttention / FF)
SITE_DEC_EMBED, SITE_DEC_FINAL, SITE_FUSE = 3, 4, 5


def dec_site(layer, kind):
    return 256 + 8 * layer + kind


class HashDropout:
    """drop(site, x, p=None): x * mask(site); p defaults to the T5 rate."""

    def __init__(self, p, seed, counter):
        self.p, self.seed, self.counter = float(p), int(seed), int(counter)

    def __call__(self, site, x, p=None):
        p = self.p if p is None else float(p)
        if self.p <= 0.0 or p <= 0.0:
            return x
        m = dropout_multiplier(p, self.seed, self.counter, site, x.numel())
        return x * torch.from_numpy(m).view(x.shape)


def _nodrop(site, x, p=None):
    return x


def vit_pooled(sd, pix, prefix="vision_model.", attentions=None):
    """ViTModel(pixel_values).pooler_output (transformers ViTEmbeddings / ViTLayer (pre-LN) /
    ViTPooler): [B, 768].  Dropout probabilities are 0 in the ViT-base config.  attentions: a
    list that receives each layer's softmax probabilities [B, 12, L, L] (output_attentions=True,
    vit_vqa_model.py:238-240)."""
    g = lambda k: sd[prefix + k]
    B = pix.shape[0]
    x = F.conv2d(pix, g("embeddings.patch_embeddings.projection.weight"),
                 g("embeddings.patch_embeddings.projection.bias"), stride=VIT_PATCH)
    x = x.flatten(2).transpose(1, 2)
    x = torch.cat([g("embeddings.cls_token").expand(B, -1, -1), x], dim=1) + g("embeddings.position_embeddings")
    L = x.shape[1]
    for i in range(12):
        p = f"encoder.layer.{i}."
        n = F.layer_norm(x, (768,), g(p + "layernorm_before.weight"), g(p + "layernorm_before.bias"), VIT_EPS)
        qkv = [(n @ g(p + f"attention.attention.{t}.weight").T + g(p + f"attention.attention.{t}.bias"))
               .view(B, L, VIT_HEADS, VIT_DH).transpose(1, 2) for t in ("query", "key", "value")]
        s = qkv[0] @ qkv[1].transpose(2, 3) / math.sqrt(VIT_DH)
        if attentions is not None:
            attentions.append(torch.softmax(s, dim=-1))
        ctx = (torch.softmax(s, dim=-1) @ qkv[2]).transpose(1, 2).reshape(B, L, 768)
        x = ctx @ g(p + "attention.output.dense.weight").T + g(p + "attention.output.dense.bias") + x
        n = F.layer_norm(x, (768,), g(p + "layernorm_after.weight"), g(p + "layernorm_after.bias"), VIT_EPS)
        f = F.gelu(n @ g(p + "intermediate.dense.weight").T + g(p + "intermediate.dense.bias"))
        x = f @ g(p + "output.dense.weight").T + g(p + "output.dense.bias") + x
    x = F.layer_norm(x, (768,), g("layernorm.weight"), g("layernorm.bias"), VIT_EPS)
    return torch.tanh(x[:, 0] @ g("pooler.dense.weight").T + g("pooler.dense.bias"))


def t5_encoder(sd, ids, mask, drop=_nodrop, prefix="lang_model.encoder."):
    """T5Stack encoder (same restatement as vqa_oracle.t5_encoder, config-4 key prefix)."""
    g = lambda k: sd[prefix + k]
    B, L = ids.shape
    h = drop(SITE_EMBED, g("embed_tokens.weight")[ids])
    ext = (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    bias = t5_position_bias(g("block.0.layer.0.SelfAttention.relative_attention_bias.weight"), L, L)
    for i in range(12):
        p = f"block.{i}.layer."
        n = t5_rmsnorm(h, g(p + "0.layer_norm.weight"))
        q, k, v = [(n @ g(p + f"0.SelfAttention.{t}.weight").T).view(B, L, T5_HEADS, T5_DKV).transpose(1, 2)
                   for t in "qkv"]
        a = drop(t5_site(i, 0), torch.softmax((q @ k.transpose(2, 3) + bias + ext).float(), dim=-1))
        o = (a @ v).transpose(1, 2).reshape(B, L, 768)
        h = h + drop(t5_site(i, 1), o @ g(p + "0.SelfAttention.o.weight").T)
        n = t5_rmsnorm(h, g(p + "1.layer_norm.weight"))
        f = drop(t5_site(i, 2), F.relu(n @ g(p + "1.DenseReluDense.wi.weight").T))
        h = h + drop(t5_site(i, 3), f @ g(p + "1.DenseReluDense.wo.weight").T)
    return drop(SITE_FINAL, t5_rmsnorm(h, g("final_layer_norm.weight")))


def causal_position_bias(rel_emb, L, num_buckets=32, max_distance=128):
    """compute_bias with bidirectional=False (decoder): relative_position = -min(j - i, 0)."""
    i = torch.arange(L)[:, None]
    j = torch.arange(L)[None, :]
    n = -torch.min(j - i, torch.zeros_like(j - i))
    max_exact = num_buckets // 2
    large = max_exact + (torch.log(n.float() / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = torch.clamp(large, max=num_buckets - 1)
    bucket = torch.where(n < max_exact, n, large)
    return rel_emb[bucket].permute(2, 0, 1).unsqueeze(0)


def t5_decoder(sd, ids, mask, enc, drop=_nodrop, prefix="lang_model.decoder."):
    """T5Stack decoder (TF modeling_t5 T5Stack with is_decoder; blocks = self-attention with a
    causal + padding mask, cross-attention over `enc` [B, 1, 768] with no mask, ReLU FF),
    vit_vqa_model.py:199-205.  Returns last_hidden_state [B, L, 768]."""
    g = lambda k: sd[prefix + k]
    B, L = ids.shape
    h = drop(SITE_DEC_EMBED, g("embed_tokens.weight")[ids])
    causal = (torch.arange(L)[None, :] <= torch.arange(L)[:, None]).float()
    ext = (1.0 - causal[None, None] * mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    bias = causal_position_bias(g("block.0.layer.0.SelfAttention.relative_attention_bias.weight"), L) + ext
    for i in range(12):
        p = f"block.{i}.layer."
        n = t5_rmsnorm(h, g(p + "0.layer_norm.weight"))
        q, k, v = [(n @ g(p + f"0.SelfAttention.{t}.weight").T).view(B, L, T5_HEADS, T5_DKV).transpose(1, 2)
                   for t in "qkv"]
        a = drop(dec_site(i, 0), torch.softmax((q @ k.transpose(2, 3) + bias).float(), dim=-1))
        o = (a @ v).transpose(1, 2).reshape(B, L, 768)
        h = h + drop(dec_site(i, 1), o @ g(p + "0.SelfAttention.o.weight").T)
        n = t5_rmsnorm(h, g(p + "1.layer_norm.weight"))                 # T5LayerCrossAttention
        q = (n @ g(p + "1.EncDecAttention.q.weight").T).view(B, L, T5_HEADS, T5_DKV).transpose(1, 2)
        k = (enc @ g(p + "1.EncDecAttention.k.weight").T).view(B, 1, T5_HEADS, T5_DKV).transpose(1, 2)
        v = (enc @ g(p + "1.EncDecAttention.v.weight").T).view(B, 1, T5_HEADS, T5_DKV).transpose(1, 2)
        a = drop(dec_site(i, 2), torch.softmax((q @ k.transpose(2, 3)).float(), dim=-1))
        o = (a @ v).transpose(1, 2).reshape(B, L, 768)
        h = h + drop(dec_site(i, 3), o @ g(p + "1.EncDecAttention.o.weight").T)
        n = t5_rmsnorm(h, g(p + "2.layer_norm.weight"))
        f = drop(dec_site(i, 4), F.relu(n @ g(p + "2.DenseReluDense.wi.weight").T))
        h = h + drop(dec_site(i, 5), f @ g(p + "2.DenseReluDense.wo.weight").T)
    return drop(SITE_DEC_FINAL, t5_rmsnorm(h, g("final_layer_norm.weight")))


def model_forward(sd, batch, drop=_nodrop, pooled=None):
    """VitVQAModel.forward (:166-225) -> (log_probs, loss).  `pooled` overrides the ViT's
    pooled output (tests: isolating the frozen ViT's bf16 error from the trained part)."""
    if pooled is None:
        with torch.no_grad():
            pooled = vit_pooled(sd, batch["pixel_values"])
    enc = t5_encoder(sd, batch["question_input_ids"], batch["question_attention_masks"], drop)
    cat = torch.cat([pooled, enc[:, 0, :]], dim=1)
    fused = drop(SITE_FUSE, F.relu(cat @ sd["fusing_layer.0.weight"].T + sd["fusing_layer.0.bias"]), FUSE_P)
    dmask = batch["decoder_question_attention_masks"]
    dec = t5_decoder(sd, batch["decoder_question_input_ids"], dmask, fused.unsqueeze(1), drop)
    L = dmask.shape[1]
    last = torch.max(torch.where(dmask == 1, torch.arange(L), torch.zeros_like(dmask)), dim=1).values
    ans = dec[torch.arange(dec.shape[0]), last]
    lp = F.log_softmax(ans @ sd["classification_layer.weight"].T + sd["classification_layer.bias"], dim=-1)
    loss = F.nll_loss(lp, batch["annotation_ids"])
    return lp, loss


TIED = ("lang_model.encoder.embed_tokens.weight", "lang_model.decoder.embed_tokens.weight",
        "lang_model.lm_head.weight")
GROUP_LRS = {"classification_layer": 1e-5, "fusing_layer": 1e-5, "lang_model": 5e-3}


def group_of(key):
    return key.split(".", 1)[0]


class VitOracleTrainer:
    """zero_grad -> fwd -> bwd -> clip_grad_norm_(1.0) -> AdamW(amsgrad) -> sched over the
    trainable groups (vision: no gradient, skipped by AdamW), fp32 on the CPU."""

    def __init__(self, sd, warmup=10, total=100, dropout=0.0, seed=0, group_lr=None):
        self.warmup, self.total = warmup, total
        self.dropout, self.seed, self.rng_counter = float(dropout), int(seed), 0
        self.lrs = dict(GROUP_LRS, **(group_lr or {}))
        self.sd = OrderedDict((k, torch.as_tensor(v).clone()) for k, v in sd.items() if k not in TIED)
        for k in TIED:                                            # tie_word_embeddings: one tensor
            self.sd[k] = self.sd["lang_model.shared.weight"]
        self.keys = [k for k in self.sd if not k.startswith("vision_model.") and k not in TIED]
        for k in self.keys:
            self.sd[k].requires_grad_(True)
        self.m = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.v = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.vmax = {k: torch.zeros_like(self.sd[k]) for k in self.keys}
        self.step_count = 0

    def forward_backward(self, batch, pooled=None):
        for k in self.keys:
            self.sd[k].grad = None
        drop = _nodrop
        if self.dropout > 0.0:
            self.rng_counter += 1
            drop = HashDropout(self.dropout, self.seed, self.rng_counter)
        lp, loss = model_forward(self.sd, batch, drop=drop, pooled=pooled)
        loss.backward()
        for k in self.keys:                                       # parameters on the graph that got none
            if self.sd[k].grad is None:
                self.sd[k].grad = torch.zeros_like(self.sd[k])
        return lp.detach(), loss.detach()

    def grad_norm(self):
        return torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(self.sd[k].grad) for k in self.keys]))

    def group_grad_norms(self):
        out = OrderedDict()
        for k in self.keys:
            out[group_of(k)] = out.get(group_of(k), 0.0) + float(self.sd[k].grad.double().pow(2).sum())
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
            lr = self.lrs[group_of(k)] * lam
            p.mul_(1 - lr * WEIGHT_DECAY)
            self.m[k].lerp_(g, 1 - b1)
            self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
            torch.maximum(self.vmax[k], self.v[k], out=self.vmax[k])
            denom = (self.vmax[k].sqrt() / math.sqrt(bc2)).add_(ADAM_EPS)
            p.addcdiv_(self.m[k], denom, value=-(lr / bc1))
        self.step_count += 1
        return total

    def train_one_step(self, batch):
        lp, loss = self.forward_backward(batch)
        return lp, loss, self.clip_and_step()
