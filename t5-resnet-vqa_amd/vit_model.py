"""Parameters, synthetic data and the flat arena of BASELINE config 4:
`VitVQAModel` (model/vit_vqa_model.py:127-227) -- a frozen ViT-base
(`google/vit-base-patch16-224-in21k`, :143-144, run under no_grad :183-186), the
T5-base encoder-decoder of `T5ForConditionalGeneration` (:146-147), the fusing
MLP Linear(1536, 768) + ReLU + Dropout(0.5) (:149-153) and the answer classifier
(:155-157), trained by the ViT trainer's AdamW groups
(trainer/vit_vqa_trainer.py:300-322: vision (no gradients), lang_model,
fusing_layer and classification_layer, the last two at `classifier_lr`).

State-dict keys are the reference's (transformers 4.34 module names,
SURVEY.md §0): `vision_model.embeddings...`, `vision_model.encoder.layer.{i}.
attention.attention.query...`, `lang_model.shared.weight` (tied to
`encoder.embed_tokens`, `decoder.embed_tokens` and `lm_head`), etc.

Kernel layout of the trainable arena (exact permutations / concatenations):
  * encoder / decoder self-attention q|k|v stacked into one [2304, 768] matrix;
  * the decoder's 12 cross-attention value projections side by side as ONE
    [12*768, 768] matrix: the encoder side of every cross-attention is the same
    single fused token, so all 12 value projections are one GEMM (and their
    input gradient one GEMM with K = 12*768);
  * the cross-attention q and k projections (and the cross sub-layer's
    layer norm) only ever receive zero gradients -- softmax over one key is
    constant -- but are kept and decayed like the reference's.
The frozen ViT weights live outside the arena (bf16 GEMM operands).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import numpy as np

from . import synthetic as S
from .layout import ALIGN, Segment

D = S.D_MODEL
VIT_LAYERS, VIT_HEADS, VIT_DH, VIT_FF = 12, 12, 64, 3072
VIT_PATCH, VIT_IMAGE = 16, 224
VIT_EPS = 1e-12                                   # ViTConfig.layer_norm_eps
DEC_LEN = 20                                      # Enums.MAX_LEN (dataset_utils/enums.py:50)
FUSE_P = 0.5                                      # fusing_layer Dropout(0.5) (:152)

# the reference ViT trainer's groups (vit_vqa_trainer.py:300-316; vit_daquar_config.json lrs)
VIT_GROUP_LR = OrderedDict([("classification_layer", 1e-5), ("fusing_layer", 1e-5), ("lang_model", 5e-3)])


def vit_tokens(image=VIT_IMAGE, patch=VIT_PATCH):
    return (image // patch) ** 2 + 1


def vit_specs(image=VIT_IMAGE):
    """ViTModel (transformers 4.34 names) key -> shape."""
    sp = OrderedDict()
    sp["embeddings.cls_token"] = (1, 1, D)
    sp["embeddings.position_embeddings"] = (1, vit_tokens(image), D)
    sp["embeddings.patch_embeddings.projection.weight"] = (D, 3, VIT_PATCH, VIT_PATCH)
    sp["embeddings.patch_embeddings.projection.bias"] = (D,)
    for i in range(VIT_LAYERS):
        p = f"encoder.layer.{i}."
        for n in ("query", "key", "value"):
            sp[f"{p}attention.attention.{n}.weight"] = (D, D)
            sp[f"{p}attention.attention.{n}.bias"] = (D,)
        sp[f"{p}attention.output.dense.weight"] = (D, D)
        sp[f"{p}attention.output.dense.bias"] = (D,)
        sp[f"{p}intermediate.dense.weight"] = (VIT_FF, D)
        sp[f"{p}intermediate.dense.bias"] = (VIT_FF,)
        sp[f"{p}output.dense.weight"] = (D, VIT_FF)
        sp[f"{p}output.dense.bias"] = (D,)
        for n in ("layernorm_before", "layernorm_after"):
            sp[f"{p}{n}.weight"] = (D,)
            sp[f"{p}{n}.bias"] = (D,)
    sp["layernorm.weight"] = (D,)
    sp["layernorm.bias"] = (D,)
    sp["pooler.dense.weight"] = (D, D)
    sp["pooler.dense.bias"] = (D,)
    return sp


def t5_stack_specs(decoder):
    sp = OrderedDict()
    for i in range(S.T5_LAYERS):
        p = f"block.{i}.layer."
        for n in "qkvo":
            sp[f"{p}0.SelfAttention.{n}.weight"] = (D, D)
        if i == 0:
            sp[f"{p}0.SelfAttention.relative_attention_bias.weight"] = (S.T5_BUCKETS, S.T5_HEADS)
        sp[f"{p}0.layer_norm.weight"] = (D,)
        f = 1
        if decoder:
            for n in "qkvo":
                sp[f"{p}1.EncDecAttention.{n}.weight"] = (D, D)
            sp[f"{p}1.layer_norm.weight"] = (D,)
            f = 2
        sp[f"{p}{f}.DenseReluDense.wi.weight"] = (S.T5_DFF, D)
        sp[f"{p}{f}.DenseReluDense.wo.weight"] = (D, S.T5_DFF)
        sp[f"{p}{f}.layer_norm.weight"] = (D,)
    sp["final_layer_norm.weight"] = (D,)
    return sp


def model_specs(answer_spaces=170, image=VIT_IMAGE):
    """`VitVQAModel.state_dict()` key -> shape (module registration order)."""
    sp = OrderedDict()
    for k, s in vit_specs(image).items():
        sp["vision_model." + k] = s
    sp["lang_model.shared.weight"] = (S.T5_VOCAB, D)
    sp["lang_model.encoder.embed_tokens.weight"] = (S.T5_VOCAB, D)
    for k, s in t5_stack_specs(False).items():
        sp["lang_model.encoder." + k] = s
    sp["lang_model.decoder.embed_tokens.weight"] = (S.T5_VOCAB, D)
    for k, s in t5_stack_specs(True).items():
        sp["lang_model.decoder." + k] = s
    sp["lang_model.lm_head.weight"] = (S.T5_VOCAB, D)
    sp["fusing_layer.0.weight"] = (D, 2 * D)
    sp["fusing_layer.0.bias"] = (D,)
    sp["classification_layer.weight"] = (answer_spaces, D)
    sp["classification_layer.bias"] = (answer_spaces,)
    return sp


TIED = ("lang_model.encoder.embed_tokens.weight", "lang_model.decoder.embed_tokens.weight",
        "lang_model.lm_head.weight")                     # = lang_model.shared.weight (tie_word_embeddings)


def init_param(key, shape, seed=0):
    """Closed-form initial value of one state-dict entry (ViTModel / T5 / nn.Linear init scales)."""
    if key in TIED:
        key = "lang_model.shared.weight"
    g = np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(("vit:" + key).encode())]))
    n = int(np.prod(shape))

    def normal(std):
        return (g.standard_normal(n, dtype=np.float32) * np.float32(std)).reshape(shape)

    def uniform(lo, hi):
        return (g.random(n, dtype=np.float32) * np.float32(hi - lo) + np.float32(lo)).reshape(shape)

    leaf = key.rsplit(".", 1)[-1]
    if key.startswith("vision_model."):                  # ViTPreTrainedModel._init_weights: trunc-normal 0.02
        if "layernorm" in key:
            return (1.0 + normal(0.05)).astype(np.float32) if leaf == "weight" else normal(0.02)
        if leaf == "bias":
            return normal(0.02)
        return normal(0.02)
    if key.startswith("lang_model."):
        if "shared" in key:
            return normal(1.0)
        if "relative_attention_bias" in key:
            return normal(D ** -0.5)
        if "layer_norm" in key:
            return (1.0 + normal(0.05)).astype(np.float32)
        if key.endswith(".q.weight"):
            return normal((D * S.T5_DKV) ** -0.5)
        if key.endswith(".wo.weight"):
            return normal(S.T5_DFF ** -0.5)
        return normal(D ** -0.5)
    fan_in = shape[-1] if len(shape) > 1 else (2 * D if key.startswith("fusing_layer") else D)
    b = 1.0 / np.sqrt(fan_in)                             # nn.Linear default
    return uniform(-b, b)


def make_state_dict(seed=0, answer_spaces=170, image=VIT_IMAGE):
    return OrderedDict((k, init_param(k, s, seed)) for k, s in model_specs(answer_spaces, image).items())


def make_batch(batch, seq_len, dec_len=DEC_LEN, image=VIT_IMAGE, seed=1, answer_spaces=170):
    """`VitVQADataset` collate shapes (dataset_utils/vit_vqa_daquar_dataset.py:130-195) as
    numpy: pixel_values (ViTImageProcessor: (x - 0.5) / 0.5 of a [0, 1] image), the question,
    and the decoder question `[QUESTION] text [ANSWER]` padded to MAX_LEN."""
    g = np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, 0x717A]))
    pix = (g.random((batch, 3, image, image), dtype=np.float32) - np.float32(0.5)) / np.float32(0.5)

    def text(L, lo):
        ids = np.zeros((batch, L), np.int64)
        mask = np.zeros((batch, L), np.int64)
        for b in range(batch):
            ell = int(g.integers(min(lo, L), L + 1))
            ids[b, 0] = S.QUESTION_TOKEN
            if ell > 2:
                ids[b, 1:ell - 1] = g.integers(2, 32100, size=ell - 2)
            ids[b, ell - 1] = 1
            mask[b, :ell] = 1
        return ids, mask
    q, qm = text(seq_len, 6)
    dq, dm = text(dec_len, 4)
    return {
        "question_input_ids": q, "question_attention_masks": qm,
        "decoder_question_input_ids": dq, "decoder_question_attention_masks": dm,
        "annotation_ids": g.integers(0, answer_spaces, size=batch).astype(np.int64),
        "pixel_values": pix, "image_tensors": None,
        "answer_input_ids": np.zeros((batch, dec_len), np.int64),
        "answer_attention_masks": np.zeros((batch, dec_len), np.int64), "question_type_ids": None,
    }


def causal_bucket_map(lq, num_buckets=S.T5_BUCKETS, max_distance=S.T5_MAX_DIST):
    """Decoder relative-position buckets (T5Attention._relative_position_bucket with
    bidirectional=False: relative_position = -min(j - i, 0), all 32 buckets on one side), with
    -1 where j > i (the causal mask; vqa_t5_relbias_fwd writes finfo.min there)."""
    i = np.arange(lq)[:, None]
    j = np.arange(lq)[None, :]
    n = np.maximum(i - j, 0)
    max_exact = num_buckets // 2
    safe = np.maximum(n, 1).astype(np.float32)
    large = max_exact + (np.log(safe / np.float32(max_exact)) / np.float32(np.log(max_distance / max_exact))
                         * np.float32(num_buckets - max_exact)).astype(np.int64)
    large = np.minimum(large, num_buckets - 1)
    out = np.where(n < max_exact, n, large)
    return np.where(j > i, -1, out).astype(np.int32)


class VitLayout:
    """Flat fp32 arena of the trainable parameters (classifier | fusing | lang_model)."""

    def __init__(self, answer_spaces=170):
        self.answer_spaces = A = answer_spaces
        segs = []
        add = lambda *a, **k: segs.append(Segment(*a, **k))
        add("cls_w", (A, D), "classification_layer", ["classification_layer.weight"])
        add("cls_b", (A,), "classification_layer", ["classification_layer.bias"])
        add("fuse_w", (D, 2 * D), "fusing_layer", ["fusing_layer.0.weight"])
        add("fuse_b", (D,), "fusing_layer", ["fusing_layer.0.bias"])
        dec, enc = "lang_model.decoder.", "lang_model.encoder."
        add("dec.final_ln", (D,), "lang_model", [dec + "final_layer_norm.weight"])
        for i in reversed(range(S.T5_LAYERS)):
            b = f"{dec}block.{i}.layer."
            add(f"dec.{i}.wo", (D, S.T5_DFF), "lang_model", [b + "2.DenseReluDense.wo.weight"])
            add(f"dec.{i}.wi", (S.T5_DFF, D), "lang_model", [b + "2.DenseReluDense.wi.weight"])
            add(f"dec.{i}.ln2", (D,), "lang_model", [b + "2.layer_norm.weight"])
            add(f"dec.{i}.xo_w", (D, D), "lang_model", [b + "1.EncDecAttention.o.weight"])
            add(f"dec.{i}.xq_w", (D, D), "lang_model", [b + "1.EncDecAttention.q.weight"])
            add(f"dec.{i}.xk_w", (D, D), "lang_model", [b + "1.EncDecAttention.k.weight"])
            add(f"dec.{i}.ln1", (D,), "lang_model", [b + "1.layer_norm.weight"])
            add(f"dec.{i}.o_w", (D, D), "lang_model", [b + "0.SelfAttention.o.weight"])
            add(f"dec.{i}.qkv_w", (3 * D, D), "lang_model", [b + f"0.SelfAttention.{x}.weight" for x in "qkv"])
            add(f"dec.{i}.ln0", (D,), "lang_model", [b + "0.layer_norm.weight"])
        add("dec.xv_w", (S.T5_LAYERS * D, D), "lang_model",
            [f"{dec}block.{i}.layer.1.EncDecAttention.v.weight" for i in range(S.T5_LAYERS)])
        add("dec.relbias", (S.T5_BUCKETS, S.T5_HEADS), "lang_model",
            [dec + "block.0.layer.0.SelfAttention.relative_attention_bias.weight"])
        add("enc.final_ln", (D,), "lang_model", [enc + "final_layer_norm.weight"])
        for i in reversed(range(S.T5_LAYERS)):
            b = f"{enc}block.{i}.layer."
            add(f"enc.{i}.qkv_w", (3 * D, D), "lang_model", [b + f"0.SelfAttention.{x}.weight" for x in "qkv"])
            add(f"enc.{i}.o_w", (D, D), "lang_model", [b + "0.SelfAttention.o.weight"])
            add(f"enc.{i}.ln0", (D,), "lang_model", [b + "0.layer_norm.weight"])
            add(f"enc.{i}.wi", (S.T5_DFF, D), "lang_model", [b + "1.DenseReluDense.wi.weight"])
            add(f"enc.{i}.wo", (D, S.T5_DFF), "lang_model", [b + "1.DenseReluDense.wo.weight"])
            add(f"enc.{i}.ln1", (D,), "lang_model", [b + "1.layer_norm.weight"])
        add("enc.relbias", (S.T5_BUCKETS, S.T5_HEADS), "lang_model",
            [enc + "block.0.layer.0.SelfAttention.relative_attention_bias.weight"])
        add("embed", (S.T5_VOCAB, D), "lang_model", ["lang_model.shared.weight"])
        off = 0
        self.segments = OrderedDict()
        for s in segs:
            s.offset = off
            off += (s.numel + ALIGN - 1) // ALIGN * ALIGN
            self.segments[s.name] = s
        self.total = off
        self.groups = OrderedDict()
        for s in segs:
            g = self.groups.setdefault(s.group, [s.offset, s.offset + s.numel])
            g[1] = s.offset + (s.numel + ALIGN - 1) // ALIGN * ALIGN
        self.trainable_keys = [k for s in segs for k in s.parts] + list(TIED)
        self.num_params = sum(s.numel for s in segs)

    def __getitem__(self, name):
        return self.segments[name]

    def pack(self, sd):
        flat = np.zeros(self.total, dtype=np.float32)
        for s in self.segments.values():
            vals = [np.asarray(sd[k], dtype=np.float32) for k in s.parts]
            v = np.concatenate(vals, axis=0) if len(vals) > 1 else vals[0]
            assert v.shape == s.shape, (s.name, v.shape, s.shape)
            flat[s.offset:s.offset + s.numel] = v.reshape(-1)
        return flat

    def unpack(self, flat):
        flat = np.asarray(flat)
        specs = model_specs(self.answer_spaces)
        out = OrderedDict()
        for s in self.segments.values():
            v = flat[s.offset:s.offset + s.numel].reshape(s.shape)
            rows = [specs[k][0] for k in s.parts]
            for k, a, b in zip(s.parts, np.cumsum([0] + rows[:-1]), np.cumsum(rows)):
                out[k] = np.ascontiguousarray(v[a:b]).reshape(specs[k])
        for k in TIED:
            out[k] = out["lang_model.shared.weight"]
        return out

    def group_of_element(self, group_lr=None):
        ends = [v[1] for v in self.groups.values()]
        ends[-1] = self.total
        lr = dict(VIT_GROUP_LR, **(group_lr or {}))
        return ends, [lr[g] for g in self.groups]
