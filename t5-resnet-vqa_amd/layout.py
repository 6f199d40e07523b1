"""Flat parameter arena of the trainable part of `ResnetVQAModel`, in kernel
layout, and its exact mapping to/from the reference `state_dict()` keys
(SURVEY.md Appendix B).

All trainable parameters, their gradients and the three AdamW(amsgrad) states
live in single flat fp32 buffers (plus one bf16 shadow of the parameters for
the GEMM operands).  Segments are 64-element aligned and ordered in REVERSE
backward order (classifier ... embedding) so gradient buckets become ready
front to back; the optimizer groups of the reference trainer
(`faster_rcnn_vqa_trainer.py:231-267`) are contiguous ranges:
classification_layer | attention_pooler | sga_modules | scaler | lang_model.

Kernel-layout repacks (all exact permutations / concatenations):
  * SGA mhatt1 q|k|v and T5 q|k|v weights/biases are stacked into one [2304, 768]
    projection; SGA mhatt2 k|v into one [1536, 768] projection;
  * the ConvTranspose2d scaler weight W[c, o, p, q] (resnet_vqa_model.py:64-78)
    is stored as the equivalent convolution weight Wc[o, kh, kw, c] =
    W[c, o, 2-kh, 2-kw] so its forward/weight-grad are NHWC implicit GEMMs.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from . import synthetic as S

ALIGN = 64
GROUP_LR = OrderedDict([            # vit_daquar_config.json:40-48; trainer hard-codes 5e-4 (:244-261)
    ("classification_layer", 1e-5), ("attention_pooler", 5e-4), ("sga_modules", 5e-4),
    ("scaler", 5e-4), ("lang_model", 5e-3)])


def _convT_to_conv(w):          # [Cin, Cout, 3, 3] -> [Cout, 3, 3, Cin]
    return np.ascontiguousarray(w[:, :, ::-1, ::-1].transpose(1, 2, 3, 0))


def _conv_to_convT(w):          # inverse of the above
    return np.ascontiguousarray(w.transpose(3, 0, 1, 2)[:, :, ::-1, ::-1])


class Segment:
    __slots__ = ("name", "shape", "offset", "numel", "group", "parts", "kind")

    def __init__(self, name, shape, group, parts, kind="cat"):
        self.name, self.shape, self.group, self.parts, self.kind = name, tuple(shape), group, parts, kind
        self.numel = int(np.prod(self.shape))
        self.offset = -1


class ParamLayout:
    def __init__(self, vision="resnet50", answer_spaces=170, num_blocks=3, language_model="t5-base"):
        self.vision, self.answer_spaces, self.num_blocks = vision, answer_spaces, num_blocks
        self.dims = dm = S.lm_dims(language_model)
        D, A = dm.d_model, answer_spaces
        HI = dm.t5_heads * dm.t5_dkv                 # T5 attention inner width (= D for t5-base/large)
        self.scaler = "downscale_layer" if vision == "resnet50" else "upscale_layer"
        self.scaler_cin = 2048 if vision == "resnet50" else 512
        segs = []
        add = lambda *a, **k: segs.append(Segment(*a, **k))
        add("cls_w", (A, D), "classification_layer", ["classification_layer.weight"])
        add("cls_b", (A,), "classification_layer", ["classification_layer.bias"])
        add("pool_w", (D,), "attention_pooler", ["attention_pooler.attention.0.weight"], kind="flat")
        add("pool_b", (1,), "attention_pooler", ["attention_pooler.attention.0.bias"])
        for n in reversed(range(num_blocks)):
            p = f"sga_modules.{n}."
            m2 = p + "mhatt2."
            add(f"sga{n}.q2_w", (D, D), "sga_modules", [m2 + "linear_q.weight"])
            add(f"sga{n}.q2_b", (D,), "sga_modules", [m2 + "linear_q.bias"])
            add(f"sga{n}.kv2_w", (2 * D, D), "sga_modules", [m2 + f"linear_{x}.weight" for x in "kv"])
            add(f"sga{n}.kv2_b", (2 * D,), "sga_modules", [m2 + f"linear_{x}.bias" for x in "kv"])
            add(f"sga{n}.m2_w", (D, D), "sga_modules", [m2 + "linear_merge.weight"])
            add(f"sga{n}.m2_b", (D,), "sga_modules", [m2 + "linear_merge.bias"])
            for fc in ("fc1", "fc2"):
                add(f"sga{n}.{fc}_w", (D, D), "sga_modules", [p + f"ffn.mlp.{fc}.weight"])
                add(f"sga{n}.{fc}_b", (D,), "sga_modules", [p + f"ffn.mlp.{fc}.bias"])
            for ln in (1, 2, 3):
                add(f"sga{n}.ln{ln}_g", (D,), "sga_modules", [p + f"norm{ln}.norm.weight"])
                add(f"sga{n}.ln{ln}_b", (D,), "sga_modules", [p + f"norm{ln}.norm.bias"])
        # the self-attention halves of the blocks (x = the T5 output for every block)
        # run as batched launches after the blocks' sequential parts: their weights sit side
        # by side in block order, so the three q|k|v projections form one [3*2304, 768] matrix
        # and the three merges one batch with a constant stride
        m1 = lambda n: f"sga_modules.{n}.mhatt1."
        for n in range(num_blocks):
            add(f"sga{n}.qkv1_w", (3 * D, D), "sga_modules", [m1(n) + f"linear_{x}.weight" for x in "qkv"])
        for n in range(num_blocks):
            add(f"sga{n}.qkv1_b", (3 * D,), "sga_modules", [m1(n) + f"linear_{x}.bias" for x in "qkv"])
        for n in range(num_blocks):
            add(f"sga{n}.m1_w", (D, D), "sga_modules", [m1(n) + "linear_merge.weight"])
        for n in range(num_blocks):
            add(f"sga{n}.m1_b", (D,), "sga_modules", [m1(n) + "linear_merge.bias"])
        add("scaler_w", (D, 3, 3, self.scaler_cin), "scaler", [self.scaler + ".weight"], kind="convT")
        add("scaler_b", (D,), "scaler", [self.scaler + ".bias"])
        t5 = "lang_model."
        add("t5.final_ln", (D,), "lang_model", [t5 + "final_layer_norm.weight"])
        for i in reversed(range(dm.t5_layers)):
            b = f"{t5}block.{i}.layer."
            add(f"t5.{i}.qkv_w", (3 * HI, D), "lang_model", [b + f"0.SelfAttention.{x}.weight" for x in "qkv"])
            add(f"t5.{i}.o_w", (D, HI), "lang_model", [b + "0.SelfAttention.o.weight"])
            add(f"t5.{i}.ln0", (D,), "lang_model", [b + "0.layer_norm.weight"])
            add(f"t5.{i}.wi", (dm.t5_dff, D), "lang_model", [b + "1.DenseReluDense.wi.weight"])
            add(f"t5.{i}.wo", (D, dm.t5_dff), "lang_model", [b + "1.DenseReluDense.wo.weight"])
            add(f"t5.{i}.ln1", (D,), "lang_model", [b + "1.layer_norm.weight"])
        add("t5.relbias", (S.T5_BUCKETS, dm.t5_heads), "lang_model",
            [t5 + "block.0.layer.0.SelfAttention.relative_attention_bias.weight"])
        add("t5.embed", (S.T5_VOCAB, D), "lang_model", [t5 + "embed_tokens.weight"])

        off = 0
        self.segments = OrderedDict()
        for s in segs:
            s.offset = off
            off += (s.numel + ALIGN - 1) // ALIGN * ALIGN
            self.segments[s.name] = s
        self.total = off
        # contiguous optimizer groups
        self.groups = OrderedDict()
        for s in segs:
            g = self.groups.setdefault(s.group, [s.offset, s.offset + s.numel])
            g[1] = s.offset + (s.numel + ALIGN - 1) // ALIGN * ALIGN
        starts = [v[0] for v in self.groups.values()]
        assert starts == sorted(starts), "optimizer groups must be contiguous"
        self.trainable_keys = [k for s in segs for k in s.parts]
        self.num_params = sum(s.numel for s in segs)

    def __getitem__(self, name) -> Segment:
        return self.segments[name]

    # ------------------------------------------------------------------ conversions
    def pack(self, sd) -> np.ndarray:
        """reference state_dict (numpy/torch values) -> flat fp32 arena (kernel layout)."""
        flat = np.zeros(self.total, dtype=np.float32)
        for s in self.segments.values():
            vals = [np.asarray(sd[k], dtype=np.float32) for k in s.parts]
            if s.kind == "convT":
                v = _convT_to_conv(vals[0])
            elif s.kind == "flat":
                v = vals[0].reshape(-1)
            else:
                v = np.concatenate(vals, axis=0) if len(vals) > 1 else vals[0]
            assert v.shape == s.shape, (s.name, v.shape, s.shape)
            flat[s.offset:s.offset + s.numel] = v.reshape(-1)
        return flat

    def unpack(self, flat) -> "OrderedDict[str, np.ndarray]":
        """flat arena -> reference state_dict entries (reference shapes/layout)."""
        flat = np.asarray(flat)
        out = OrderedDict()
        specs = S.model_specs(self.vision, self.answer_spaces, self.num_blocks, self.dims)
        for s in self.segments.values():
            v = flat[s.offset:s.offset + s.numel].reshape(s.shape)
            if s.kind == "convT":
                out[s.parts[0]] = _conv_to_convT(v)
            elif s.kind == "flat":
                out[s.parts[0]] = v.reshape(specs[s.parts[0]]).copy()
            else:
                rows = [specs[k][0] for k in s.parts]
                for k, a, b in zip(s.parts, np.cumsum([0] + rows[:-1]), np.cumsum(rows)):
                    out[k] = np.ascontiguousarray(v[a:b]).reshape(specs[k])
        return out

    def group_of_element(self):
        """(group_end_exclusive list, lr list) for the AdamW kernel."""
        ends = [v[1] for v in self.groups.values()]
        ends[-1] = self.total
        return ends, [GROUP_LR[g] for g in self.groups]


def t5_bucket_map(lq, lk, num_buckets=S.T5_BUCKETS, max_distance=S.T5_MAX_DIST):
    """Bidirectional relative-position buckets (transformers
    T5Attention._relative_position_bucket, TF/models/t5/modeling_t5.py:217-262),
    restated in fp32 numpy so the table matches torch's fp32 log/truncation."""
    rel = np.arange(lk)[None, :] - np.arange(lq)[:, None]
    nb = num_buckets // 2
    out = (rel > 0).astype(np.int64) * nb
    n = np.abs(rel)
    max_exact = nb // 2
    safe = np.maximum(n, 1).astype(np.float32)
    large = max_exact + (np.log(safe / np.float32(max_exact)) / np.float32(np.log(max_distance / max_exact))
                         * np.float32(nb - max_exact)).astype(np.int64)
    large = np.minimum(large, nb - 1)
    return (out + np.where(n < max_exact, n, large)).astype(np.int32)


def fold_bn(w, bn_w, bn_b, rm, rv, eps=1e-5):
    """conv + frozen eval BatchNorm -> conv with per-channel scale folded in, bias."""
    scale = (bn_w / np.sqrt(rv + eps)).astype(np.float32)
    return (w * scale[:, None, None, None]).astype(np.float32), (bn_b - rm * scale).astype(np.float32)
