"""Deterministic parameter and batch generators for the ResNet+T5+SGA VQA step.

No network is available, so neither `resnet50(pretrained=True)`
(reference `model/resnet_vqa_model.py:51-58`) nor
`T5ForQuestionAnswering.from_pretrained("t5-base")` (`:60-62`) can be fetched.
Every parameter is instead produced by a closed-form generator keyed on
(seed, parameter name), so the golden-fixture script (which loads these values
into the real reference module), the CPU oracle and the HIP engine all see
bit-identical weights on any machine.

Names and shapes follow the reference `ResnetVQAModel.state_dict()`
(torchvision ResNet children names, transformers
`T5Stack` names, `multi_head_vision_text_attn.py:31-34, 92-93, 108, 123,
132-143`, `resnet_vqa_model.py:64-89`).

The synthetic batch follows SURVEY.md §8(d): images U[0,1) (reference collate
applies ToTensor only, `dataset_utils/resnet_vqa_daquar_dataset.py:131-137`),
questions `[Question]`-prefixed, EOS=1 terminated and zero padded
(`:157-158, 192`), answer ids U[0, answer_spaces).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import NamedTuple

import numpy as np

D_MODEL = 768
T5_LAYERS = 12
T5_HEADS = 12
T5_DKV = 64
T5_DFF = 3072
T5_VOCAB = 32128
T5_BUCKETS = 32
T5_MAX_DIST = 128
SGA_HEADS = 8
SGA_DHEAD = 96
QUESTION_TOKEN = 32100      # id of the added "[Question]" special token



class LMDims(NamedTuple):
    """Widths of the language model and of the SGA blocks built to its width."""
    name: str
    d_model: int
    t5_layers: int
    t5_heads: int
    t5_dkv: int
    t5_dff: int
    sga_heads: int          # MULTI_HEAD (multi_head_vision_text_attn.py:10)
    sga_dhead: int          # HIDDEN_SIZE_HEAD = HIDDEN_SIZE // MULTI_HEAD (:11)


# t5-base: the reference's configuration (TextConfiguration / ImageConfiguration, :7-24).
# t5-large: BASELINE configs[4] -- the T5-large encoder (published t5-large sizes) with the SGA
# blocks, scaler, pooler and classifier at its width 1024 (8 heads of 128, FF 1024), i.e. the
# reference modules built from configuration instances with HIDDEN_SIZE = FF_SIZE = 1024.
LM_DIMS = {"t5-base": LMDims("t5-base", 768, 12, 12, 64, 3072, 8, 96),
           "t5-large": LMDims("t5-large", 1024, 24, 16, 64, 4096, 8, 128)}
BASE = LM_DIMS["t5-base"]


def lm_dims(language_model="t5-base") -> LMDims:
    if isinstance(language_model, LMDims):
        return language_model
    if language_model not in LM_DIMS:
        raise ValueError(f"language_model {language_model!r}: this path supports {tuple(LM_DIMS)}")
    return LM_DIMS[language_model]


RESNET_LAYERS = {"resnet18": (2, 2, 2, 2), "resnet34": (3, 4, 6, 3), "resnet50": (3, 4, 6, 3)}


def resnet_specs(arch: str):
    """torchvision ResNet v1.5 parameter/buffer names and shapes (stride on the 3x3)."""
    if arch not in RESNET_LAYERS:
        raise ValueError(f"unsupported vision model {arch!r}")
    bottleneck = arch == "resnet50"
    specs = OrderedDict()

    def conv(name, cout, cin, k):
        specs[name + ".weight"] = (cout, cin, k, k)

    def bn(name, c):
        for s in ("weight", "bias", "running_mean", "running_var"):
            specs[f"{name}.{s}"] = (c,)
        specs[f"{name}.num_batches_tracked"] = ()

    conv("conv1", 64, 3, 7)
    bn("bn1", 64)
    inplanes = 64
    for li, (planes, nblk) in enumerate(zip((64, 128, 256, 512), RESNET_LAYERS[arch])):
        for bi in range(nblk):
            stride = (1 if li == 0 else 2) if bi == 0 else 1
            p = f"layer{li + 1}.{bi}."
            if bottleneck:
                out = planes * 4
                conv(p + "conv1", planes, inplanes, 1); bn(p + "bn1", planes)
                conv(p + "conv2", planes, planes, 3); bn(p + "bn2", planes)
                conv(p + "conv3", out, planes, 1); bn(p + "bn3", out)
            else:
                out = planes
                conv(p + "conv1", planes, inplanes, 3); bn(p + "bn1", planes)
                conv(p + "conv2", planes, planes, 3); bn(p + "bn2", planes)
            if bi == 0 and (stride != 1 or inplanes != out):
                conv(p + "downsample.0", out, inplanes, 1); bn(p + "downsample.1", out)
            inplanes = out
    specs["fc.weight"] = (1000, inplanes)
    specs["fc.bias"] = (1000,)
    return specs


def t5_specs(dims=BASE):
    d = lm_dims(dims)
    D = d.d_model
    specs = OrderedDict()
    specs["embed_tokens.weight"] = (T5_VOCAB, D)
    for i in range(d.t5_layers):
        p = f"block.{i}.layer."
        inner = d.t5_heads * d.t5_dkv
        for n in "qkv":
            specs[f"{p}0.SelfAttention.{n}.weight"] = (inner, D)
        specs[f"{p}0.SelfAttention.o.weight"] = (D, inner)
        if i == 0:
            specs[f"{p}0.SelfAttention.relative_attention_bias.weight"] = (T5_BUCKETS, d.t5_heads)
        specs[f"{p}0.layer_norm.weight"] = (D,)
        specs[f"{p}1.DenseReluDense.wi.weight"] = (d.t5_dff, D)
        specs[f"{p}1.DenseReluDense.wo.weight"] = (D, d.t5_dff)
        specs[f"{p}1.layer_norm.weight"] = (D,)
    specs["final_layer_norm.weight"] = (D,)
    return specs


def sga_specs(dims=BASE):
    D = lm_dims(dims).d_model
    specs = OrderedDict()
    for m in ("mhatt1", "mhatt2"):
        for lin in ("linear_v", "linear_k", "linear_q", "linear_merge"):
            specs[f"{m}.{lin}.weight"] = (D, D)
            specs[f"{m}.{lin}.bias"] = (D,)
    for fc in ("fc1", "fc2"):
        specs[f"ffn.mlp.{fc}.weight"] = (D, D)
        specs[f"ffn.mlp.{fc}.bias"] = (D,)
    for n in ("norm1", "norm2", "norm3"):
        specs[f"{n}.norm.weight"] = (D,)
        specs[f"{n}.norm.bias"] = (D,)
    return specs


def model_specs(vision: str = "resnet50", answer_spaces: int = 170, num_attention_blocks: int = 3,
                language_model="t5-base"):
    """Full `ResnetVQAModel.state_dict()` key -> shape, in module registration order."""
    d = lm_dims(language_model)
    D = d.d_model
    specs = OrderedDict()
    for k, s in resnet_specs(vision).items():
        specs["vision_model." + k] = s
    for k, s in t5_specs(d).items():
        specs["lang_model." + k] = s
    specs["upscale_layer.weight"] = (512, D, 3, 3)
    specs["upscale_layer.bias"] = (D,)
    specs["downscale_layer.weight"] = (2048, D, 3, 3)
    specs["downscale_layer.bias"] = (D,)
    for n in range(num_attention_blocks):
        for k, s in sga_specs(d).items():
            specs[f"sga_modules.{n}.{k}"] = s
    specs["classification_layer.weight"] = (answer_spaces, D)
    specs["classification_layer.bias"] = (answer_spaces,)
    specs["attention_pooler.attention.0.weight"] = (1, D)
    specs["attention_pooler.attention.0.bias"] = (1,)
    return specs


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def init_param(key: str, shape, seed: int = 0, vision: str = "resnet50", dims=BASE) -> np.ndarray:
    """Closed-form initial value of one state-dict entry (float32; int64 for counters)."""
    d = lm_dims(dims)
    D_MODEL, T5_DKV, T5_DFF = d.d_model, d.t5_dkv, d.t5_dff
    if key.endswith("num_batches_tracked"):
        return np.array(0, dtype=np.int64)
    g = _rng(seed, key)
    n = int(np.prod(shape)) if shape else 1

    def normal(std):
        return (g.standard_normal(n, dtype=np.float32) * np.float32(std)).reshape(shape)

    def uniform(lo, hi):
        return (g.random(n, dtype=np.float32) * np.float32(hi - lo) + np.float32(lo)).reshape(shape)

    leaf = key.rsplit(".", 1)[-1]
    if key.startswith("vision_model."):
        if len(shape) == 4:                                   # conv: kaiming-normal fan_out (torchvision)
            return normal(np.sqrt(2.0 / (shape[0] * shape[2] * shape[3])))
        if key.startswith("vision_model.fc."):
            b = 1.0 / np.sqrt(shape[-1] if leaf == "weight" else 2048)
            return uniform(-b, b)
        # the BN closing each residual branch gets a small scale so the residual stream stays O(1)
        last_bn = ".bn3." in key or (vision != "resnet50" and ".bn2." in key)
        if leaf == "weight":                                  # frozen BN (folded), nontrivial stats
            return uniform(0.15, 0.35) if last_bn else uniform(0.7, 1.3)
        if leaf == "bias":
            return normal(0.05)
        if leaf == "running_mean":
            return normal(0.1)
        if leaf == "running_var":
            return uniform(0.5, 1.5)
    if key.startswith("lang_model."):                         # T5 _init_weights scales
        if "embed_tokens" in key:
            return normal(1.0)
        if "relative_attention_bias" in key:
            return normal(D_MODEL ** -0.5)
        if "layer_norm" in key:
            return (1.0 + normal(0.05)).astype(np.float32)
        if key.endswith(".q.weight"):
            return normal((D_MODEL * T5_DKV) ** -0.5)
        if key.endswith((".k.weight", ".v.weight", ".o.weight", ".wi.weight")):
            return normal(D_MODEL ** -0.5)
        if key.endswith(".wo.weight"):
            return normal(T5_DFF ** -0.5)
    if key.startswith(("upscale_layer.", "downscale_layer.")):
        # ConvTranspose2d default init: fan_in = weight.size(1) * k * k
        b = 1.0 / np.sqrt(D_MODEL * 9)
        return uniform(-b, b)
    if ".norm" in key and key.startswith("sga_modules."):
        return (1.0 + normal(0.05)).astype(np.float32) if leaf == "weight" else normal(0.02)
    # nn.Linear default: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias
    b = 1.0 / np.sqrt(D_MODEL)
    return uniform(-b, b)


def make_state_dict(vision: str = "resnet50", seed: int = 0, answer_spaces: int = 170,
                    num_attention_blocks: int = 3, keys=None, language_model="t5-base") -> "OrderedDict[str, np.ndarray]":
    d = lm_dims(language_model)
    specs = model_specs(vision, answer_spaces, num_attention_blocks, d)
    out = OrderedDict()
    for k, s in specs.items():
        if keys is not None and k not in keys:
            continue
        out[k] = init_param(k, s, seed, vision, d)
    return out


def make_batch(batch: int, seq_len: int, image_size: int, seed: int = 1, answer_spaces: int = 170,
               full_length: bool = False) -> dict:
    """Synthetic batch dict matching `DaquarFasterRcnnT5CollateFn.__call__`
    (`dataset_utils/resnet_vqa_daquar_dataset.py:197-227`) as numpy arrays."""
    g = np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, 0x5A17]))
    images = g.random((batch, 3, image_size, image_size), dtype=np.float32)
    ids = np.zeros((batch, seq_len), dtype=np.int64)
    mask = np.zeros((batch, seq_len), dtype=np.int64)
    lo = min(6, seq_len)
    for b in range(batch):
        ell = seq_len if full_length else int(g.integers(lo, seq_len + 1))
        ids[b, 0] = QUESTION_TOKEN
        if ell > 2:
            ids[b, 1:ell - 1] = g.integers(2, 32100, size=ell - 2)
        ids[b, ell - 1] = 1
        mask[b, :ell] = 1
    targets = g.integers(0, answer_spaces, size=batch).astype(np.int64)
    dec_len = 20
    return {
        "question_input_ids": ids,
        "decoder_question_input_ids": np.zeros((batch, dec_len), dtype=np.int64),
        "question_attention_masks": mask,
        "decoder_question_attention_masks": np.zeros((batch, dec_len), dtype=np.int64),
        "annotation_ids": targets,
        "pixel_values": None,
        "image_tensors": images,
        "question_type_ids": None,
        "answer_input_ids": np.zeros((batch, dec_len), dtype=np.int64),
        "answer_attention_masks": np.zeros((batch, dec_len), dtype=np.int64),
    }
