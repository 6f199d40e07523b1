"""Golden fixtures of BASELINE config 4 from the REFERENCE `VitVQAModel`
(model/vit_vqa_model.py:127-227; build container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_vit.py

Recipe (as make_golden.py):
  * `/root/reference` on sys.path (read-only; bytecode writing disabled);
  * torchvision is absent: a stub module answers the reference's
    `from torchvision.models.detection import fasterrcnn_resnet50_fpn` (unused there);
  * `ViTModel.from_pretrained("google/vit-base-patch16-224-in21k")` -> ViTModel(ViTConfig())
    (the in21k base config: 768 / 12 layers / 12 heads / 3072 / GELU / eps 1e-12) and
    `T5ForConditionalGeneration.from_pretrained("t5-base")` -> built from the t5-base
    T5Config; eager attention; no network;
  * weights from `vit_model.make_state_dict` (reference / transformers-4.34 key names),
    renamed to the installed transformers' ViT module names, loaded strictly.
The model runs in eval mode (dropout off).  The step restates the ViT trainer
(trainer/vit_vqa_trainer.py:300-322, 450-464): AdamW(amsgrad, wd 0.1) over the
vision (no gradients) / lang_model / fusing_layer / classification_layer groups,
clip_grad_norm_(1.0), get_linear_schedule_with_warmup.
"""
import os
import sys
import types

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import transformers  # noqa: E402  (must precede the stub)
from transformers import T5Config, T5ForConditionalGeneration, ViTConfig, ViTModel  # noqa: E402

tv = types.ModuleType("torchvision")
tvm = types.ModuleType("torchvision.models")
tvd = types.ModuleType("torchvision.models.detection")
tvd.fasterrcnn_resnet50_fpn = lambda *a, **k: None
tvm.detection = tvd
tv.models = tvm
sys.modules.update({"torchvision": tv, "torchvision.models": tvm, "torchvision.models.detection": tvd})

T5_BASE = dict(vocab_size=32128, d_model=768, d_kv=64, d_ff=3072, num_layers=12, num_decoder_layers=12,
               num_heads=12, relative_attention_num_buckets=32, relative_attention_max_distance=128,
               dropout_rate=0.1, layer_norm_epsilon=1e-6, feed_forward_proj="relu")


def _t5(cls, name, **kw):
    cfg = T5Config(**T5_BASE)
    cfg._attn_implementation = "eager"
    return cls(cfg)


def _vit(cls, name, **kw):
    cfg = ViTConfig()
    cfg._attn_implementation = "eager"
    return cls(cfg)


T5ForConditionalGeneration.from_pretrained = classmethod(_t5)
ViTModel.from_pretrained = classmethod(_vit)

sys.path.insert(0, "/root/reference")
from model.vit_vqa_model import VitVQAModel  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

vm = load_package().vit_model
torch.set_num_threads(os.cpu_count())
GROUPS = ("lang_model", "fusing_layer", "classification_layer")


def installed_vit_key(k):
    """reference (transformers 4.34) ViT key -> the installed transformers' module name."""
    if not k.startswith("vision_model.encoder.layer."):
        return k
    rest = k[len("vision_model.encoder.layer."):]
    i, tail = rest.split(".", 1)
    for a, b in (("attention.attention.query", "attention.q_proj"), ("attention.attention.key", "attention.k_proj"),
                 ("attention.attention.value", "attention.v_proj"), ("attention.output.dense", "attention.o_proj"),
                 ("intermediate.dense", "mlp.fc1"), ("output.dense", "mlp.fc2")):
        if tail.startswith(a):
            tail = b + tail[len(a):]
            break
    return f"vision_model.layers.{i}.{tail}"


def build_model():
    m = VitVQAModel("google/vit-base-patch16-224-in21k", "t5-base", answer_spaces=170)
    sd = vm.make_state_dict(seed=0)
    m.load_state_dict({installed_vit_key(k): torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    m.eval()
    return m


def group_norms(model):
    acc = {g: 0.0 for g in GROUPS}
    seen = set()
    for name, p in model.named_parameters():
        if p.grad is None or id(p) in seen:
            continue
        seen.add(id(p))
        acc[name.split(".", 1)[0]] += float(p.grad.double().pow(2).sum())
    return np.array([np.sqrt(acc[g]) for g in GROUPS])


def full_case(B, L, nsteps=3, warmup=2, total=20, seed=1):
    torch.manual_seed(0)
    model = build_model()
    groups = [{"params": model.vision_model.parameters(), "lr": 0.008},
              {"params": model.lang_model.parameters(), "lr": 0.005},
              {"params": model.fusing_layer.parameters(), "lr": 1e-5},
              {"params": model.classification_layer.parameters(), "lr": 1e-5}]
    opt = torch.optim.AdamW(groups, weight_decay=0.1, amsgrad=True)
    sched = transformers.get_linear_schedule_with_warmup(opt, num_warmup_steps=warmup, num_training_steps=total)
    nb = vm.make_batch(B, L, seed=seed)
    batch = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
    out = {"B": B, "L": L, "warmup": warmup, "total": total,
           "pix_sum": np.array([nb["pixel_values"].astype(np.float64).sum()]),
           "ids": nb["question_input_ids"], "dec_ids": nb["decoder_question_input_ids"],
           "dec_mask": nb["decoder_question_attention_masks"], "targets": nb["annotation_ids"]}
    with torch.no_grad():
        out["vit_pooled"] = model.vision_model(batch["pixel_values"]).pooler_output.numpy()
    losses, norms, gnorms = [], [], []
    params = [p for p in model.parameters()]
    for s in range(nsteps):
        opt.zero_grad()
        lp, loss = model(**batch)
        loss.backward()
        if s == 0:
            out["log_probs"] = lp.detach().numpy()
        gnorms.append(group_norms(model))
        gn = torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        sched.step()
        losses.append(float(loss))
        norms.append(float(gn))
    out["losses"] = np.array(losses)
    out["grad_norms"] = np.array(norms)
    out["group_grad_norms"] = np.array(gnorms)
    sd = model.state_dict()
    out["post_cls_w"] = sd["classification_layer.weight"][:4, :16].numpy().copy()
    out["post_fuse_w"] = sd["fusing_layer.0.weight"][:4, :16].numpy().copy()
    out["post_dec_wi0"] = sd["lang_model.decoder.block.0.layer.2.DenseReluDense.wi.weight"][:4, :16].numpy().copy()
    out["post_dec_xv0"] = sd["lang_model.decoder.block.0.layer.1.EncDecAttention.v.weight"][:4, :16].numpy().copy()
    out["post_enc_q0"] = sd["lang_model.encoder.block.0.layer.0.SelfAttention.q.weight"][:4, :16].numpy().copy()
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "vit_model_b4_l16.npz"), **full_case(4, 16))
    print("vit done", flush=True)


if __name__ == "__main__":
    main()
