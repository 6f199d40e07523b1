"""Generate the golden fixtures from the REFERENCE modules (build container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Recipe:
  * `/root/reference` on sys.path (read-only; bytecode writing disabled);
  * transformers imported before the torchvision stub (it probes
    torchvision.__spec__ at import time);
  * `torchvision.models` -> tests/golden/tv_stub.py (torchvision is absent);
  * `T5ForQuestionAnswering.from_pretrained` -> build from a local t5-base
    `T5Config` (no network), eager attention;
  * weights from `synthetic.make_state_dict` loaded with load_state_dict(strict).
The model runs in eval mode (dropout off, Q7).  The training step restates
`faster_rcnn_vqa_trainer.py:391-406` with torch's own clip_grad_norm_,
AdamW(amsgrad) over the trainer's 6 groups (`:231-267`) and transformers'
get_linear_schedule_with_warmup (`:279-287`).

Only outputs, norms and hashes are stored (no weights): the tests regenerate
weights and batches from the same seeds and check the batch hashes.
"""
import hashlib
import os
import sys
import types

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import transformers  # noqa: E402  (must precede the stub)
from transformers import T5Config, T5ForQuestionAnswering  # noqa: E402

sys.path.insert(0, HERE)
import tv_stub  # noqa: E402

tv = types.ModuleType("torchvision")
tvm = types.ModuleType("torchvision.models")
for n in ("resnet18", "resnet34", "resnet50"):
    setattr(tvm, n, getattr(tv_stub, n))
tv.models = tvm
sys.modules["torchvision"] = tv
sys.modules["torchvision.models"] = tvm

T5_BASE = dict(vocab_size=32128, d_model=768, d_kv=64, d_ff=3072, num_layers=12, num_decoder_layers=12,
               num_heads=12, relative_attention_num_buckets=32, relative_attention_max_distance=128,
               dropout_rate=0.1, layer_norm_epsilon=1e-6, feed_forward_proj="relu")
# t5-large (BASELINE configs[4]): the published t5-large hyper-parameters
T5_LARGE = dict(T5_BASE, d_model=1024, d_ff=4096, num_layers=24, num_decoder_layers=24, num_heads=16)


def _from_pretrained(cls, name, **kw):
    cfg = T5Config(**T5_BASE)
    cfg._attn_implementation = "eager"
    return cls(cfg)


T5ForQuestionAnswering.from_pretrained = classmethod(_from_pretrained)

sys.path.insert(0, "/root/reference")
from model.resnet_vqa_model import AttentionPooler, ResnetVQAModel  # noqa: E402
from model.multi_head_vision_text_attn import SGA, ImageConfiguration, TextConfiguration  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

syn = load_package().synthetic
torch.set_num_threads(os.cpu_count())


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def tb(np_batch):
    return {k: (None if v is None else torch.as_tensor(v)) for k, v in np_batch.items()}


def build_model(vision):
    m = ResnetVQAModel(vision, "t5-base", answer_spaces=170)
    sd = syn.make_state_dict(vision, seed=0)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    m.eval()
    return m


def optimizer_groups(model):
    """faster_rcnn_vqa_trainer.py:231-267 with vit_daquar_config.json lrs."""
    groups = [
        {"params": model.vision_model.parameters(), "lr": 0.008},
        {"params": model.lang_model.parameters(), "lr": 0.005},
        {"params": (model.downscale_layer if model.vision_model_name == "resnet50"
                    else model.upscale_layer).parameters(), "lr": 0.0005},
        {"params": model.sga_modules.parameters(), "lr": 0.0005},
        {"params": model.attention_pooler.parameters(), "lr": 0.0005},
        {"params": model.classification_layer.parameters(), "lr": 1e-5},
    ]
    return torch.optim.AdamW(groups, weight_decay=0.1, amsgrad=True)


GROUPS = ("lang_model", "scaler", "sga_modules", "attention_pooler", "classification_layer")


def group_norms(model):
    acc = {g: 0.0 for g in GROUPS}
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        top = name.split(".", 1)[0]
        g = "scaler" if top in ("upscale_layer", "downscale_layer") else top
        acc[g] += float(p.grad.double().pow(2).sum())
    return np.array([np.sqrt(acc[g]) for g in GROUPS])


def full_model_case(vision, B, L, H, nsteps=3, warmup=2, total=20, seed=1, builder=None, blocks=3, lm="t5-base"):
    torch.manual_seed(0)
    model = build_model(vision) if builder is None else builder()
    opt = optimizer_groups(model)
    sched = transformers.get_linear_schedule_with_warmup(opt, num_warmup_steps=warmup, num_training_steps=total)
    nb = syn.make_batch(B, L, H, seed=seed)
    batch = tb(nb)
    out = {"image_sha": sha(nb["image_tensors"]), "ids": nb["question_input_ids"],
           "mask": nb["question_attention_masks"], "targets": nb["annotation_ids"],
           "B": B, "L": L, "H": H, "warmup": warmup, "total": total}
    losses, norms, gnorms = [], [], []
    for s in range(nsteps):
        opt.zero_grad()
        lp, loss = model(**batch)
        loss.backward()
        if s == 0:
            out["log_probs"] = lp.detach().numpy()
            # features of the frozen ResNet (first step only)
            _, _, fmap = model.generate_answers(**{k: v for k, v in batch.items() if k != "annotation_ids"})
            f = fmap["features"].detach().numpy()
            out["feat_sum"] = np.array([f.sum(), np.abs(f).sum(), (f * f).sum()], dtype=np.float64)
            out["feat_slice"] = f[:, :8, :, :].copy()
        gnorms.append(group_norms(model))
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
        losses.append(float(loss))
        norms.append(float(gn))
    out["losses"] = np.array(losses)
    out["grad_norms"] = np.array(norms)
    out["group_grad_norms"] = np.array(gnorms)
    # parameter state after nsteps: per-group checksums + a few slices
    sd = model.state_dict()
    out["post_t5_q0"] = sd["lang_model.block.0.layer.0.SelfAttention.q.weight"][:4, :16].numpy().copy()
    out["post_cls_w"] = sd["classification_layer.weight"][:4, :16].numpy().copy()
    out["post_sga_fc1"] = sd[f"sga_modules.{blocks - 1}.ffn.mlp.fc1.weight"][:4, :16].numpy().copy()
    scaler = "downscale_layer" if vision == "resnet50" else "upscale_layer"
    out["post_scaler_w"] = sd[scaler + ".weight"][:4, :4].numpy().copy()
    init = syn.make_state_dict(vision, seed=0, num_attention_blocks=blocks, language_model=lm)
    delta = {g: 0.0 for g in GROUPS}
    for k, v in sd.items():
        if k.startswith("vision_model"):
            continue
        top = k.split(".", 1)[0]
        g = "scaler" if top in ("upscale_layer", "downscale_layer") else top
        delta[g] += float(np.abs(v.numpy().astype(np.float64) - init[k]).sum())
    out["group_abs_delta"] = np.array([delta[g] for g in GROUPS])
    return out


def sga_case():
    torch.manual_seed(0)
    blk = SGA(ImageConfiguration(), TextConfiguration())
    sd = {k[len("sga_modules.0."):]: torch.as_tensor(v)
          for k, v in syn.make_state_dict("resnet50", seed=0).items() if k.startswith("sga_modules.0.")}
    blk.load_state_dict(sd, strict=True)
    blk.eval()
    g = np.random.Generator(np.random.PCG64(7))
    x = torch.tensor(g.standard_normal((2, 32, 768), dtype=np.float32), requires_grad=True)
    y = torch.tensor(g.standard_normal((2, 49, 768), dtype=np.float32), requires_grad=True)
    out = blk(x, y)
    gout = torch.tensor(g.standard_normal((2, 32, 768), dtype=np.float32))
    (out * gout).sum().backward()
    pn = np.array([float(p.grad.norm()) for _, p in blk.named_parameters()])
    return {"x": x.detach().numpy(), "y": y.detach().numpy(), "gout": gout.numpy(), "out": out.detach().numpy(),
            "dx": x.grad.numpy(), "dy": y.grad.numpy(), "param_grad_norms": pn,
            "param_names": np.array([n for n, _ in blk.named_parameters()])}


def t5_case():
    torch.manual_seed(0)
    model = build_model("resnet50")
    enc = model.lang_model
    nb = syn.make_batch(2, 32, 32, seed=3)
    ids, mask = torch.as_tensor(nb["question_input_ids"]), torch.as_tensor(nb["question_attention_masks"])
    h = enc(input_ids=ids, attention_mask=mask).last_hidden_state
    from transformers.models.t5.modeling_t5 import T5Attention
    rel = torch.arange(-40, 41)
    buckets = T5Attention._relative_position_bucket(rel, bidirectional=True, num_buckets=32, max_distance=128)
    return {"ids": nb["question_input_ids"], "mask": nb["question_attention_masks"], "hidden": h.detach().numpy(),
            "rel": rel.numpy(), "buckets": buckets.numpy()}


# --------------------------------------------------------------------------- config 5 (width 1024)
def wide_configs(hidden=1024):
    """The reference SGA reads its widths from configuration INSTANCES
    (multi_head_vision_text_attn.py:7-24, 128-143): instances with HIDDEN_SIZE 1024 (8 heads of
    128, FF 1024) give the reference's own SGA at T5-large width; no reference file changes."""
    cfgs = []
    for cls in (ImageConfiguration, TextConfiguration):
        c = cls()
        c.HIDDEN_SIZE, c.FF_SIZE = hidden, hidden
        c.HIDDEN_SIZE_HEAD = c.HIDDEN_SIZE // c.MULTI_HEAD
        cfgs.append(c)
    return cfgs


def t5_large_encoder():
    cfg = T5Config(**T5_LARGE)
    cfg._attn_implementation = "eager"
    return T5ForQuestionAnswering(cfg).encoder


def build_model_c5(num_blocks=6):
    """ResnetVQAModel at config-5 width: the reference class with its width-dependent children
    replaced by the same module types at d = 1024 (resnet_vqa_model.py:60-89 hard-codes 768
    only in these constructors); the reference forward() runs unchanged."""
    m = ResnetVQAModel("resnet50", "t5-base", answer_spaces=170, num_attention_blocks=num_blocks)
    img_c, txt_c = wide_configs()
    m.lang_model = t5_large_encoder()
    m.upscale_layer = torch.nn.ConvTranspose2d(512, 1024, kernel_size=3, stride=1, padding=1)
    m.downscale_layer = torch.nn.ConvTranspose2d(2048, 1024, kernel_size=3, stride=1, padding=1)
    m.sga_modules = torch.nn.ModuleList([SGA(img_c, txt_c) for _ in range(num_blocks)])
    m.classification_layer = torch.nn.Linear(1024, 170)
    m.attention_pooler = AttentionPooler(1024)
    sd = syn.make_state_dict("resnet50", seed=0, num_attention_blocks=num_blocks, language_model="t5-large")
    m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    m.eval()
    return m


def sga1024_case():
    torch.manual_seed(0)
    blk = SGA(*wide_configs())
    sd = {k[len("sga_modules.0."):]: torch.as_tensor(v)
          for k, v in syn.make_state_dict("resnet50", seed=0, language_model="t5-large").items()
          if k.startswith("sga_modules.0.")}
    blk.load_state_dict(sd, strict=True)
    blk.eval()
    g = np.random.Generator(np.random.PCG64(8))
    x = torch.tensor(g.standard_normal((2, 32, 1024), dtype=np.float32), requires_grad=True)
    y = torch.tensor(g.standard_normal((2, 144, 1024), dtype=np.float32), requires_grad=True)   # 384^2: 12 x 12
    out = blk(x, y)
    gout = torch.tensor(g.standard_normal((2, 32, 1024), dtype=np.float32))
    (out * gout).sum().backward()
    pn = np.array([float(p.grad.norm()) for _, p in blk.named_parameters()])
    return {"x": x.detach().numpy(), "y": y.detach().numpy(), "gout": gout.numpy(), "out": out.detach().numpy(),
            "dx": x.grad.numpy(), "dy": y.grad.numpy(), "param_grad_norms": pn,
            "param_names": np.array([n for n, _ in blk.named_parameters()])}


def t5_large_case():
    torch.manual_seed(0)
    enc = t5_large_encoder()
    sd = syn.make_state_dict("resnet50", seed=0, language_model="t5-large")
    enc.load_state_dict({k[len("lang_model."):]: torch.as_tensor(v) for k, v in sd.items()
                         if k.startswith("lang_model.")}, strict=True)
    enc.eval()
    nb = syn.make_batch(2, 32, 32, seed=3)
    ids, mask = torch.as_tensor(nb["question_input_ids"]), torch.as_tensor(nb["question_attention_masks"])
    h = enc(input_ids=ids, attention_mask=mask).last_hidden_state
    return {"ids": nb["question_input_ids"], "mask": nb["question_attention_masks"], "hidden": h.detach().numpy()}


def main_c5(model_only=False):
    if not model_only:
        np.savez_compressed(os.path.join(HERE, "sga1024_block.npz"), **sga1024_case())
        print("sga1024 done", flush=True)
        np.savez_compressed(os.path.join(HERE, "t5_large_encoder.npz"), **t5_large_case())
        print("t5-large done", flush=True)
    np.savez_compressed(os.path.join(HERE, "model_c5_r50_384_l32.npz"),
                        **full_model_case("resnet50", 4, 32, 384, builder=build_model_c5, blocks=6,
                                          lm="t5-large"))
    print("config-5 model done", flush=True)


def main():
    os.makedirs(HERE, exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "sga_block.npz"), **sga_case())
    print("sga done", flush=True)
    np.savez_compressed(os.path.join(HERE, "t5_encoder.npz"), **t5_case())
    print("t5 done", flush=True)
    np.savez_compressed(os.path.join(HERE, "model_r50_224_l32.npz"), **full_model_case("resnet50", 4, 32, 224))
    print("r50 done", flush=True)
    np.savez_compressed(os.path.join(HERE, "model_r34_256_l16.npz"), **full_model_case("resnet34", 4, 16, 256))
    print("r34 done", flush=True)
    np.savez_compressed(os.path.join(HERE, "model_r18_256_l16.npz"), **full_model_case("resnet18", 4, 16, 256))
    print("r18 done", flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["c5"]:
        main_c5(model_only=sys.argv[2:] == ["model"])
    else:
        main()
