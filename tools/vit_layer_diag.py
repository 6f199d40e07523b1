"""Where the config-4 engine's frozen-ViT error comes from: the engine's residual stream after
each of the 12 ViT layers (VH32), its pooled output, and layer 0's attention output, against the
fp32 oracle (oracle/vit_oracle.py) and against the same oracle on bf16-rounded matmul operands
(tools/drift_ab_vit.py Bf16Operands: what bf16 MFMA inputs alone explain), on the golden batch
(B = 4, L = 16).

  python tools/vit_layer_diag.py [OUT.json]"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from drift_ab_vit import Bf16Operands, load_package, orc  # noqa: E402

F = torch.nn.functional
pkg = load_package()
vm = pkg.vit_model
B, L = 4, 16
nb = vm.make_batch(B, L, seed=1)
sd = {k: torch.as_tensor(v) for k, v in vm.make_state_dict(seed=0).items()}
eng = pkg.vit_engine.VitVQAEngine(vm.make_state_dict(seed=0), batch=B, seq_len=L, dropout=0.0)
eng.load_batch(nb)


def oracle_layers(pix):
    """vit_pooled with the residual stream after every layer and layer 0's attention context."""
    g = lambda k: sd["vision_model." + k]
    x = F.conv2d(pix, g("embeddings.patch_embeddings.projection.weight"),
                 g("embeddings.patch_embeddings.projection.bias"), stride=16)
    x = x.flatten(2).transpose(1, 2)
    x = torch.cat([g("embeddings.cls_token").expand(B, -1, -1), x], dim=1) + g("embeddings.position_embeddings")
    n_ = x.shape[1]
    hs, ctx0 = [], None
    for i in range(12):
        p = f"encoder.layer.{i}."
        n = F.layer_norm(x, (768,), g(p + "layernorm_before.weight"), g(p + "layernorm_before.bias"), 1e-12)
        qkv = [(n @ g(p + f"attention.attention.{t}.weight").T + g(p + f"attention.attention.{t}.bias"))
               .view(B, n_, 12, 64).transpose(1, 2) for t in ("query", "key", "value")]
        s = qkv[0] @ qkv[1].transpose(2, 3) / 8.0
        ctx = (torch.softmax(s, dim=-1) @ qkv[2]).transpose(1, 2).reshape(B, n_, 768)
        if i == 0:
            ctx0 = ctx
        x = ctx @ g(p + "attention.output.dense.weight").T + g(p + "attention.output.dense.bias") + x
        n = F.layer_norm(x, (768,), g(p + "layernorm_after.weight"), g(p + "layernorm_after.bias"), 1e-12)
        f = F.gelu(n @ g(p + "intermediate.dense.weight").T + g(p + "intermediate.dense.bias"))
        x = f @ g(p + "output.dense.weight").T + g(p + "output.dense.bias") + x
        hs.append(x)
    pooled = orc.vit_pooled(sd, pix)
    return hs, ctx0, pooled


pix = torch.as_tensor(nb["pixel_values"])
with torch.no_grad():
    h32, c32, p32 = oracle_layers(pix)
    with Bf16Operands():
        h16, c16, p16 = oracle_layers(pix)


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


s = pkg.lib.stream_handle()
out = {"layers": []}
for i in range(12):
    end = eng._vit_attn_at[i] + 4                         # o-proj, ln2, fc1, fc2 follow the attention
    for c in eng.fwd_calls[:end]:
        c(s)
    torch.cuda.synchronize()
    vh = eng.VH32.view(B, -1, 768).cpu()
    row = {"layer": i, "engine_vs_fp32": rel(vh, h32[i]), "engine_vs_bf16ops": rel(vh, h16[i]),
           "bf16ops_vs_fp32": rel(h16[i], h32[i])}
    if i == 0:
        for c in eng.fwd_calls[:eng._vit_attn_at[0]]:
            c(s)
        torch.cuda.synchronize()
        vo = eng.VO16.float().view(B, -1, 768).cpu()
        row.update({"ctx0_engine_vs_fp32": rel(vo, c32), "ctx0_engine_vs_bf16ops": rel(vo, c16),
                    "ctx0_bf16ops_vs_fp32": rel(c16, c32)})
    out["layers"].append(row)
    print(json.dumps(row), flush=True)
for c in eng.fwd_calls[:eng.vit_calls]:
    c(s)
torch.cuda.synchronize()
pe = eng.vit_pooled().cpu()
out["pooled"] = {"engine_vs_fp32": rel(pe, p32), "engine_vs_bf16ops": rel(pe, p16), "bf16ops_vs_fp32": rel(p16, p32)}
print(json.dumps(out["pooled"]), flush=True)
# ---- layer 0 op by op: each engine op against fp32 / bf16-operand math on the ENGINE's own
# inputs (so every op's own error is isolated); relative L2 over the whole tensor
def rl2(a, b):
    return float((a - b).norm() / b.norm())


def upto(n):
    for c in eng.fwd_calls[:n]:
        c(s)
    torch.cuda.synchronize()


g = lambda k: sd["vision_model." + k].float()
p0 = "encoder.layer.0."
a0 = eng._vit_attn_at[0]                 # index of the o-projection; the attention is a0 - 1
steps = {}
upto(a0 - 3)                              # patch embedding + CLS / position rows -> VH32
x = eng.VH32.view(B, -1, 768).cpu().clone()
upto(a0 - 2)                              # ln1 -> VLN16
n16 = eng.VLN16.float().view(B, -1, 768).cpu()
ref = F.layer_norm(x, (768,), g(p0 + "layernorm_before.weight"), g(p0 + "layernorm_before.bias"), 1e-12)
steps["ln1"] = {"vs_fp32": rl2(n16, ref), "vs_fp32_rounded": rl2(n16, ref.bfloat16().float())}
upto(a0 - 1)                              # qkv GEMM -> VQKV16
qkv16 = eng.VQKV16.float().view(B, -1, 2304).cpu()
W = torch.cat([g(p0 + f"attention.attention.{t}.weight") for t in ("query", "key", "value")])
bq = torch.cat([g(p0 + f"attention.attention.{t}.bias") for t in ("query", "key", "value")])
ref = n16 @ W.T + bq
ref16 = n16 @ W.bfloat16().float().T + bq
steps["qkv"] = {"vs_fp32": rl2(qkv16, ref), "vs_bf16ops": rl2(qkv16, ref16),
                "vs_bf16ops_rounded": rl2(qkv16, ref16.bfloat16().float())}
upto(a0)                                  # attention -> VO16
o16 = eng.VO16.float().view(B, -1, 768).cpu()
q, k, v = (qkv16[..., j * 768:(j + 1) * 768].reshape(B, -1, 12, 64).transpose(1, 2) for j in range(3))
P = torch.softmax(q @ k.transpose(2, 3) / 8.0, -1)
ref = (P @ v).transpose(1, 2).reshape(B, -1, 768)
ref16 = (P.bfloat16().float() @ v).transpose(1, 2).reshape(B, -1, 768)
steps["attention"] = {"vs_fp32": rl2(o16, ref), "vs_bf16P": rl2(o16, ref16),
                      "fp32_rounded_vs_fp32": rl2(ref.bfloat16().float(), ref)}
upto(a0 + 1)                              # o-proj + bias + residual -> VH32
h = eng.VH32.view(B, -1, 768).cpu().clone()
ref = o16 @ g(p0 + "attention.output.dense.weight").T + g(p0 + "attention.output.dense.bias") + x
ref16 = o16 @ g(p0 + "attention.output.dense.weight").bfloat16().float().T + g(p0 + "attention.output.dense.bias") + x
steps["o_proj"] = {"vs_fp32": rl2(h - x, ref - x), "vs_bf16ops": rl2(h - x, ref16 - x)}
upto(a0 + 2)                              # ln2 -> VLN16
n16 = eng.VLN16.float().view(B, -1, 768).cpu()
ref = F.layer_norm(h, (768,), g(p0 + "layernorm_after.weight"), g(p0 + "layernorm_after.bias"), 1e-12)
steps["ln2"] = {"vs_fp32": rl2(n16, ref), "vs_fp32_rounded": rl2(n16, ref.bfloat16().float())}
upto(a0 + 3)                              # fc1 + GELU -> VFF16
f16 = eng.VFF16.float().view(B, -1, 3072).cpu()
ref = F.gelu(n16 @ g(p0 + "intermediate.dense.weight").T + g(p0 + "intermediate.dense.bias"))
ref16 = F.gelu(n16 @ g(p0 + "intermediate.dense.weight").bfloat16().float().T + g(p0 + "intermediate.dense.bias"))
steps["fc1_gelu"] = {"vs_fp32": rl2(f16, ref), "vs_bf16ops": rl2(f16, ref16),
                     "vs_bf16ops_rounded": rl2(f16, ref16.bfloat16().float())}
upto(a0 + 4)                              # fc2 + bias + residual -> VH32
h2 = eng.VH32.view(B, -1, 768).cpu().clone()
ref = f16 @ g(p0 + "output.dense.weight").T + g(p0 + "output.dense.bias") + h
ref16 = f16 @ g(p0 + "output.dense.weight").bfloat16().float().T + g(p0 + "output.dense.bias") + h
steps["fc2"] = {"vs_fp32": rl2(h2 - h, ref - h), "vs_bf16ops": rl2(h2 - h, ref16 - h)}
out["layer0_ops_rel_l2"] = steps
for k_, v_ in steps.items():
    print(k_, json.dumps(v_), flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
