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
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
