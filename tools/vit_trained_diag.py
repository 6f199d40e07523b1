"""Where config 4's trained-path error comes from: the engine's step-0
gradients and intermediates of the trained part of `VitVQAModel` (T5 encoder, fusing layer, T5
decoder, answer gather, head) against the fp32 oracle and against the same oracle on
bf16-rounded matmul operands (tools/drift_ab_vit.py Bf16Operands), both fed the ENGINE's own
pooled ViT output (the frozen ViT is diagnosed by tools/vit_layer_diag.py), eval mode, on the
golden batch (B = 4, L = 16, decoder 20).

Per parameter tensor: relative L2 of engine vs fp32, bf16-operand vs fp32 and engine vs
bf16-operand; per intermediate the same.  A tensor whose engine error is far above the
bf16-operand oracle's is the defect.

  python tools/vit_trained_diag.py [OUT.json] [B L]"""
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from drift_ab_vit import Bf16Operands, load_package, orc  # noqa: E402
from oracle.vqa_oracle import t5_rmsnorm  # noqa: E402

F = torch.nn.functional
pkg = load_package()
vm = pkg.vit_model
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
L = int(sys.argv[3]) if len(sys.argv) > 3 else 16
nb = vm.make_batch(B, L, seed=1)
sd0 = vm.make_state_dict(seed=0)
eng = pkg.vit_engine.VitVQAEngine(sd0, batch=B, seq_len=L, dropout=0.0)
lp_e, loss_e = eng.forward_backward(nb)
torch.cuda.synchronize()
pooled = eng.vit_pooled().cpu()


def rl2(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    d = float(b.norm())
    return float((a - b).norm()) / d if d > 0 else float((a - b).norm())


def oracle_run(bf16):
    """model_forward (oracle/vit_oracle.py) restated with captures; returns (caps, grads)."""
    tr = orc.VitOracleTrainer(sd0, dropout=0.0)
    sd = tr.sd
    tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
    cap = {}

    def keep(name, t):
        if t.requires_grad:
            t.retain_grad()
        cap[name] = t
        return t

    ctxm = Bf16Operands() if bf16 else contextlib.nullcontext()
    with ctxm:
        enc = keep("enc_out", orc.t5_encoder(sd, tb["question_input_ids"], tb["question_attention_masks"]))
        cls = keep("cls", enc[:, 0, :])
        cat = torch.cat([pooled, cls], dim=1)
        pre = keep("fuse_pre", cat @ sd["fusing_layer.0.weight"].T + sd["fusing_layer.0.bias"])
        fused = keep("fused", F.relu(pre))
        g = lambda k: sd["lang_model.decoder." + k]
        ids, mask = tb["decoder_question_input_ids"], tb["decoder_question_attention_masks"]
        Ld = ids.shape[1]
        h = g("embed_tokens.weight")[ids]
        causal = (torch.arange(Ld)[None, :] <= torch.arange(Ld)[:, None]).float()
        ext = (1.0 - causal[None, None] * mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
        bias = orc.causal_position_bias(g("block.0.layer.0.SelfAttention.relative_attention_bias.weight"), Ld) + ext
        enc1 = fused.unsqueeze(1)
        for i in range(12):
            p = f"block.{i}.layer."
            n = t5_rmsnorm(h, g(p + "0.layer_norm.weight"))
            q, k, v = [(n @ g(p + f"0.SelfAttention.{t}.weight").T).view(B, Ld, 12, 64).transpose(1, 2) for t in "qkv"]
            a = torch.softmax((q @ k.transpose(2, 3) + bias).float(), dim=-1)
            o = keep(f"dec{i}.self_ctx", (a @ v).transpose(1, 2).reshape(B, Ld, 768))
            h = keep(f"dec{i}.h_self", h + o @ g(p + "0.SelfAttention.o.weight").T)
            v1 = keep(f"dec{i}.xv", enc1 @ g(p + "1.EncDecAttention.v.weight").T)
            ctx = v1.expand(B, Ld, 768)
            h = keep(f"dec{i}.h_cross", h + ctx @ g(p + "1.EncDecAttention.o.weight").T)
            n = t5_rmsnorm(h, g(p + "2.layer_norm.weight"))
            f = F.relu(n @ g(p + "2.DenseReluDense.wi.weight").T)
            h = keep(f"dec{i}.h_ff", h + f @ g(p + "2.DenseReluDense.wo.weight").T)
        dec = keep("dec_out", t5_rmsnorm(h, g("final_layer_norm.weight")))
        last = torch.max(torch.where(mask == 1, torch.arange(Ld), torch.zeros_like(mask)), dim=1).values
        ans = keep("ans", dec[torch.arange(B), last])
        lp = F.log_softmax(ans @ sd["classification_layer.weight"].T + sd["classification_layer.bias"], dim=-1)
        loss = F.nll_loss(lp, tb["annotation_ids"])
        loss.backward()
    grads = {k: (sd[k].grad.detach().clone() if sd[k].grad is not None else torch.zeros_like(sd[k])) for k in tr.keys}
    cap["log_probs"] = lp
    return cap, grads, float(loss)


c32, g32, l32 = oracle_run(False)
c16, g16, l16 = oracle_run(True)

# ---- engine intermediates (eager forward_backward above left them in place)
TD, T, Ld = eng.TD, eng.T, eng.Ld
ecap = {"log_probs": torch.as_tensor(lp_e),
        "enc_out": eng.TXT32.cpu().view(B, L, 768),
        "fused": eng.FUSED16.float().cpu(),
        "dec_out": eng.DEC32.cpu().view(B, Ld, 768),
        "ans": eng.ANS32.cpu()}
for i in range(12):
    ecap[f"dec{i}.h_self"] = eng.HM_d[i].cpu().view(B, Ld, 768)
    ecap[f"dec{i}.h_cross"] = eng.HX_d[i].cpu().view(B, Ld, 768)
    ecap[f"dec{i}.h_ff"] = eng.HS_d[i + 1].cpu().view(B, Ld, 768)
    ecap[f"dec{i}.xv"] = eng.VALL16[:, i * 768:(i + 1) * 768].float().cpu().view(B, 1, 768)
    ecap[f"dec{i}.self_ctx"] = eng.O_d[i].float().cpu().view(B, Ld, 768)
egrad = {"ans": eng.dANS32.cpu(), "fuse_pre": eng.dPRE16.float().cpu(), "cls": eng.dCLS32.cpu()}
for i in range(12):
    egrad[f"dec{i}.xv"] = eng.dVALL16[:, i * 768:(i + 1) * 768].float().cpu().view(B, 1, 768)

out = {"B": B, "L": L, "loss_rel": {"engine": abs(loss_e - l32) / abs(l32), "bf16ops": abs(l16 - l32) / abs(l32)},
       "forward": {}, "activation_grads": {}, "param_grads": {}}
for k, e in ecap.items():
    a, b = c32[k].detach(), c16[k].detach()
    out["forward"][k] = {"engine_vs_fp32": rl2(e, a), "bf16ops_vs_fp32": rl2(b, a), "engine_vs_bf16ops": rl2(e, b)}
for k, e in egrad.items():
    a, b = c32[k].grad, c16[k].grad
    if a is None:
        continue
    # the engine's dPRE16 is the gradient after the ReLU / dropout mask (= d pre-activation)
    out["activation_grads"][k] = {"engine_vs_fp32": rl2(e, a), "bf16ops_vs_fp32": rl2(b, a),
                                  "engine_vs_bf16ops": rl2(e, b)}
for k in g32:
    pv = eng.param_view(k)
    if pv is None:
        continue
    ge = pv[1].cpu()
    a, b = g32[k], g16[k]
    out["param_grads"][k] = {"engine_vs_fp32": rl2(ge, a), "bf16ops_vs_fp32": rl2(b, a),
                             "engine_vs_bf16ops": rl2(ge, b), "norm": float(a.norm())}


def show(sec):
    rows = sorted(out[sec].items(), key=lambda kv: -kv[1]["engine_vs_fp32"] / max(kv[1]["bf16ops_vs_fp32"], 1e-12))
    print(f"== {sec}: name  engine/fp32  bf16ops/fp32  engine/bf16ops", flush=True)
    for k, v in rows:
        print(f"{k:70s} {v['engine_vs_fp32']:.3e} {v['bf16ops_vs_fp32']:.3e} {v['engine_vs_bf16ops']:.3e}", flush=True)


print("loss rel", out["loss_rel"])
for sec in ("forward", "activation_grads", "param_grads"):
    show(sec)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
