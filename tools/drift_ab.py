"""A/B for the bf16 engine's trajectory drift against the fp32 golden:
the CPU oracle run twice on the golden R50 batch (B = 4, 224 x 224, L = 32, 3 eval-mode steps,
the golden's warm-up / schedule) -- once in fp32, once with every Linear GEMM of the T5 encoder
and SGA blocks on bf16-rounded operands (forward x, W; backward dY, W and dY, X: the engine's
GEMM inputs) -- and both compared with the reference's own golden trajectory
(tests/golden/model_r50_224_l32.npz).  If the bf16-operand oracle drifts from the golden as the
engine does (grad-norm rel 2.3e-4 at step 0, 1.13e-2 at step 3: profiles/r02_parity_report.json),
the drift is bf16 arithmetic amplified by AdamW, not an engine defect.

  python tools/drift_ab.py [OUT.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from oracle import vqa_oracle as orc  # noqa: E402

torch.set_num_threads(os.cpu_count())


def r16(t):
    return t.bfloat16().float()


class _Bf16Matmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return r16(x) @ r16(w).T

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        d = r16(dy)
        return d @ r16(w), d.reshape(-1, d.shape[-1]).T @ r16(x).reshape(-1, x.shape[-1])


class _Bf16ConvT(torch.autograd.Function):
    """ConvTranspose2d on bf16-rounded operands (the engine's layer4 map and scaler weight are
    bf16 GEMM operands; its dW reads the bf16 map and the bf16 vision-token gradient)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _CT(r16(x), r16(w), b, stride=1, padding=1)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        xr, wr, dr = r16(x).requires_grad_(False), r16(w).requires_grad_(True), r16(dy)
        with torch.enable_grad():
            y = _CT(xr, wr, None, stride=1, padding=1)
            (dw,) = torch.autograd.grad(y, wr, dr)
        return None, dw, dy.sum((0, 2, 3))


F = torch.nn.functional
_CT = F.conv_transpose2d                  # the unpatched op (the A/B swaps the module attribute)
S = load_package().synthetic
g = np.load(os.path.join(ROOT, "tests", "golden", "model_r50_224_l32.npz"))
B, L, H = int(g["B"]), int(g["L"]), int(g["H"])
sd = S.make_state_dict("resnet50", seed=0)
batch = orc.to_torch_batch(S.make_batch(B, L, H, seed=1))
fp32_mm, fp32_ct, fp32_res = orc._mm, orc.F.conv_transpose2d, orc.resnet_features
out = {}
for mode in ("fp32", "bf16_gemm_operands", "bf16_gemm_operands+features+convT"):
    orc._mm = fp32_mm if mode == "fp32" else (lambda x, w, fp8=False: _Bf16Matmul.apply(x, w))
    full = mode.endswith("convT")
    orc.resnet_features = (lambda *a, **k: r16(fp32_res(*a, **k))) if full else fp32_res
    orc.F.conv_transpose2d = (lambda x, w, b, stride=1, padding=1: _Bf16ConvT.apply(x, w, b)) if full else fp32_ct
    tr = orc.OracleTrainer(sd, "resnet50", warmup=int(g["warmup"]), total=int(g["total"]))
    losses, norms, groups = [], [], []
    for s in range(len(g["losses"])):
        _, loss = tr.forward_backward(batch)
        gg = tr.group_grad_norms()
        groups.append([gg[k] for k in ("lang_model", "scaler", "sga_modules", "attention_pooler",
                                       "classification_layer")])
        norms.append(float(tr.clip_and_step()))
        losses.append(float(loss))
    out[mode] = {"group_grad_norm_rel_vs_golden": (np.abs(np.array(groups) - g["group_grad_norms"])
                                                   / g["group_grad_norms"]).tolist(),
                 "loss_rel_vs_golden": (np.abs(np.array(losses) - g["losses"]) / np.abs(g["losses"])).tolist(),
                 "grad_norm_rel_vs_golden": (np.abs(np.array(norms) - g["grad_norms"]) / g["grad_norms"]).tolist()}
    print(mode, json.dumps(out[mode]), flush=True)
orc._mm, orc.F.conv_transpose2d, orc.resnet_features = fp32_mm, fp32_ct, fp32_res
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
