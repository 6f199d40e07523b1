"""Accuracy of the folded RMSNorm (VQA_NORM_FOLD) against the fp32 CPU oracle: the same
eval-mode step (B = 4, L = 16, R34 @ 256, the golden R34 case) with and without it; relative
L2 error of T5 weight gradients (whole tensor and the golden test's [:4, :16] q slice)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from oracle import vqa_oracle as orc  # noqa: E402

pkg = load_package()
vision, B, L, H = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else \
    ("resnet34", 4, 16, 256)
sd = pkg.synthetic.make_state_dict(vision, seed=0)
nb = pkg.synthetic.make_batch(B, L, H, seed=1)
ot = orc.OracleTrainer(sd, vision, warmup=2, total=10, dropout=0.0)
olp, oloss = ot.forward_backward(orc.to_torch_batch(nb))
D = 768


def og(i, w):
    p = f"lang_model.block.{i}."
    if w == "q":
        return ot.sd[p + "layer.0.SelfAttention.q.weight"].grad
    if w == "k":
        return ot.sd[p + "layer.0.SelfAttention.k.weight"].grad
    if w == "wi":
        return ot.sd[p + "layer.1.DenseReluDense.wi.weight"].grad
    if w == "ln0":
        return ot.sd[p + "layer.0.layer_norm.weight"].grad
    return ot.sd[p + "layer.1.DenseReluDense.wo.weight"].grad


def eg(e, i, w):
    if w == "q":
        return e.segment_grad(f"t5.{i}.qkv_w")[:D].cpu()
    if w == "k":
        return e.segment_grad(f"t5.{i}.qkv_w")[D:2 * D].cpu()
    if w == "ln0":
        return e.segment_grad(f"t5.{i}.ln0").cpu()
    return e.segment_grad(f"t5.{i}.{w}").cpu()


def rel(a, b):
    a, b = a.double().reshape(b.shape), b.double()
    return float((a - b).norm() / b.norm())


for v in ("0", "1"):
    os.environ["VQA_NORM_FOLD"] = v
    e = pkg.engine.VQAEngine(sd, vision=vision, batch=B, seq_len=L, image_size=H, warmup=2, total=10, dropout=0.0)
    lp, loss = e.forward_backward(nb)
    line = [f"fold={v}: loss rel {abs(loss - float(oloss)) / abs(float(oloss)):.2e} lp {float(np.abs(lp - olp.numpy()).max()):.2e}"]
    for i in (0, 1, 6, 11):
        for w in ("q", "k", "wi", "wo", "ln0"):
            line.append(f"{w}{i} {rel(eg(e, i, w), og(i, w)):.3f}")
    q0 = rel(eg(e, 0, "q").reshape(D, D)[:4, :16], og(0, "q")[:4, :16])
    line.append(f"q0[:4,:16] {q0:.3f}")
    print(" ".join(line), flush=True)
    del e
    torch.cuda.empty_cache()
