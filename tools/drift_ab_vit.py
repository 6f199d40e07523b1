"""Config 4 (VitVQAModel) drift A/B: is the engine's trajectory error
against the fp32 oracle bf16 arithmetic, or a defect?  The CPU oracle (oracle/vit_oracle.py) is
run with every matmul on bf16-rounded operands -- the frozen ViT's projections and attention,
the T5 encoder / decoder projections and attention, the fusing layer and the classifier, forward
and backward (dY, W and dY, X), and the patch-embedding convolution: the engine's MFMA inputs --
and compared with the fp32 oracle, at the two places the GPU tests measure:

  golden_b4: eval mode on the reference-written fixture's batch (B = 4, L = 16, 3 steps), per-step
             group grad norms of both oracles against the fixture's
             (test_vit_gpu.py::test_vit_engine_matches_reference_golden; the engine measured a
             step-2 lang_model error of 0.114 there);
  bench_b64: the benched configuration (B = 64, L = 32, decoder 20, dropout 0.1 / 0.5 from the
             shared hash), 3 steps: log-probs, loss, grad norms, groups and the per-group update
             rel-L2 of the bf16-operand oracle against the fp32 one (the engine measured log-probs
             0.100 at step 2 and update rel-L2 0.158 (T5) / 0.194 (fusing layer):
             test_z_vit_bench_step_gpu.py).

  python tools/drift_ab_vit.py OUT.json [b4|b64|both]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from oracle import vit_oracle as orc  # noqa: E402
from oracle.bf16_mode import Bf16Operands  # noqa: E402,F401  (re-exported for tools/)

torch.set_num_threads(min(16, os.cpu_count()))   # the GPU box shows the whole host
F = torch.nn.functional
GROUPS = ("lang_model", "fusing_layer", "classification_layer")


def updates(tr, p0):
    return {k: (tr.sd[k].detach() - p0[k]).double() for k in tr.keys}


def golden_b4(vm):
    fix = np.load(os.path.join(ROOT, "tests", "golden", "vit_model_b4_l16.npz"), allow_pickle=False)
    B, L = int(fix["B"]), int(fix["L"])
    nb = {k: (None if v is None else torch.as_tensor(v)) for k, v in vm.make_batch(B, L, seed=1).items()}
    out = {}
    for mode in ("fp32", "bf16_operands"):
        tr = orc.VitOracleTrainer(vm.make_state_dict(seed=0), warmup=int(fix["warmup"]), total=int(fix["total"]))
        groups, norms, losses = [], [], []
        for _ in range(len(fix["losses"])):
            if mode == "fp32":
                _, loss = tr.forward_backward(nb)
            else:
                with Bf16Operands():
                    _, loss = tr.forward_backward(nb)
            gg = tr.group_grad_norms()
            groups.append([gg[g] for g in GROUPS])
            norms.append(float(tr.clip_and_step()))
            losses.append(float(loss))
        out[mode] = {"group_grad_norm_rel_vs_golden": (np.abs(np.array(groups) - fix["group_grad_norms"])
                                                       / fix["group_grad_norms"]).tolist(),
                     "loss_rel_vs_golden": (np.abs(np.array(losses) - fix["losses"]) / np.abs(fix["losses"])).tolist(),
                     "grad_norm_rel_vs_golden": (np.abs(np.array(norms) - fix["grad_norms"])
                                                 / fix["grad_norms"]).tolist()}
        print("golden_b4", mode, json.dumps(out[mode]), flush=True)
    return out


def bench_b64(vm, B=64, L=32, Ld=20, steps=3):
    sd = vm.make_state_dict(seed=0)
    nbs = [{k: (None if v is None else torch.as_tensor(v)) for k, v in vm.make_batch(B, L, dec_len=Ld, seed=1 + i).items()}
           for i in range(steps)]
    runs = {}
    for mode in ("fp32", "bf16_operands"):
        t0 = time.time()
        tr = orc.VitOracleTrainer(sd, warmup=10, total=100000, dropout=0.1, seed=0)
        p0 = {k: tr.sd[k].detach().clone() for k in tr.keys}
        rec = []
        for i, nb in enumerate(nbs):
            tr.rng_counter = i                                  # the same dropout draws in both runs
            if mode == "fp32":
                lp, loss = tr.forward_backward(nb)
            else:
                with Bf16Operands():
                    lp, loss = tr.forward_backward(nb)
            gg = tr.group_grad_norms()
            gn = float(tr.clip_and_step())
            rec.append((lp.numpy(), float(loss), gn, {g: gg[g] for g in GROUPS}))
        runs[mode] = (rec, updates(tr, p0), tr)
        print("bench_b64", mode, f"{time.time() - t0:.0f} s", flush=True)
    (ra, ua, ta), (rb, ub, _) = runs["fp32"], runs["bf16_operands"]
    out = {}
    for i in range(steps):
        a, b = ra[i], rb[i]
        out[f"step{i}"] = {"log_prob_max_abs": float(np.abs(a[0] - b[0]).max()),
                           "loss_rel": abs(a[1] - b[1]) / abs(a[1]), "grad_norm_rel": abs(a[2] - b[2]) / a[2],
                           "group_grad_norm_rel": {g: abs(a[3][g] - b[3][g]) / a[3][g] for g in GROUPS}}
    delta = {}
    for g in GROUPS:
        num = den = 0.0
        for k in ua:
            if orc.group_of(k) != g:
                continue
            num += float(((ub[k] - ua[k]) ** 2).sum())
            den += float((ua[k] ** 2).sum())
        delta[g] = (num / den) ** 0.5 if den > 0 else 0.0
    out["update_rel_l2"] = delta
    print("bench_b64 bf16-operand oracle vs fp32 oracle", json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    vm = load_package().vit_model
    what = sys.argv[2] if len(sys.argv) > 2 else "both"
    res = {}
    if what in ("b4", "both"):
        res["golden_b4"] = golden_b4(vm)
    if what in ("b64", "both"):
        res["bench_b64"] = bench_b64(vm)
    json.dump(res, open(sys.argv[1], "w"), indent=1)
