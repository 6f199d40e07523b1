"""What row-wise e4m3 forward GEMMs cost against fp32 (BASELINE configs[4] "fp8 MFMA weights"):
the CPU oracle with and without its fp8 restatement (oracle/vqa_oracle.py fp8_rows / _Fp8Matmul)
on the config-5 golden batch (R50, t5-large, 6 SGA blocks at 1024, 384 x 384, B = 4), three
eval-mode steps.  The differences calibrate the fp8 engine's tolerance against the fp32 golden
(tests/test_config5_gpu.py); the engine is checked tightly against the fp8 oracle itself.

  python tools/fp8_calibrate.py [OUT.json]"""
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
S = load_package().synthetic
B, L, H = 4, 32, 384
sd = S.make_state_dict("resnet50", seed=0, num_attention_blocks=6, language_model="t5-large")
batch = orc.to_torch_batch(S.make_batch(B, L, H, seed=1))
res = {}
for fp8 in (False, True):
    tr = orc.OracleTrainer(sd, "resnet50", warmup=2, total=20, num_blocks=6, fp8=fp8)
    steps = []
    for s in range(3):
        lp, loss = tr.forward_backward(batch)
        gg = tr.group_grad_norms()
        gn = float(tr.clip_and_step())
        steps.append({"lp": lp.numpy().tolist(), "loss": float(loss), "gn": gn, "groups": dict(gg)})
    res[fp8] = steps
    print("fp8" if fp8 else "fp32", [(round(x["loss"], 6), round(x["gn"], 5)) for x in steps], flush=True)
out = {"batch": [B, L, H], "steps": []}
for a, b in zip(res[False], res[True]):
    out["steps"].append({
        "log_prob_max_abs": float(np.abs(np.array(a["lp"]) - np.array(b["lp"])).max()),
        "loss_rel": abs(a["loss"] - b["loss"]) / abs(a["loss"]),
        "grad_norm_rel": abs(a["gn"] - b["gn"]) / a["gn"],
        "group_grad_norm_rel": {g: abs(a["groups"][g] - b["groups"][g]) / a["groups"][g] for g in a["groups"]}})
print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
