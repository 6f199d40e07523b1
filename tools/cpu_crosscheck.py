"""SURVEY §8d cross-check (build container only: it imports the reference): the CPU oracle
restatement's step time against the reference's own step at the same shapes and step
definition -- BASELINE configs[1] shapes (R50, B = 64, 224 x 224, L = 32), train mode
(dropout 0.1), zero_grad + forward + backward + clip_grad_norm_(1.0) + AdamW(amsgrad) +
scheduler, torch CPU on this container's threads, median of 5 steps after 2 warm-ups.  The
reference is imported exactly as tests/golden/make_golden.py does (torchvision architecture
stub, locally configured t5-base).  The bench's cpu_baseline (kind "port") times the oracle on
the GPU box, where the reference cannot travel; this records how far that port is from the
reference itself.

  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_crosscheck.py OUT.json [B]"""
import json
import os
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402  (reference import recipe)
from oracle import vqa_oracle as orc  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
L, H, WARM, STEPS = 32, 224, 2, 5
threads = torch.get_num_threads()
nb = mg.syn.make_batch(B, L, H, seed=1)


def median_time(step):
    ts = []
    for i in range(WARM + STEPS):
        t0 = time.perf_counter()
        step()
        if i >= WARM:
            ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


# the reference: ResnetVQAModel in train mode, the trainer's optimizer groups and schedule
torch.manual_seed(0)
model = mg.build_model("resnet50")
model.train()
opt = mg.optimizer_groups(model)
sched = mg.transformers.get_linear_schedule_with_warmup(opt, num_warmup_steps=10, num_training_steps=1000)
batch = mg.tb(nb)


def ref_step():                                 # faster_rcnn_vqa_trainer.py:391-406
    opt.zero_grad()
    _, loss = model(**batch)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    sched.step()


t_ref, ts_ref = median_time(ref_step)
del model, opt
sd = mg.syn.make_state_dict("resnet50", seed=0)
tr = orc.OracleTrainer(sd, "resnet50", warmup=10, total=1000, dropout=0.1)
ob = orc.to_torch_batch(nb)
t_orc, ts_orc = median_time(lambda: tr.train_one_step(ob))
out = {"shapes": f"R50 + t5-base + 3xSGA, B={B}, {H}x{H}, L={L}, train mode (dropout 0.1)",
       "threads": threads, "reference_s_per_step": t_ref, "oracle_s_per_step": t_orc,
       "reference_pairs_per_s": B / t_ref, "oracle_pairs_per_s": B / t_orc,
       "oracle_over_reference": t_orc / t_ref, "within_20pct": abs(t_orc / t_ref - 1.0) <= 0.2,
       "reference_steps_s": ts_ref, "oracle_steps_s": ts_orc}
print(json.dumps(out), flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
