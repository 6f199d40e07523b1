"""Bitwise fingerprint of the benched step under the library in t5-resnet-vqa_amd/lib (an A/B of
two builds that must give the same bits: run once per build, compare the printed lines).
Builds the bench engine (B = 64, 224², pipelined, tuned, graphed, dropout 0.1), runs 3 steps and
prints the losses and a SHA-256 of the fp32 parameters, AdamW moments and bf16 shadow.
  python tools/lib_bitwise.py"""
import hashlib
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
args = types.SimpleNamespace(batch=64, seq_len=32, image_size=224, blocks=3, no_pipeline=False, dp_groups=False,
                             config5=False, tune_table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning",
                                                                    "gemm_gfx950.json"),
                             tune_save=None, no_graph=False, shard_optimizer=False, dp_res_split=None,
                             res_cumask=None)
pool = []
for i in range(4):
    nb = pkg.synthetic.make_batch(64, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng, _, step = bench.make_step(args, pkg, dev, pool, False, 0, "t5-base")
losses = []
for i in range(3):
    step(i)
    torch.cuda.synchronize()
    losses.append(float(eng.LOSS.item()))
eng.flush_optimizer()
torch.cuda.synchronize()
h = hashlib.sha256()
for t in (eng.P32, eng.M, eng.V, eng.VMAX, eng.P16, eng.LOGP):
    h.update(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())
print(json.dumps({"losses": losses, "sha256": h.hexdigest()}))
