"""Scratch: per-step loss / grad-norm trajectory of the engine vs the CPU oracle."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from __graft_entry__ import load_package
from oracle import vqa_oracle as orc
pkg = load_package()
B, L, H, steps = int(sys.argv[1]), 32, int(sys.argv[2]), int(sys.argv[3])
with_oracle = len(sys.argv) > 4
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=10, total=100000)
ot = orc.OracleTrainer(sd, "resnet50", warmup=10, total=100000) if with_oracle else None
batches = [pkg.synthetic.make_batch(B, L, H, seed=1 + i) for i in range(4)]
for s in range(steps):
    nb = batches[s % 4]
    lp, loss = eng.forward_backward(nb)
    gn_pre = eng.grad_norm()
    eng.optimizer_step(); torch.cuda.synchronize()
    line = f"step {s:3d} eng loss {loss:10.5f} gn {eng.last_grad_norm():12.5e} (host {gn_pre:12.5e})"
    if ot is not None:
        olp, oloss, ogn = ot.train_one_step(orc.to_torch_batch(nb))
        line += f" | oracle loss {float(oloss):10.5f} gn {float(ogn):12.5e}"
    print(line, flush=True)
