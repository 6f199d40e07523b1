"""Scratch: B=64 trajectory, eager vs captured graph (+ device-resident batches like bench.py)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from __graft_entry__ import load_package
pkg = load_package()
B, L, H, steps, mode = int(sys.argv[1]), 32, 224, int(sys.argv[2]), sys.argv[3]
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=10, total=100000)
pool = [{k: torch.as_tensor(v).cuda() for k, v in pkg.synthetic.make_batch(B, L, H, seed=1 + i).items() if v is not None} for i in range(4)]
eng.load_batch(pool[0])
if mode == "graph":
    eng.capture()
for s in range(steps):
    eng.load_batch(pool[s % 4])
    eng.train_step()
    torch.cuda.synchronize()
    print(f"{mode} step {s:3d} loss {float(eng.LOSS):10.5f} gn {eng.last_grad_norm():12.5e} lr_scale {float(eng.opt_state[3]):.3f}", flush=True)
