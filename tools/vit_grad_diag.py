"""Per-segment gradient error of the config-4 engine against the CPU oracle fed the engine's
own ViT pooled output (eval mode, B=4, L=16): which parameters deviate."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from oracle import vit_oracle as orc  # noqa: E402

pkg = load_package()
vm = pkg.vit_model
B, L = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 16
nb = vm.make_batch(B, L, seed=1)
sd = vm.make_state_dict(seed=0)
eng = pkg.vit_engine.VitVQAEngine(sd, batch=B, seq_len=L, dropout=0.0)
lp, loss = eng.forward_backward(nb)
ot = orc.VitOracleTrainer(sd)
tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
olp, oloss = ot.forward_backward(tb, pooled=eng.vit_pooled().cpu())
grads = {k: (ot.sd[k].grad.numpy() if ot.sd[k].grad is not None else np.zeros(ot.sd[k].shape, np.float32))
         for k in ot.sd if not k.startswith("vision_model.")}
lay = eng.lay
go = lay.pack(grads)
ge = eng.G32.cpu().numpy()
rows = []
for s in lay.segments.values():
    a, b = ge[s.offset:s.offset + s.numel], go[s.offset:s.offset + s.numel]
    nb_ = np.linalg.norm(b)
    rows.append((np.linalg.norm(a - b) / max(nb_, 1e-30), s.name, nb_, np.linalg.norm(a)))
rows.sort(reverse=True)
print(f"loss engine {loss:.6f} oracle {float(oloss):.6f}  lp max-abs {np.abs(lp - olp.numpy()).max():.3e}")
og, eg = ot.group_grad_norms(), eng.group_grad_norms()
print("group grad-norm rel:", {k: abs(eg[k] - og[k]) / og[k] for k in og})
tot = np.sqrt(sum(np.linalg.norm(ge[s.offset:s.offset + s.numel] - go[s.offset:s.offset + s.numel]) ** 2
                  for s in lay.segments.values())) / np.linalg.norm(go)
print(f"whole-gradient relative L2 error {tot:.3e}")
for r in rows[:12]:
    print(f"{r[0]:.3e}  {r[1]:16s} |g_oracle| {r[2]:.4e} |g_engine| {r[3]:.4e}")
