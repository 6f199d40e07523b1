"""Scratch: which gradient segment differs between graph replay and eager at B=64."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from __graft_entry__ import load_package
pkg = load_package()
B = int(sys.argv[1]); L, H = 32, 224
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
e1 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=10, total=100000)
e2 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=10, total=100000)
nb = pkg.synthetic.make_batch(B, L, H, seed=1)
e1.load_batch(nb); e2.load_batch(nb)
e2.capture()
for s in range(2):
    e1.train_step(); e2.train_step(); torch.cuda.synchronize()
    print("step", s, float(e1.LOSS), float(e2.LOSS), e1.last_grad_norm(), e2.last_grad_norm())
    bad = []
    for name, seg in e1.lay.segments.items():
        a, b = e1.g32[name], e2.g32[name]
        d = (a - b).abs().max().item()
        bad.append((d, name, a.abs().max().item(), b.abs().max().item(), torch.isfinite(b).all().item()))
    bad.sort(reverse=True)
    for x in bad[:8]: print("   ", x)
    for nm in ("HS", "QKV", "FF", "PT"):
        arrs = getattr(e1, nm)
        for i in range(len(arrs)):
            d = (getattr(e1, nm)[i].float() - getattr(e2, nm)[i].float()).abs().max().item()
            if d > 1e-3: print("   act", nm, i, d)
    for k in ("VIS32", "TXT32", "dTXT", "dVIS32", "dH32", "F4", "dPB", "LOGP"):
        d = (getattr(e1, k).float() - getattr(e2, k).float()).abs().max().item()
        print("   buf", k, d)
