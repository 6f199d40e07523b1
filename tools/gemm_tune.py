"""Time every GEMM launch of the real B=64 step under each tile config (1,2,3) and auto (0)."""
import sys, os, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from __graft_entry__ import load_package
pkg = load_package()
L = pkg.lib
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000)
eng.load_batch(pkg.synthetic.make_batch(B, 32, 224, seed=1))
eng.forward(); eng.backward(); torch.cuda.synchronize()
lib = L.load()
s = L.stream_handle()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
rows = []
for phase, calls in (("fwd", eng.fwd_calls), ("bwd", eng.bwd_calls)):
    for c in calls:
        if c.name != "vqa_gemm":
            continue
        d = c.desc
        res = {}
        for cfg in (0, 1, 2, 3):
            d.config = cfg
            for _ in range(2): c(s)
            st.record(); 
            for _ in range(10): c(s)
            en.record(); en.synchronize()
            res[cfg] = st.elapsed_time(en) / 10 * 1e3
        d.config = 0
        fl = 2.0 * d.m * d.n * d.k
        kind = f"{'A^T' if d.a_trans else 'A'}{'c' if d.a_conv else ''} {'B^T' if d.b_trans else 'B'}{'c' if d.b_conv else ''}"
        rows.append((phase, kind, d.m, d.n, d.k, fl, res))
tot = {c: 0.0 for c in range(4)}
best = 0.0
for ph, kind, m, n, k, fl, r in rows:
    b = min(r[1], r[2], r[3])
    best += b
    for c in range(4): tot[c] += r[c]
    print(f"{ph} {kind:10s} {m:6d} {n:6d} {k:6d} {fl/1e9:7.2f}GF auto {r[0]:8.1f}us ({fl/r[0]/1e6:6.1f}TF) c1 {r[1]:8.1f} c2 {r[2]:8.1f} c3 {r[3]:8.1f}  best {fl/b/1e6:6.1f}TF")
print("total us per step: auto %.1f c1 %.1f c2 %.1f c3 %.1f best %.1f" % (tot[0], tot[1], tot[2], tot[3], best))
