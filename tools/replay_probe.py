"""Back-to-back graph replays of the benched step: host time of each replay() call (does a
launch wait for the previous launch of the same graph?) and the step time when two
separately captured, identical graphs alternate."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
dev = torch.device("cuda", 0)
B, L, H = 64, 32, 224
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, device=dev, warmup=10, total=100000, dropout=0.1,
                           pipeline=True)
nb = {k: torch.as_tensor(v).to(dev) for k, v in pkg.synthetic.make_batch(B, L, H, seed=1).items() if v is not None}
eng.prime(nb["image_tensors"])
eng.F4.copy_(eng.F4N)
eng.load_batch(nb, next_images=nb["image_tensors"])
eng.forward()
eng.backward()
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
eng.capture()
ga = eng.graph[0]
eng.capture()
gb = eng.graph[0]
for _ in range(5):
    ga.replay()
torch.cuda.synchronize()


def run(seq, n=30):
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for i in range(n):
        a = time.perf_counter()
        seq[i % len(seq)].replay()
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    h = sorted(host)
    return wall * 1e3, h[len(h) // 2] * 1e3, h[-1] * 1e3


for name, seq in (("same", [ga]), ("alternate", [ga, gb]), ("same", [ga]), ("alternate", [ga, gb])):
    w, hm, hx = run(seq)
    print(f"{name:9s}: step {w:.3f} ms, replay() host median {hm:.3f} ms max {hx:.3f} ms", flush=True)
