"""Host-side cost of launching the captured step graph: time of g.replay() itself
(submission) vs the GPU time of the step, and the number of graph nodes."""
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
g = eng.graph[0]
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
host = []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
gpu0 = time.perf_counter()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
gpu = (time.perf_counter() - gpu0) / 10
n_calls = len(eng.res_calls) + len(eng.fwd_calls) + len(eng.bwd_calls) + len(eng.opt_calls) + len(eng.adam_segs)
print(f"graph replay host time: median {sorted(host)[5] * 1e3:.3f} ms, step {gpu * 1e3:.3f} ms, ~{n_calls} kernel calls")
# submission of a long chain of tiny kernels: host cost per node
small = torch.zeros(1, device=dev)
g2 = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    small.add_(1)
torch.cuda.synchronize()
with torch.cuda.graph(g2, stream=s):
    for _ in range(300):
        small.add_(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
g2.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"300-node tiny chain: replay() host {1e3 * (t1 - t0):.3f} ms, done after {1e3 * (t2 - t0):.3f} ms")
