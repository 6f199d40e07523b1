"""Host-side view of the pipelined graph step: how long does each part of
train_step take on the host, and does the order of the two graph replays
(the next batch's ResNet on its own stream, the step's chain on the current
stream) change the GPU time per step?

  python tools/pipe_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
B = 64
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000, pipeline=True)
pool = [pkg.synthetic.make_batch(B, 32, 224, seed=s) for s in range(2)]
pool = [{k: (torch.as_tensor(v).cuda() if v is not None else None) for k, v in b.items()} for b in pool]
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
eng.prime(pool[0]["image_tensors"])
eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
eng.capture()
res_begin2, g2, _ = eng.graph
eng.capture()
res_begin, g, res_end = eng.graph


def run(order, steps=20):
    host = {"a": 0.0, "b": 0.0, "c": 0.0, "load": 0.0}
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(steps + 3):
        if i == 3:
            torch.cuda.synchronize()
            e0.record()
            t0 = time.perf_counter()
        ta = time.perf_counter()
        if order == "alt":
            rb, gg = (res_begin, g) if i % 2 == 0 else (res_begin2, g2)
            rb()
            tb = time.perf_counter()
            gg.replay()
        elif order == "res_first":
            res_begin()
            tb = time.perf_counter()
            g.replay()
        elif order == "main_first":
            eng.F4.copy_(eng.F4N)
            ev = torch.cuda.Event()
            ev.record()
            tb = time.perf_counter()
            g.replay()
            eng._rstream.wait_event(ev)
            with torch.cuda.stream(eng._rstream):
                RES.replay()
        elif order == "serial":
            eng.F4.copy_(eng.F4N)
            RES.replay()
            tb = time.perf_counter()
            g.replay()
        tc = time.perf_counter()
        res_end()
        td = time.perf_counter()
        eng.load_batch(pool[i % 2], next_images=pool[(i + 1) % 2]["image_tensors"])
        te = time.perf_counter()
        if i >= 3:
            host["a"] += tb - ta
            host["b"] += tc - tb
            host["c"] += td - tc
            host["load"] += te - td
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / steps
    print(f"{order:11s} gpu {gpu:7.3f} ms/step  host-issue {1e3 * (t1 - t0) / steps:7.3f} ms/step  "
          + "  ".join(f"{k} {1e3 * v / steps:7.3f}" for k, v in host.items()), flush=True)


# the res graph: capture it again standalone (same calls) for the variants
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
RES = torch.cuda.CUDAGraph()
with torch.cuda.graph(RES, stream=s):
    eng._run(eng.res_calls)
torch.cuda.synchronize()
for order in ("res_first", "alt", "main_first", "serial", "res_first", "alt"):
    run(order)
