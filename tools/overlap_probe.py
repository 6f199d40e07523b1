"""Does the next batch's frozen ResNet overlap the step's chain, by how it is launched?

  python tools/overlap_probe.py [--steps 20]

Builds the bench engine (B = 64, 224^2, L = 32, tuned table, pipelined) and times, per step:
  A  the bench graph (ResNet branch captured first inside the one step graph)
  B  the step graph WITHOUT the ResNet + the ResNet launched eagerly on its own stream
  C  the step graph WITHOUT the ResNet + the ResNet as a graph of its own on its own stream
  D  the step graph without the ResNet alone (lower bound)
  E  the ResNet alone, eager
Variants B / C join the ResNet stream into the main stream after the step graph, so every
step sees the same dependencies as A (F4 <- F4N before the ResNet of the next batch)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--variants", default="ABCDEA")
args = ap.parse_args()
pkg = load_package()
L = pkg.lib
B = 64
dev = torch.device("cuda", 0)
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=100000, dropout=0.1,
                           pipeline=True)
pool = []
for i in range(4):
    nb = pkg.synthetic.make_batch(B, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng.prime(pool[0]["image_tensors"])
eng.F4.copy_(eng.F4N)
eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
eng.forward()
eng.backward()
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))

eng.capture()
g_full = eng.graph
res_calls, copy_f4 = eng.res_calls, eng.copy_f4
eng.res_calls, eng.copy_f4 = [], (lambda h: None)
eng.capture()
g_chain = eng.graph[0]
eng.res_calls, eng.copy_f4 = res_calls, copy_f4
eng.graph = g_full
g_res = torch.cuda.CUDAGraph()
s = torch.cuda.Stream(dev)
with pkg.engine.no_gc_capture(), torch.cuda.graph(g_res, stream=s):
    hs = L.stream_handle(s)
    for c in res_calls:
        c(hs)
main = torch.cuda.current_stream(dev)
rs = eng._rstream


def res_branch(mode):
    copy_f4(L.stream_handle(main))
    ev = torch.cuda.Event()
    ev.record(main)
    rs.wait_event(ev)
    if mode == "eager":
        h = L.stream_handle(rs)
        for c in res_calls:
            c(h)
    else:
        with torch.cuda.stream(rs):
            g_res.replay()


def join():
    ev = torch.cuda.Event()
    ev.record(rs)
    main.wait_event(ev)


def run(v, i):
    eng.load_batch(pool[i % 4], next_images=pool[(i + 1) % 4]["image_tensors"])
    if v == "A":
        g_full[0].replay()
    elif v in "BC":
        res_branch("eager" if v == "B" else "graph")
        g_chain.replay()
        join()
    elif v == "D":
        g_chain.replay()
    elif v == "E":
        res_branch("eager")
        join()


out = {}
for v in args.variants:
    for i in range(5):
        run(v, i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = 0.0
    t0 = time.perf_counter()
    e0.record(main)
    for i in range(args.steps):
        h0 = time.perf_counter()
        run(v, i)
        host += time.perf_counter() - h0
    e1.record(main)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps * 1e3
    gpu = e0.elapsed_time(e1) / args.steps
    key = v if v not in out else v + "2"
    out[key] = {"gpu_ms": round(gpu, 3), "wall_ms": round(wall, 3), "host_ms": round(host / args.steps * 1e3, 3)}
    print(key, out[key], flush=True)
print(json.dumps(out))
