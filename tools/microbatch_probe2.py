"""Two half-batch chains as two branches of ONE graph (graph branches are known to run
concurrently; two separately launched graphs may not -- tools/microbatch_probe.py).

Every engine runs its forward + backward call lists on a single stream (pipelined
engines: no ResNet; no optimizer).  Captured:
  one64      one B = 64 engine, one stream
  one32      one B = 32 engine, one stream
  two32      two B = 32 engines on two forked streams, calls issued alternately
  two32ser   the same two engines one after the other on one stream

  python tools/microbatch_probe2.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["VQA_DEFER_OPT"] = "0"
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
L = pkg.lib
TABLE = os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json")
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)


def make(B):
    e = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000, pipeline=True)
    b = pkg.synthetic.make_batch(B, 32, 224, seed=1)
    b = {k: (torch.as_tensor(v).cuda() if v is not None else None) for k, v in b.items()}
    e.autotune(table=TABLE)
    e.prime(b["image_tensors"])
    e.load_batch(b, next_images=b["image_tensors"])
    e.F4.copy_(e.F4N)
    e._run(e.fwd_calls + e.bwd_calls)
    torch.cuda.synchronize()
    return e


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with pkg.engine.no_gc_capture():
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.synchronize()
    return g


def timeit(g, reps=30):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


e64, ea, eb = make(64), make(32), make(32)


def one(e):
    def f():
        h = L.stream_handle()
        for c in e.fwd_calls + e.bwd_calls:
            c(h)
    return f


def two_branches():
    cur = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    fork = torch.cuda.Event()
    fork.record(cur)
    s2.wait_event(fork)
    h1, h2 = L.stream_handle(cur), L.stream_handle(s2)
    la, lb = ea.fwd_calls + ea.bwd_calls, eb.fwd_calls + eb.bwd_calls
    for i in range(max(len(la), len(lb))):
        if i < len(la):
            la[i](h1)
        if i < len(lb):
            lb[i](h2)
    join = torch.cuda.Event()
    join.record(s2)
    cur.wait_event(join)


def two_serial():
    one(ea)()
    one(eb)()


g64, g32, g2, g2s = capture(one(e64)), capture(one(ea)), capture(two_branches), capture(two_serial)
for rnd in range(3):
    print(f"round {rnd}: one64 {timeit(g64):.3f} | one32 {timeit(g32):.3f} | two32 branches {timeit(g2):.3f} | "
          f"two32 serial {timeit(g2s):.3f} ms", flush=True)
