"""Would two half-batch chains running concurrently beat one full-batch chain?

Times the forward + backward of the step (no ResNet: pipelined engines; no
optimizer) as one captured graph for
  * one engine at B = 64,
  * one engine at B = 32,
  * two B = 32 engines whose graphs are replayed on two streams at once.

  python tools/microbatch_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["VQA_DEFER_OPT"] = "0"                  # no AdamW ranges inside the forward
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
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
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        e.run_forward_streams()
        e.run_backward_streams()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with pkg.engine.no_gc_capture():
        with torch.cuda.graph(g, stream=s):
            e.run_forward_streams()
            e.run_backward_streams()
    torch.cuda.synchronize()
    return e, g


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


e64, g64 = make(64)
ea, ga = make(32)
eb, gb = make(32)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def two():
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    sa.wait_event(ev)
    sb.wait_event(ev)
    with torch.cuda.stream(sa):
        ga.replay()
    with torch.cuda.stream(sb):
        gb.replay()
    for s in (sa, sb):
        e = torch.cuda.Event()
        e.record(s)
        cur.wait_event(e)


def serial():
    ga.replay()
    gb.replay()


for rnd in range(2):
    t64 = timeit(g64.replay)
    t32 = timeit(ga.replay)
    t2s = timeit(serial)
    t2c = timeit(two)
    print(f"round {rnd}: fwd+bwd B=64 {t64:.3f} ms | B=32 {t32:.3f} ms | 2 x B=32 serial {t2s:.3f} ms | "
          f"2 x B=32 concurrent {t2c:.3f} ms", flush=True)
