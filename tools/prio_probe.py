"""Does stream priority help the pipelined step?  Two graphs (the step's chain; the next
batch's ResNet) replayed on two streams with different priorities, GPU time per step.

  python tools/prio_probe.py
"""
import os
import sys

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
eng.capture()                                    # single graph (reference)
single = eng.graph
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
MAIN, RES = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.graph(MAIN, stream=s):
    eng._run_step_streams()
with torch.cuda.graph(RES, stream=s):
    eng._run(eng.res_calls)
torch.cuda.synchronize()
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
print("priority range", lo, hi, flush=True)


def run(name, steps=20, mp=0, rp=0):
    ms = torch.cuda.Stream(priority=mp)
    rs = torch.cuda.Stream(priority=rp)
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(steps + 3):
        if i == 3:
            torch.cuda.synchronize()
            e0.record(cur)
        if name == "single":
            for g in single:
                g() if callable(g) else g.replay()
        else:
            eng.F4.copy_(eng.F4N)
            ev = torch.cuda.Event()
            ev.record(cur)
            ms.wait_event(ev)
            rs.wait_event(ev)
            with torch.cuda.stream(rs):
                RES.replay()
            with torch.cuda.stream(ms):
                MAIN.replay()
            for st in (ms, rs):
                j = torch.cuda.Event()
                j.record(st)
                cur.wait_event(j)
        eng.load_batch(pool[i % 2], next_images=pool[(i + 1) % 2]["image_tensors"])
    e1.record(cur)
    torch.cuda.synchronize()
    print(f"{name:10s} main_prio={mp} res_prio={rp}  {e0.elapsed_time(e1) / steps:7.3f} ms/step", flush=True)


run("single")
run("two", mp=0, rp=0)
run("two", mp=-1, rp=0)
run("two", mp=0, rp=1)
run("two", mp=-1, rp=1)
run("single")
run("two", mp=-1, rp=0)
