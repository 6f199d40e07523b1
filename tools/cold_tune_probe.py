"""Warm vs cold GEMM tuning, judged by the step.

The autotuner times each candidate replayed back to back (operands hot in L2); inside the
step every GEMM reads an operand another kernel just wrote (another XCD's L2, the Infinity
Cache) and weights last read a step ago.  This captures the benched step with the
committed (warm-tuned) table, then re-tunes every GEMM from cold caches
(VQAEngine.autotune(cold=True)), re-captures, and times both.

  python tools/cold_tune_probe.py [OUT_TABLE.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
B = 64
TABLE = os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json")
out = sys.argv[1] if len(sys.argv) > 1 else None
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000, pipeline=True)
pool = [pkg.synthetic.make_batch(B, 32, 224, seed=s) for s in range(2)]
pool = [{k: (torch.as_tensor(v).cuda() if v is not None else None) for k, v in b.items()} for b in pool]
eng.prime(pool[0]["image_tensors"])
eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
eng.forward()
eng.backward()


def step_ms(steps=30, warm=5):
    eng.capture()
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(steps + warm):
        if i == warm:
            torch.cuda.synchronize()
            e0.record(cur)
        eng.train_step()
        eng.load_batch(pool[i % 2], next_images=pool[(i + 1) % 2]["image_tensors"])
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


warm_choice = eng.autotune(table=TABLE)
t_warm = step_ms()
print(f"warm-tuned table: {t_warm:.3f} ms/step", flush=True)
cold_choice = eng.autotune(cold=True)
t_cold = step_ms()
print(f"cold-tuned:       {t_cold:.3f} ms/step  ({sum(warm_choice[k] != cold_choice.get(k) for k in warm_choice)} "
      f"of {len(warm_choice)} choices differ)", flush=True)
for k in warm_choice:
    if warm_choice[k] != cold_choice.get(k):
        print(f"  {warm_choice[k]:4d} -> {cold_choice.get(k)!s:5s} {k[:110]}")
eng.autotune(table=TABLE)
print(f"warm-tuned again: {step_ms():.3f} ms/step", flush=True)
eng.autotune(cold=True)
print(f"cold-tuned again: {step_ms():.3f} ms/step", flush=True)
if out:
    json.dump(dict(sorted(cold_choice.items())), open(out, "w"), indent=0)
