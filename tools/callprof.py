"""Per-call timing of the real training step (eager, HIP events, N reps each).

  python tools/callprof.py [B] [--configs]

Prints one line per prepared call (phase, index, name, shape, us, TF/s for
GEMMs) and a summary grouped by kernel family, so each change can be judged
against where the step time actually goes.  --configs also times every GEMM
under each tile configuration.
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
L = pkg.lib
args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 64
CONFIGS = "--configs" in sys.argv
REPS = 10
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000)
eng.load_batch(pkg.synthetic.make_batch(B, 32, 224, seed=1))
eng.forward()
eng.backward()
torch.cuda.synchronize()
if "--autotune" in sys.argv:
    eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
s = L.stream_handle()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timeit(c):
    for _ in range(2):
        c(s)
    st.record()
    for _ in range(REPS):
        c(s)
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / REPS * 1e3


rows = []
fam = defaultdict(float)
for phase, calls in (("fwd", eng.fwd_calls), ("bwd", eng.bwd_calls), ("opt", eng.opt_calls)):
    for i, c in enumerate(calls):
        if c.name == "vqa_rng_advance":
            continue
        us = timeit(c)
        info, key = "", c.name
        if c.name == "vqa_gemm":
            d = c.desc
            fl = 2.0 * d.m * d.n * d.k * max(1, d.batch)
            kind = (f"{'At' if d.a_trans else 'A'}{'c' if d.a_conv else ''}"
                    f"{'Bt' if d.b_trans else 'B'}{'c' if d.b_conv else ''}")
            cfg = L.load().vqa_gemm_select(d)
            info = (f"{kind:6s} m={d.m:6d} n={d.n:6d} k={d.k:6d} b={max(1, d.batch)} cfg={cfg} sk={d.splitk} "
                    f"{fl / us / 1e6:6.1f}TF")
            key = f"gemm {phase} {'conv' if d.a_conv or d.b_conv else 'lin'} {kind}"
            if CONFIGS:
                alt = []
                for cf in (1, 2, 3, 4):
                    d.config = cf
                    alt.append(f"c{cf} {timeit(c):7.1f}")
                d.config = 0
                info += "  " + " ".join(alt)
        elif c.desc is not None and hasattr(c.desc, "heads"):
            d = c.desc
            info = f"B={d.batch} H={d.heads} lq={d.lq} lk={d.lk} dh={d.dh}"
        fam[key] += us
        rows.append((phase, i, c.name, info, us))
        print(f"{phase} {i:4d} {c.name:24s} {us:8.1f}us  {info}", flush=True)

tot = sum(r[-1] for r in rows)
print(f"\nTOTAL eager sum {tot:.1f} us")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"  {v:9.1f} us  {100 * v / tot:5.1f}%  {k}")
