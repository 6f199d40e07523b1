"""Stand-alone time of every call of the frozen ResNet chain (engine.res_calls),
each replayed `reps` times between HIP events on one stream, with its GEMM shape,
FLOP rate and output-byte rate: where the feature extractor's time goes.

  python tools/res_micro.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
L = pkg.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = 64
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000, pipeline=True)
eng.load_batch(pkg.synthetic.make_batch(B, 32, 224, seed=1), next_images=pkg.synthetic.make_batch(B, 32, 224, seed=2)["image_tensors"])
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
s = L.stream_handle()
eng._run(eng.res_calls)
torch.cuda.synchronize()
tot = 0.0
for i, c in enumerate(eng.res_calls):
    for _ in range(2):
        c(s)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        c(s)
    en.record()
    en.synchronize()
    t = st.elapsed_time(en) / reps * 1e3
    tot += t
    d = c.desc
    if isinstance(d, L.GemmDesc):
        fl = 2.0 * d.m * d.n * d.k
        print(f"{i:3d} gemm M={d.m:7d} N={d.n:5d} K={d.k:5d} cfg={d.config:3d} sk={d.splitk} {t:8.1f} us "
              f"{fl / t / 1e6:6.0f} TF/s  out {d.m * d.n * 2 / t / 1e3:6.0f} GB/s", flush=True)
    else:
        print(f"{i:3d} {c.name:28s} {t:8.1f} us", flush=True)
print(f"total {tot:.1f} us")
