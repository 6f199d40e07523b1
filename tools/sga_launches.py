"""Per-launch table of the SGA GEMMs bench.py's sga_mfma counts (and, with `all`, every GEMM
of the step): shape, operand layout, tile config, split-K, stand-alone event time and
TFLOP/s, each launch replayed REPS times back to back on its stream (host launches), and the
same REPS launches captured as one graph and replayed (g_us: as inside the step graph).

  python tools/sga_launches.py [REPS] [all] [--config5] > out.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
ALL = "all" in sys.argv
C5 = "--config5" in sys.argv
pkg = load_package()
L = pkg.lib
dev = torch.device("cuda", 0)
B, Lq, H = 64, 32, (384 if C5 else 224)
lm = "t5-large" if C5 else "t5-base"
NB = 6 if C5 else 3
sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=NB, language_model=lm)
eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=Lq, image_size=H, device=dev, warmup=10,
                           total=100000, dropout=0.1, seed=0, num_blocks=NB, language_model=lm, fp8=C5)
del sd
eng.load_batch(pkg.synthetic.make_batch(B, Lq, H, seed=1))
eng.forward()
eng.backward()
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
eng.forward()
eng.backward()
torch.cuda.synchronize()
stream = torch.cuda.current_stream(dev)
h = L.stream_handle(stream)


def time_call(c):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        c(h)
    a.record(stream)
    for _ in range(REPS):
        c(h)
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / REPS * 1e-3


def time_graph(c):
    """the same REPS launches captured as one graph (as they run inside the step graph)"""
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream(dev)
    st.wait_stream(stream)
    with torch.cuda.stream(st):
        c(L.stream_handle(st))
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=st):
        hs = L.stream_handle(st)
        for _ in range(REPS):
            c(hs)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    g.replay()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / REPS * 1e-3


if ALL:
    calls = [c for c in (list(eng.res_calls) if eng.pipeline else []) + eng.fwd_calls + eng.bwd_calls
             if c.name in ("vqa_gemm", "vqa_gemm_pair")]
else:
    calls = [c for c in eng.sga_vision_calls + eng.fwd_calls[eng._fsplit[2]:] + eng.bwd_calls[:eng._bsplit[0]]
             if c.name in ("vqa_gemm", "vqa_gemm_pair")]
tot_f = tot_t = 0.0
print(f"{'m':>6} {'n':>6} {'k':>6} {'bat':>3} {'tr':>3} {'cfg':>4} {'sk':>2} {'us':>8} {'TF/s':>7} {'frac':>6} {'g_us':>7}")
tot_g = 0.0
for c in calls:
    ds = c.desc if c.name == "vqa_gemm_pair" else (c.desc,)
    fl = sum(2.0 * d.m * d.n * d.k * max(1, d.batch) for d in ds)
    t = time_call(c)
    tg = time_graph(c)
    tot_f += fl
    tot_t += t
    tot_g += tg
    for d in ds:
        cfg = L.load().vqa_gemm_select(d)
        tr = f"{'T' if d.a_trans else 'N'}{'T' if d.b_trans else 'N'}" + ("8" if getattr(d, "fp8", 0) else "")
        print(f"{d.m:6d} {d.n:6d} {d.k:6d} {max(1, d.batch):3d} {tr:>3} {cfg:4d} {max(1, d.splitk):2d} "
              f"{t * 1e6:8.1f} {fl / t / 1e12:7.1f} {fl / t / 1e12 / 2517:6.3f} {tg * 1e6:7.1f}" + ("  (pair)" if len(ds) > 1 else ""))
print(f"total {len(calls)} launches {tot_f / 1e9:.1f} GFLOP {tot_t * 1e6:.1f} us {tot_f / tot_t / 1e12:.1f} TFLOP/s "
      f"= {tot_f / tot_t / 1e12 / 2517:.4f} of bf16 peak; graph-replayed {tot_g * 1e6:.1f} us = "
      f"{tot_f / tot_g / 1e12 / 2517:.4f}", flush=True)
