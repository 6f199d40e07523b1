"""Where does a T5 projection GEMM's in-graph time go?  In the step's trace the 2048-row
projections fit t = 13 us + 0.9 us/GFLOP; replayed back to back they cost ~4 us + the
same slope.  Times the T5 forward shapes (tuned tile choice) four ways:

  warm     replayed back to back (the autotuner's view)
  cold     a 512 MiB write before each launch (L2 + Infinity Cache evicted)
  chain    the producer of A (a copy that rewrites A) right before each launch
  graph12  12 launches of the shape, each after its A-producer, captured in one graph
           (event time / 12, producers included; producer alone subtracted)

  python tools/gemm_cold_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L, E = pkg.ops, pkg.lib, pkg.engine
s = L.stream_handle()
table = json.load(open(os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json")))
flush = torch.empty(128 << 20, dtype=torch.float32, device="cuda")
REPS = 20


def ev_time(fn, reps=REPS, pre=None):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        if pre:
            pre()
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return ts[reps // 2]


def graph_time(fn, n=12, reps=10):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(n):
            fn()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / n


M = 2048
shapes = [("o   ", 768, 768, "res"), ("qkv ", 2304, 768, "c16"), ("wi  ", 3072, 768, "relu"), ("wo  ", 768, 3072, "res")]
for tag, N, K, kind in shapes:
    a = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
    asrc = a.clone()
    w = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
    c16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c32 = torch.empty(M, N, device="cuda", dtype=torch.float32)
    res = torch.randn(M, N, device="cuda")
    kw = dict(lda=K, ldb=K)
    if kind == "res":
        kw.update(c32=c32, ldc32=N, res32=res, ldres=N)
    else:
        kw.update(c16=c16, ldc16=N, relu=kind == "relu")
    d = ops.gemm_desc(a, w, M, N, K, **kw)
    key = repr(E._gemm_key(d))
    choice = table.get(key)
    for cfg in sorted({choice % 100 if choice else 4, 3, 4, 5}):
        d.config = cfg
        call = ops.gemm_call(d, (a, w, c16, c32, res))
        flop = 2.0 * M * N * K
        gemm = lambda: call(s)                                   # noqa: E731
        prod = lambda: a.copy_(asrc)                              # noqa: E731
        warm = ev_time(gemm)
        cold = ev_time(gemm, pre=lambda: flush.fill_(1.0))
        chain = ev_time(gemm, pre=prod)
        p_only = graph_time(prod)
        g12 = graph_time(lambda: (prod(), gemm())) - p_only
        mark = "*" if choice and cfg == choice % 100 else " "
        print(f"{tag} N={N:4d} K={K:4d} cfg{cfg:2d}{mark} {flop / 1e9:5.2f} GF | warm {warm:6.2f} cold {cold:6.2f} "
              f"chain {chain:6.2f} graph12 {g12:6.2f} us (producer {p_only:5.2f})", flush=True)
