"""Tile-config x split-K sweep of the step's recurring GEMM shapes (forward Linear
layout C = A B^T), plus a K sweep at M=2048, N=768 for the fixed vs per-K-tile cost.

  python tools/gemm_lab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L = pkg.ops, pkg.lib
s = L.stream_handle()
REPS = 20
NCFG = pkg.engine.lib_gemm_configs()


def timeit(call):
    for _ in range(3):
        call(s)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(REPS):
        call(s)
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / REPS * 1e3


def sweep(M, N, K, splits=(1, 2, 3, 4)):
    a = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = []
    for cfg in range(1, NCFG + 1):
        for sk in splits:
            d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c16=c, ldc16=N)
            d.config = cfg
            ws = None
            if sk > 1:
                ops.set_splitk(d, sk)
                ws = ops.splitk_workspace(d)
                ops.set_splitk(d, sk, ws)
            t = timeit(ops.gemm_call(d, (a, b, c, ws)))
            res.append((t, cfg, sk))
    res.sort()
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K}: " + "  ".join(f"c{c}s{k} {t:.1f}us({fl / t / 1e6:.0f}TF)" for t, c, k in res[:6]), flush=True)


for M, N, K in ((2048, 768, 768), (2048, 2304, 768), (2048, 3072, 768), (2048, 768, 3072), (2048, 6912, 768),
                (200704, 256, 64), (12544, 1024, 256), (50176, 512, 128)):
    sweep(M, N, K)
for cfg in (4, 8, 11):
    line = f"K sweep 2048x768 c{cfg}:"
    for K in (64, 128, 256, 512, 768, 1536, 3072):
        a = torch.randn(2048, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(768, K, device="cuda").to(torch.bfloat16)
        c = torch.empty(2048, 768, device="cuda", dtype=torch.bfloat16)
        d = ops.gemm_desc(a, b, 2048, 768, K, lda=K, ldb=K, c16=c, ldc16=768)
        d.config = cfg
        line += f" {K}:{timeit(ops.gemm_call(d, (a, b, c))):.1f}"
    print(line, flush=True)
