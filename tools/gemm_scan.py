"""Fixed-cost vs per-K-tile cost of the GEMM kernel: time C[M,N] = A[M,K] B[N,K]^T
for a K sweep at a few (M, N) and tile configs (intercept = launch + prologue +
epilogue, slope = steady-state cost of one 64-deep K-tile)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L = pkg.ops, pkg.lib
s = L.stream_handle()
reps = 20
for M, N in ((2048, 768), (2048, 3072), (8192, 8192)):
    for cfg in (4, 6, 8, 11):
        line = f"{M:5d}x{N:5d} c{cfg:<2d}"
        for K in (64, 128, 256, 512, 1024, 2048, 4096):
            a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c16=c, ldc16=N)
            d.config = cfg
            call = ops.gemm_call(d, (a, b, c))
            for _ in range(3):
                call(s)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(reps):
                call(s)
            en.record()
            en.synchronize()
            t = st.elapsed_time(en) / reps * 1e3
            line += f" K{K}:{t:7.1f}"
        print(line, flush=True)
# empty-kernel floor: back-to-back launches of a 1-tile GEMM
a = torch.randn(64, 64, device="cuda").to(torch.bfloat16)
c = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
d = ops.gemm_desc(a, a, 64, 64, 64, lda=64, ldb=64, c16=c, ldc16=64)
d.config = 4
call = ops.gemm_call(d, (a, c))
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(200):
    call(s)
en.record()
en.synchronize()
print(f"1-tile GEMM back to back: {st.elapsed_time(en) / 200 * 1e3:.2f} us per launch")
