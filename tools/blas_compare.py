"""Compare our GEMM (best tile config) with torch.matmul (hipBLASLt) on the step's linear shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L = pkg.ops, pkg.lib
torch.backends.cuda.matmul.allow_tf32 = False
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps * 1e3


shapes = [  # (name, M, N, K, layout)  layout: fwd = A[M,K] W[N,K]^T ; dx = dY[M,N'] W[N',K] ; dw = dY^T X
    ("qkv fwd", 2048, 2304, 768, "fwd"), ("o fwd", 2048, 768, 768, "fwd"), ("wi fwd", 2048, 3072, 768, "fwd"),
    ("wo fwd", 2048, 768, 3072, "fwd"),
    ("qkv dx", 2048, 768, 2304, "dx"), ("wi dx", 2048, 768, 3072, "dx"), ("wo dx", 2048, 3072, 768, "dx"),
    ("qkv dw", 2304, 768, 2048, "dw"), ("wi dw", 3072, 768, 2048, "dw"), ("wo dw", 768, 3072, 2048, "dw"),
    ("convT fwd-like", 3136, 768, 18432, "fwd"), ("big", 8192, 8192, 8192, "fwd"),
]
for name, M, N, K, lay in shapes:
    if lay == "fwd":
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        ref = lambda: torch.matmul(a, b.T)
        kw = dict(lda=K, ldb=K)
    elif lay == "dx":     # out[M,N] = dY[M,K] W[K,N]  (W stored [K][N])
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(K, N, device="cuda").bfloat16()
        ref = lambda: torch.matmul(a, b)
        kw = dict(lda=K, ldb=N, b_trans=True)
    else:                 # out[M,N] = dY[K,M]^T X[K,N]
        a = torch.randn(K, M, device="cuda").bfloat16()
        b = torch.randn(K, N, device="cuda").bfloat16()
        ref = lambda: torch.matmul(a.T, b)
        kw = dict(lda=M, ldb=N, a_trans=True, b_trans=True)
    c = torch.empty(M, N, device="cuda")
    d = ops.gemm_desc(a, b, M, N, K, c32=c, ldc32=N, **kw)
    call = ops.gemm_call(d)
    s = L.stream_handle()
    best = None
    for cfg in range(1, 9):
        d.config = cfg
        us = t(lambda: call(s))
        if best is None or us < best[0]:
            best = (us, cfg)
    tb = t(ref)
    fl = 2.0 * M * N * K
    print(f"{name:14s} {M:5d}x{N:5d}x{K:5d}  ours {best[0]:8.1f}us ({fl / best[0] / 1e6:6.1f} TF, cfg {best[1]})  "
          f"hipBLASLt {tb:8.1f}us ({fl / tb / 1e6:6.1f} TF)", flush=True)
