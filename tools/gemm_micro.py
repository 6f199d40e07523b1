"""Micro-benchmark: our GEMM (configs) vs torch.matmul (hipBLASLt, reference point only)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from __graft_entry__ import load_package
pkg = load_package(); ops = pkg.ops; L = pkg.lib
shapes = [(2048, 768, 768), (2048, 3072, 768), (2048, 768, 3072), (2048, 2304, 768), (2048, 1536, 768), (3136, 1536, 768)]
if len(sys.argv) > 3:                                                        # "MxNxK,MxNxK"
    shapes = [tuple(int(v) for v in t.split("x")) for t in sys.argv[3].split(",")]
cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "3"]          # "<config>[s<splitk>]"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
s = L.stream_handle()
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    line = f"{M:5d}x{N:5d}x{K:5d}"
    fl = 2.0 * M * N * K
    for cfg in cfgs:
        d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c16=c, ldc16=N)
        cf, _, sk = cfg.partition("s")
        d.config = int(cf)
        ws = None
        if sk:
            ops.set_splitk(d, int(sk))
            ws = ops.splitk_workspace(d)
            ops.set_splitk(d, int(sk), ws)
        call = ops.gemm_call(d, (a, b, c, ws))
        for _ in range(3): call(s)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(reps): call(s)
        en.record(); en.synchronize()
        t = st.elapsed_time(en) / reps * 1e-3
        line += f" | c{cfg} {t*1e6:7.1f}us {fl/t/1e12:5.0f}"
    for _ in range(3): torch.matmul(a, b.T, out=c)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps): torch.matmul(a, b.T, out=c)
    en.record(); en.synchronize()
    t = st.elapsed_time(en) / reps * 1e-3
    line += f" | hipBLASLt {t*1e6:8.1f}us {fl/t/1e12:6.0f}TF"
    print(line, flush=True)
