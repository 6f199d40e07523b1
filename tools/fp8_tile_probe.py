"""Every e4m3 tile config on config 5's largest forward GEMMs: median of
20 back-to-back launches per (shape, config), HIP events; prints TFLOP/s and the fraction of the
5,034 TFLOP/s dense fp8 peak.  Output bf16 + bias (+ ReLU on the FFN up-projection), as in the step.
  python tools/fp8_tile_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L = pkg.ops, pkg.lib
PEAK = 5034.0
SHAPES = [(2048, 18432, 1024, False), (2048, 4096, 1024, True), (2048, 1024, 4096, False), (2048, 3072, 1024, False),
          (2048, 1024, 1024, False)]
for M, N, K, relu in SHAPES:
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    x8, w8 = torch.empty(M, K, dtype=torch.uint8, device="cuda"), torch.empty(N, K, dtype=torch.uint8, device="cuda")
    sx, sw = torch.empty(M, device="cuda"), torch.empty(N, device="cuda")
    L.call("vqa_quant_rows_fp8", x.data_ptr(), 0, K, M, K, x8.data_ptr(), K, sx.data_ptr())
    L.call("vqa_quant_rows_fp8", w.data_ptr(), 0, K, N, K, w8.data_ptr(), K, sw.data_ptr())
    bias = torch.randn(N, device="cuda")
    out16 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ref = None
    res = []
    for cfg in L.GEMM_FP8:
        d = ops.gemm_desc(x8.view(torch.bfloat16), w8.view(torch.bfloat16), M, N, K, lda=K, ldb=K, c16=out16,
                          ldc16=N, bias=bias, relu=relu)
        d.fp8, d.scale_a, d.scale_b = 1, sx.data_ptr(), sw.data_ptr()
        d.config = cfg
        ops.run(d)
        torch.cuda.synchronize()
        if ref is None:
            ref = out16.clone()
        assert torch.equal(out16, ref), f"config {cfg} bits differ"
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record()
            ops.run(d)
            b.record()
        torch.cuda.synchronize()
        us = sorted(a.elapsed_time(b) for a, b in ev)[10] * 1e3
        tf = 2.0 * M * N * K / us / 1e6
        res.append((us, cfg, tf))
    res.sort()
    print(f"{M}x{N}x{K}: " + "  ".join(f"c{c} {us:.1f}us {tf:.0f}TF({tf / PEAK:.3f})" for us, c, tf in res), flush=True)
