"""Where a 2048-row GEMM's time goes: K sweep x tile config at M=2048, N=768 (the SGA /
T5 projection shape family), each case replayed REPS times back to back, plus the
1-tile launch floor.  Prints event-timed us per launch and writes a manifest of the
dispatch order so that a rocprofv3 --kernel-trace of the same run gives in-kernel
durations per case (tools/gemm_probe.py --trace DIR MANIFEST).

  python tools/gemm_probe.py MANIFEST.json
  python tools/gemm_probe.py --trace gpurun_out/probe_kt MANIFEST.json"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] == "--trace":
    rows = []
    for f in glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows = [r for r in rows if "gemm" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    man = json.load(open(sys.argv[3]))
    i = 0
    for case in man["cases"]:
        n = case["reps"]
        ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[i:i + n])
        gaps = [int(rows[j + 1]["Start_Timestamp"]) - int(rows[j]["End_Timestamp"]) for j in range(i, i + n - 1)]
        i += n
        med = ds[len(ds) // 2] / 1e3
        fl = case["flop"]
        print(f"{case['tag']:40s} kernel {med:7.2f} us  {fl / med / 1e6:6.1f} TF   gap {sorted(gaps)[len(gaps) // 2] / 1e3:5.2f} us"
              f"   event {case['event_us']:7.2f} us")
    sys.exit(0)

import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ops, L = pkg.ops, pkg.lib
s = L.stream_handle()
REPS = 20
cases = []


def run(tag, call, flop):
    for _ in range(3):
        call(s)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(REPS):
        call(s)
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) / REPS * 1e3
    cases.append({"tag": tag, "reps": REPS + 3, "flop": flop, "event_us": us})
    print(f"{tag:40s} {us:7.2f} us  {flop / us / 1e6:6.1f} TF", flush=True)


M, N = 2048, 768
for K in (64, 256, 768, 1536, 3072):
    a = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
    c16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c32 = torch.empty(M, N, device="cuda", dtype=torch.float32)
    for cfg in (3, 4, 5, 7, 8, 13):
        for out in ("c16", "c32+c16"):
            d = ops.gemm_desc(a, b, M, N, K, lda=K, ldb=K, c16=c16, ldc16=N,
                              c32=c32 if out != "c16" else None, ldc32=N)
            d.config = cfg
            run(f"{M}x{N}x{K} cfg{cfg} {out}", ops.gemm_call(d, (a, b, c16, c32)), 2.0 * M * N * K)
a = torch.randn(64, 64, device="cuda").to(torch.bfloat16)
c = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
d = ops.gemm_desc(a, a, 64, 64, 64, lda=64, ldb=64, c16=c, ldc16=64)
d.config = 4
run("1-tile 64x64x64", ops.gemm_call(d, (a, c)), 2.0 * 64 ** 3)
torch.cuda.synchronize()
json.dump({"cases": cases}, open(sys.argv[1], "w"))
