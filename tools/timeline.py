"""Per-queue timeline of one step from a rocprofv3 kernel trace: phases of
consecutive kernels on each queue (merged when the idle gap < 3 us), with
busy time, so cross-stream overlap and idle gaps are visible.

  python tools/timeline.py gpurun_out/profX/run_kernel_trace.csv [marker]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "rng_advance"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
starts = [i for i, k in enumerate(ks) if marker in k[2]]
a, b = starts[-3], starts[-2]
win = ks[a:b]
t0, t1 = win[0][0], ks[b][0]


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:40]


segs = []
for s, e, n, q in win:
    if segs and segs[-1]["q"] == q and s - segs[-1]["e"] < 3000:
        g = segs[-1]
        g["e"] = max(g["e"], e); g["busy"] += e - s; g["n"] += 1; g["last"] = short(n)
    else:
        # a segment may also continue after another queue's kernels
        prev = [g for g in segs if g["q"] == q]
        if prev and s - prev[-1]["e"] < 3000 and segs[-1]["q"] != q:
            g = prev[-1]
            g["e"] = max(g["e"], e); g["busy"] += e - s; g["n"] += 1; g["last"] = short(n)
            continue
        segs.append(dict(q=q, s=s, e=e, busy=e - s, n=1, first=short(n), last=short(n)))
for g in segs:
    print(f"q{g['q']:>3} {(g['s'] - t0) / 1e3:8.1f} -> {(g['e'] - t0) / 1e3:8.1f} us  busy {g['busy'] / 1e3:7.1f}  "
          f"n={g['n']:4d}  {g['first']} .. {g['last']}")
# union busy
iv = sorted((s, e) for s, e, _, _ in win)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs; cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"step {(t1 - t0) / 1e3:.1f} us, union busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
tot = sum(e - s for s, e, n, q in win)
print(f"sum of kernel durations {tot / 1e3:.1f} us (> union busy = overlap)")
