"""Gap analysis of a rocprofv3 kernel trace: for the step window between two
occurrences of the first kernel of a step, sum kernel busy time (union of
intervals) vs wall time, and list the largest idle gaps.

  python tools/tracegaps.py gpurun_out/profX/run_kernel_trace.csv [marker-substring]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "rng_advance"
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90], r["Queue_Id"])
             for r in rows), key=lambda x: x[0])
starts = [i for i, k in enumerate(ks) if marker in k[2]]
print(f"{len(ks)} kernels, {len(starts)} step markers")
if len(starts) < 3:
    sys.exit(0)
a, b = starts[-3], starts[-2]                    # one full step late in the run
win = ks[a:b]
t0, t1 = win[0][0], ks[b][0]
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, n, q in win:
    if cur_e is None:
        cur_s, cur_e = s, e
        continue
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"step wall {(t1 - t0) / 1e3:.1f} us, busy (union) {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us, "
      f"{len(win)} kernels, queues {sorted(set(k[3] for k in win))}")
tot = sum(e - s for s, e, _, _ in win)
print(f"sum of kernel durations {tot / 1e3:.1f} us (overlap = {(tot - busy) / 1e3:.1f} us)")
gaps.sort(reverse=True)
print("largest gaps before:")
for g, n in gaps[:12]:
    print(f"  {g / 1e3:7.1f} us  {n}")
import collections
hist = collections.Counter(min(int(g / 1000), 10) for g, _ in gaps)
print("gap histogram (us bucket: count):", dict(sorted(hist.items())))

# per-kernel-family time inside the step window
fam = collections.defaultdict(lambda: [0, 0])
for s, e, n, q in win:
    key = n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:70]
    fam[key][0] += e - s
    fam[key][1] += 1
print("\nper kernel (one step):")
for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"  {t / 1e3:8.1f} us  {c:4d}x  {k}")
