"""One step of a rocprofv3 kernel trace (sqlite .db of ROCm 7.x), kernel by kernel.

  python tools/steptrace.py gpurun_out/X/run_results.db [marker] [--list] [--back N]

Finds the last complete step (between two launches whose name contains
`marker`, default rng_advance), prints the step wall time, per-queue busy
time, the idle gaps of the queue that carries the T5/SGA chain, and with
--list every kernel (start offset, duration, queue, name)."""
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "rng_advance"
# --back N: the N-th complete step from the end (default 2; bench --dp appends 3 timing steps)
c = sqlite3.connect(db)
rows = c.execute("select start, end, name, queue_id, stream_id from kernels order by start").fetchall()


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


idx = [i for i, r in enumerate(rows) if marker in r[2]]
back = int(sys.argv[sys.argv.index("--back") + 1]) if "--back" in sys.argv else 2   # which step from the end
a, b = idx[-1 - back], idx[-back]
win = rows[a:b]
t0, t1 = win[0][0], rows[b][0]
print(f"step wall {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels")
qs = sorted(set(r[3] for r in win))
for q in qs:
    ks = [r for r in win if r[3] == q]
    busy = sum(r[1] - r[0] for r in ks)
    print(f"queue {q}: {len(ks)} kernels, busy {busy / 1e3:.1f} us, span {(ks[-1][1] - ks[0][0]) / 1e3:.1f} us")
pairs = {}
for r in win:
    pairs[(r[4], r[3])] = pairs.get((r[4], r[3]), 0) + 1
print("(stream, queue): kernels  " + "  ".join(f"({s_},{q_}) {n_}" for (s_, q_), n_ in sorted(pairs.items())))
# union busy (any queue)
iv = sorted((r[0], r[1]) for r in win)
u, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"union busy {u / 1e3:.1f} us  (idle {(t1 - t0 - u) / 1e3:.1f} us)")
fam = {}
for s, e, n, q, _ in win:
    k = short(n).split("<")[0]
    fam[k] = fam.get(k, 0) + e - s
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:20]:
    print(f"  {v / 1e3:8.1f} us  {k}")
if "--list" in sys.argv:
    for s, e, n, q, sid in win:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} s{sid} {short(n)}")
