"""kernel_stats.csv (rocprofv3 --stats layout) from a rocprofv3 rocpd database.

  python tools/db_stats.py RUN_results.db OUT.csv

rocprofv3 on ROCm 7.2 writes its trace to a rocpd sqlite database unless `-f csv` is given;
this computes the same per-kernel summary (calls, total / average / min / max / stddev
duration in ns, share of total kernel time) from its `kernels` view."""
import csv
import math
import sqlite3
import sys
from collections import defaultdict

db, out = sys.argv[1:3]
rows = sqlite3.connect(db).execute("select name, end - start from kernels").fetchall()
per = defaultdict(list)
for name, d in rows:
    per[name].append(int(d))
total = sum(sum(v) for v in per.values())
with open(out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        n, s = len(v), sum(v)
        mu = s / n
        sd = math.sqrt(sum((x - mu) ** 2 for x in v) / n)
        w.writerow([name, n, s, round(mu, 6), round(100.0 * s / total, 2), min(v), max(v), round(sd, 6)])
