"""Per-launch PMC table of tools/kernel_replay.py passes (median over the REPS dispatches
of each launch): duration from GRBM_GUI_ACTIVE / 8 XCDs, wave-cycle breakdown, LDS bank
conflicts, L2 hit rate, MFMA pipe use.

  python tools/pmc_kernels.py MANIFEST.json PASS_DIR [PASS_DIR ...]"""
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

man = json.load(open(sys.argv[1]))
disp = man["dispatches"]
vals = [defaultdict(float) for _ in disp]
names = [None] * len(disp)
for d in sys.argv[2:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    import csv
    rows = defaultdict(lambda: defaultdict(float))
    kn = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
        kn[k] = r["Kernel_Name"]
    ids = sorted(rows)[-len(disp):]
    for i, k in enumerate(ids):
        vals[i].update(rows[k])
        names[i] = kn[k]
reps = man["reps"]
print(f"{'tag':8s} {'shape':34s} {'us':>7s} {'TF/s':>6s} {'mfma%':>6s} {'wait%':>6s} {'inst%':>6s} {'act%':>5s} "
      f"{'ldsc/ldsi':>9s} {'L2hit':>6s}")
for i in range(0, len(disp), reps):
    m = disp[i]
    g = [vals[j] for j in range(i, i + reps)]
    med = lambda key: float(np.median([x.get(key, 0.0) for x in g]))
    cyc = med("GRBM_GUI_ACTIVE") / 8.0
    us = cyc / 2.1e3 if cyc else float("nan")          # ~2.1 GHz under load (reported clock is approximate)
    wc = med("SQ_WAVE_CYCLES") or 1.0
    hit, miss = med("TCC_HIT_sum"), med("TCC_MISS_sum")
    print(f"{m['tag']:8s} {str(m.get('shape')):34s} {us:7.1f} {m['flop'] / (us * 1e6) if us == us and m['flop'] else 0:6.0f} "
          f"{100 * med('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * cyc) if cyc else 0:6.1f} "
          f"{100 * med('SQ_WAIT_ANY') / wc:6.1f} {100 * med('SQ_WAIT_INST_ANY') / wc:6.1f} "
          f"{100 * med('SQ_ACTIVE_INST_ANY') / wc:5.1f} "
          f"{med('SQ_LDS_BANK_CONFLICT') / max(med('SQ_INSTS_LDS'), 1):9.2f} "
          f"{100 * hit / max(hit + miss, 1):6.1f}  {names[i][:60] if names[i] else ''}")
