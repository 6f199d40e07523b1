"""Summarise rocprofv3 PMC passes of the benched step and of tools/kernel_replay.py.

  python tools/pmc_step.py OUT.json STEP_FETCH STEP_WRITE STEP_MFMA REP_FETCH REP_WRITE REP_MFMA MANIFEST.json

STEP_* are `rocprofv3 --pmc <counters> -f csv` output directories of
`bench.py --steps 3 --warmup 1 --no-kernel-rooflines --no-cpu-baseline`;
REP_* the same three passes over tools/kernel_replay.py.  Passes:
FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read,
so fetch bytes = 2 x 1024 x FETCH_SIZE; write bytes = 1024 x WRITE_SIZE.
MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES = 32 cycles per v_mfma_f32_32x32x16_bf16
summed over every SIMD, so busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) is
the fraction of the matrix pipes' cycles used while the kernel ran (at the
clock it ran at); FLOP / 1024 is what the algorithmic work alone would give.

Step grouping: dispatches are ordered by id; a step is the span between two
consecutive `rng_advance` dispatches (the forward's first launch); the last two
complete spans (timed steps) are averaged."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert fs, f"no counter_collection.csv under {d}"
    disp = {}
    for r in csv.DictReader(open(fs[0])):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "c": defaultdict(float)})
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def steps(ds):
    idx = [i for i, d in enumerate(ds) if "rng_advance" in d["name"]]
    spans = [ds[a:b] for a, b in zip(idx, idx[1:])]
    return spans[-2:]


def total(span, counter):
    return sum(d["c"].get(counter, 0.0) for d in span)


def main():
    out, sf, sw, sm, rf, rw, rm, man = sys.argv[1:9]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import tree_digest
    # the tree the passes ran on: bench.py quotes these counters only while its digest matches
    res = {"tree_digest": tree_digest(), "commit": os.environ.get("PMC_COMMIT"),
           "correction": "fetch = 2 x 1024 x FETCH_SIZE (gfx950 half-count); write = 1024 x WRITE_SIZE"}
    F, W, M = steps(load(sf)), steps(load(sw)), steps(load(sm))
    n = [len(s) for s in F + W + M]
    fetch = sum(2048.0 * total(s, "FETCH_SIZE") for s in F) / len(F)
    write = sum(1024.0 * total(s, "WRITE_SIZE") for s in W) / len(W)
    busy = sum(total(s, "SQ_VALU_MFMA_BUSY_CYCLES") for s in M) / len(M)
    grbm = sum(total(s, "GRBM_GUI_ACTIVE") for s in M) / len(M)
    res["step"] = {"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                   "mfma_busy_cycles": busy, "mfma_flop_equiv": busy * 1024.0,
                   "dispatches_per_step": n, "note": "sum over every dispatch of one step (all streams)"}
    mf = json.load(open(man))["dispatches"]
    per = {}
    for path, key in ((rf, "fetch"), (rw, "write"), (rm, "mfma")):
        ds = load(path)[-len(mf):]
        assert len(ds) == len(mf), (path, len(ds), len(mf))
        for d, m in zip(ds, mf):
            e = per.setdefault(m["tag"], defaultdict(float))
            e["n"] += 1 if key == "fetch" else 0
            if key == "fetch":
                e["fetch_bytes"] += 2048.0 * d["c"]["FETCH_SIZE"]
                e["flop"] += m["flop"]
                e["alg_bytes"] += m["bytes"]
            elif key == "write":
                e["write_bytes"] += 1024.0 * d["c"]["WRITE_SIZE"]
            else:
                e["mfma_busy_cycles"] += d["c"]["SQ_VALU_MFMA_BUSY_CYCLES"]
                e["grbm_gui_active"] += d["c"]["GRBM_GUI_ACTIVE"]
    reps = json.load(open(man))["reps"]
    for tag, e in per.items():
        e = {k: v / reps for k, v in e.items()}           # per launch set (one pass over the tag's calls)
        e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        if e["grbm_gui_active"] > 0:
            e["mfma_pipe_frac"] = e["mfma_busy_cycles"] / (1024.0 * e["grbm_gui_active"] / 8.0)
        if e["flop"] > 0:
            e["busy_vs_flop"] = e["mfma_busy_cycles"] * 1024.0 / e["flop"]
        res[tag] = e
    if "adamw" in res:
        res["adamw_kernel"] = {"traffic_bytes": res["adamw"]["traffic_bytes"],
                               "algorithmic_bytes": res["adamw"]["alg_bytes"]}
    if "convT_dW" in res:
        res["convT_dW"] = dict(res["convT_dW"])
    for tag, e in per.items():                             # measured HBM traffic over the algorithmic bytes
        if tag in res and res[tag].get("alg_bytes"):
            res[tag]["traffic_over_alg"] = res[tag]["traffic_bytes"] / res[tag]["alg_bytes"]
    if "sga_gemm" in res:
        g = res["sga_gemm"]
        res["sga_mfma_busy"] = {"mfma_pipe_frac_gemm": g.get("mfma_pipe_frac"),
                                "mfma_pipe_frac_all": (g["mfma_busy_cycles"] + res.get("sga_attn", {}).get(
                                    "mfma_busy_cycles", 0.0)) / (1024.0 * (g["grbm_gui_active"] + res.get(
                                        "sga_attn", {}).get("grbm_gui_active", 0.0)) / 8.0),
                                "source": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8), "
                                          "tools/kernel_replay.py launches replayed alone"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
