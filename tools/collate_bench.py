"""Throughput of the input pipeline (data.DaquarCollate) against the train step.

  python tools/collate_bench.py [OUT.json] [--batches N] [--workers 0,4,8,16]

Writes 64 DAQUAR-like JPEGs (640 x 480 NYU-Depth frames, quality 90, random smooth
content so they compress like photographs) to a temp dir, then times, per decode-pool
size: host JPEG decode alone (PIL, `decode_workers` threads) and, with a GPU, the whole
collate (decode + pack + one H2D copy + the resize / ToTensor launch + question padding)
in pairs/s over N batches of 64.  The step consumes ~9,460 pairs/s (config 2, one GPU)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402


def make_jpegs(d, n=64, seed=0):
    from PIL import Image
    g = np.random.default_rng(seed)
    paths = []
    for i in range(n):
        # low-frequency content (a photograph-like spectrum): upsampled noise + gradients
        base = g.integers(0, 256, (30, 40, 3)).astype(np.float32)
        im = Image.fromarray(base.astype(np.uint8)).resize((640, 480), Image.BILINEAR)
        a = np.asarray(im).astype(np.float32) + g.normal(0, 6, (480, 640, 3))
        p = os.path.join(d, f"img{i:03d}.jpg")
        Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(p, quality=90)
        paths.append(p)
    return paths


def main():
    args = sys.argv[1:]
    out = args[0] if args and not args[0].startswith("--") else None
    nb = int(args[args.index("--batches") + 1]) if "--batches" in args else 8
    workers = [int(w) for w in (args[args.index("--workers") + 1] if "--workers" in args else "0,4,8,16").split(",")]
    pkg = load_package()
    gpu = torch.cuda.is_available()
    res = {"batch": 64, "batches": nb, "image": "640x480 JPEG q90", "host_threads_visible": os.cpu_count(),
           "gpu": gpu, "runs": []}
    with tempfile.TemporaryDirectory() as d:
        paths = make_jpegs(d)
        res["jpeg_bytes_mean"] = int(np.mean([os.path.getsize(p) for p in paths]))
        dps = [{"image_path": p, "question_ids": [5, 6, 7, 1], "annotation_id": i % 170} for i, p in enumerate(paths)]
        for w in workers:
            col = pkg.data.DaquarCollate((224, 224), 32, device="cuda" if gpu else "cpu", decode_workers=w) \
                if gpu else None
            dec = pkg.data.DaquarCollate.__new__(pkg.data.DaquarCollate)     # decode-only twin (no GPU)
            dec._pool = None
            if w:
                from concurrent.futures import ThreadPoolExecutor
                dec._pool = ThreadPoolExecutor(max_workers=w)
            dec._decode(dps)                                                 # warm the page cache / pool
            t0 = time.perf_counter()
            for _ in range(nb):
                dec._decode(dps)
            t_dec = (time.perf_counter() - t0) / nb
            r = {"decode_workers": w, "decode_pairs_per_s": round(64 / t_dec, 1)}
            if gpu:
                col(dps)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(nb):
                    col(dps)
                torch.cuda.synchronize()
                t_all = (time.perf_counter() - t0) / nb
                r["collate_pairs_per_s"] = round(64 / t_all, 1)
            res["runs"].append(r)
            print(r, flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
