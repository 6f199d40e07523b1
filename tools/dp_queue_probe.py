"""Which hardware queue does each stream of the DP step use?  

Run under `rocprofv3 --kernel-trace` (the trace's kernel rows carry queue ids; graph-replayed
kernels report stream 0, eager ones their stream): builds the world-1 RCCL DataParallelStep at the
bench shapes (B = 64, pipelined, graphed), runs 4 DP steps, then launches one marker kernel (a
1-element torch add) on each of the step's own streams and on CANDIDATES fresh torch streams made
after the capture, one at a time with a synchronize between them, in this order:
  main, comm, tstream, engine side, wside, rstream, cand0 .. cand{N-1}
`python tools/dp_queue_probe.py --analyse <db>` prints, for the last DP step, the kernels per
queue, and the queue of each marker (in launch order).
  python tools/dp_queue_probe.py [CANDIDATES]
"""
import json
import os
import sqlite3
import sys
import types

if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
    nmark = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    c = sqlite3.connect(sys.argv[2])
    rows = c.execute("select start, end, name, queue_id, stream_id from kernels order by start").fetchall()
    marks = [r for r in rows if "elementwise" in r[2]][-nmark:]
    idx = [i for i, r in enumerate(rows) if "rng_advance" in r[2]]
    step = rows[idx[-1]:rows.index(marks[0])]               # the last DP step, up to the markers
    graph_q, eager = {}, []
    for r in step:
        if r[4] == 0:
            graph_q[r[3]] = graph_q.get(r[3], 0) + 1
        else:
            eager.append((r[2][:40], r[3], r[4]))
    comm_q = {q for _, q, _ in eager}
    print(json.dumps({"graph_kernels_per_queue": {str(k): v for k, v in sorted(graph_q.items())},
                      "eager_kernels (name, queue, stream)": eager,
                      "markers (queue, stream) in launch order": [(r[3], r[4]) for r in marks],
                      "comm_queue_carries_graph_kernels": bool(comm_q & set(graph_q))}, indent=1))
    sys.exit(0)

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

ncand = int(sys.argv[1]) if len(sys.argv) > 1 else 6
pkg = load_package()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist = bench.init_world1(dev)
args = types.SimpleNamespace(batch=64, seq_len=32, image_size=224, blocks=3, no_pipeline=False, dp_groups=False,
                             config5=False, tune_table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning",
                                                                    "gemm_gfx950.json"),
                             tune_save=None, no_graph=False, shard_optimizer=False, dp_res_split=None,
                             res_cumask=None)
pool = []
for i in range(2):
    nb = pkg.synthetic.make_batch(64, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng, dps, step = bench.make_step(args, pkg, dev, pool, True, 0, "t5-base")
cands = [torch.cuda.Stream(dev) for _ in range(ncand)]
for i in range(4):
    step(i)
torch.cuda.synchronize()
tiny = torch.zeros(1, device=dev)
named = [("main", torch.cuda.current_stream(dev)), ("comm", dps._comm), ("tstream", dps._tstream),
         ("side", eng._side), ("wside", eng._wside), ("rstream", eng._rstream)] + \
        [(f"cand{i}", s) for i, s in enumerate(cands)]
for name, s in named:
    with torch.cuda.stream(s):
        tiny.add_(1)
    torch.cuda.synchronize()
print(json.dumps({"markers": [n for n, _ in named], "stream_ids": [int(s.stream_id) for _, s in named]}))
dist.destroy_process_group()
