"""Does the step slow down with the number of hardware queues this process has materialised?
(the DP step at 8 queues, high-priority streams and a CU-masked
ResNet stream all doubled the step; the engine graph at 8 queues did not.)

Builds the benched engine (B = 64, 224², captured step graph), times graph replays with HIP
events, then repeatedly makes one more torch stream, runs one tiny kernel on it (HIP binds a
stream to a hardware queue at its first launch: round-robin over GPU_MAX_HW_QUEUES queues) and
times the replays again; finally a CU-masked stream (always a queue of its own) is created and
used once.  Nothing runs on the extra streams while the replays are timed.
  python tools/queue_probe.py [HW_QUEUES]      (GPU_MAX_HW_QUEUES for this process; default: inherited)
"""
import json
import os
import sys
import types

if len(sys.argv) > 1:                                  # before the HIP runtime starts
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1]

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
args = types.SimpleNamespace(batch=64, seq_len=32, image_size=224, blocks=3, no_pipeline=False, dp_groups=False,
                             config5=False, tune_table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning",
                                                                    "gemm_gfx950.json"),
                             tune_save=None, no_graph=False, shard_optimizer=False, dp_res_split=None,
                             res_cumask=None)
pool = []
for i in range(4):
    nb = pkg.synthetic.make_batch(64, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng, _, step = bench.make_step(args, pkg, dev, pool, False, 0, "t5-base")
main = torch.cuda.current_stream(dev)


def replay_ms(n=10):
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(main)
    for _ in range(n):
        eng.train_step()
    b.record(main)
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / n, 3)


def touch(s):
    with torch.cuda.stream(s):
        torch.ones(1, device=dev).add_(1)
    torch.cuda.synchronize()


rows = [{"extra_streams": 0, "step_ms": replay_ms()}]
keep = []
for k in range(1, 9):
    s = torch.cuda.Stream(dev)
    touch(s)
    keep.append(s)
    rows.append({"extra_streams": k, "step_ms": replay_ms()})
graph = eng.graph
eng.set_res_cumask(bench.cumask_words("all", torch.cuda.get_device_properties(dev).multi_processor_count))
masked, handle = eng.reset_res_cumask(destroy=False)  # the engine's own ResNet stream again; the
eng.graph = graph                                      # masked one exists and is used once, the step unchanged
touch(masked)
rows.append({"extra_streams": "8 + one CU-masked (own queue)", "step_ms": replay_ms()})
torch.cuda.synchronize()
pkg.lib.hip_runtime().hipStreamDestroy(handle)
print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "rows": rows}))
