"""Where the time goes when the frozen ResNet runs on a stream with a hardware queue of its own
(engine.set_res_cumask: hipExtStreamCreateWithCUMask; bench.py --res-cumask), the configuration
that doubles the step (profiles/r05_queue_probe.txt).  HIP events on each stream, no tracer (the
tracer hides the effect: DESIGN §5):
  A  the chain graph alone (main stream)
  R  the ResNet alone, eager on the dedicated-queue stream
  R0 the ResNet alone, eager on an ordinary torch stream (shares the 4 default queues)
  AR both, as the --res-cumask step issues them
  [MAIN_SIDE=1] python tools/cumask_probe.py [SPEC]   (SPEC as bench.py --res-cumask, default all;
                                                       MAIN_SIDE: the step on a non-default stream)
"""
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "all"
pkg = load_package()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if os.environ.get("MAIN_SIDE"):                  # issue everything on a stream of its own, not the null stream
    torch.cuda.set_stream(torch.cuda.Stream(dev))
args = types.SimpleNamespace(batch=64, seq_len=32, image_size=224, blocks=3, no_pipeline=False, dp_groups=False,
                             config5=False, tune_table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning",
                                                                    "gemm_gfx950.json"),
                             tune_save=None, no_graph=False, shard_optimizer=False, dp_res_split=None,
                             res_cumask=spec)
pool = []
for i in range(4):
    nb = pkg.synthetic.make_batch(64, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng, _, step = bench.make_step(args, pkg, dev, pool, False, 0, "t5-base")
main = torch.cuda.current_stream(dev)
plain = torch.cuda.Stream(dev)


def timed(fn, n=10, streams=(main,)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    for (a, _), s in zip(evs, streams):
        a.record(s)
    for _ in range(n):
        fn()
    for (_, b), s in zip(evs, streams):
        b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b) / n, 4) for a, b in evs]


def chain():
    for g in eng.graph:
        g.replay()


def res_on(s):
    def f():
        with torch.cuda.stream(s):
            eng._run(eng.res_calls)
    return f


out = {"spec": spec, "main_stream": "side" if os.environ.get("MAIN_SIDE") else "default",
       "A_chain_graph_ms": timed(chain),
       "R_resnet_dedicated_queue_ms": timed(res_on(eng._rstream), streams=(eng._rstream,)),
       "R0_resnet_shared_queue_ms": timed(res_on(plain), streams=(plain,)),
       "AR_step_ms": timed(eng.train_step),
       "AR_chain_and_resnet_ms (main, rstream)": timed(eng.train_step, streams=(main, eng._rstream))}
print(json.dumps(out))
