"""Why does the step graph captured WITHOUT the next batch's ResNet branch replay at ~2x the time
of the same chain inside the normal step graph?  

Builds the benched engine (B = 64, 224², pipelined, tuned) and captures several graphs of the
same step body that differ only in what sits beside / before the chain, then times back-to-back
replays of each with HIP events on the launch stream (no tracer: under rocprofv3 the effect
vanishes, profiles/r04_dp_ab.txt).
  full         the bench graph: F4 <- F4N, the ResNet branch forked first, the chain, join
  chain        the chain only (what --res-cumask captures)
  chain_stub   the chain with a 1-element torch kernel forked first on the ResNet stream, joined at the end
  chain_res1   the chain with the ResNet's first call only (the stem) forked first
  chain_x      the chain issued on a fresh stream forked from the capture stream after a 1-element
               kernel (the launch stream then carries only that kernel, the fork and the join)
  tiny_first   a 1-element kernel on the capture stream, then the chain
  [PRE=streams:K|cumask|prio] [POST=plain,all,hi:64,...] python tools/chain_probe.py [variant ...]
"""
import ctypes
import json
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

ALL = ["full", "chain", "chain_stub", "chain_res1", "chain_x", "tiny_first"]
variants = sys.argv[1:] or ALL
pkg = load_package()
E = pkg.engine
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
args = types.SimpleNamespace(batch=64, seq_len=32, image_size=224, blocks=3, no_pipeline=False, dp_groups=False,
                             config5=False, tune_table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning",
                                                                    "gemm_gfx950.json"),
                             tune_save=None, no_graph=True, shard_optimizer=False, dp_res_split=None,
                             res_cumask=None)
pool = []
for i in range(2):
    nb = pkg.synthetic.make_batch(64, 32, 224, seed=1 + i)
    pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
eng, _, _ = bench.make_step(args, pkg, dev, pool, False, 0, "t5-base")
eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
tiny = torch.zeros(1, device=dev)


def chain():
    eng.run_forward_streams()
    eng.run_backward_streams(sq_overlap=True)
    eng._run(eng.opt_calls[2:])


def forked(body, s):
    main = torch.cuda.current_stream(dev)
    f = torch.cuda.Event()
    f.record(main)
    s.wait_event(f)
    with torch.cuda.stream(s):
        body()
    j = torch.cuda.Event()
    j.record(s)
    return j


def v_full():
    E.VQAEngine._step_pipelined(eng)


def v_chain():
    chain()


def v_chain_stub():
    j = forked(lambda: tiny.add_(1), eng._rstream)
    chain()
    torch.cuda.current_stream(dev).wait_event(j)


def v_chain_res1():
    j = forked(lambda: eng._run(eng.res_calls[:1]), eng._rstream)
    chain()
    torch.cuda.current_stream(dev).wait_event(j)


_x = torch.cuda.Stream(dev)


def v_chain_x():
    tiny.add_(1)              # a node on the capture stream first (a fork from an empty capture crashed capture_end)
    j = forked(chain, _x)
    torch.cuda.current_stream(dev).wait_event(j)


def v_tiny_first():
    tiny.add_(1)
    chain()


BODY = {k: globals()["v_" + k] for k in ALL}


def capture(body):
    """The engine's own capture (warm-up launch on the capture stream, RNG / optimizer state
    restored) with the step body swapped (a hand-rolled capture on a fresh stream crashed the
    runtime in capture_end on the box)."""
    eng._step_pipelined = body
    try:
        eng.capture()
    finally:
        del eng._step_pipelined
    torch.cuda.synchronize()
    return eng.graph[0]


for st in (torch.cuda.current_stream(dev), eng._rstream, _x):      # torch's add kernel loaded before any capture
    with torch.cuda.stream(st):
        tiny.add_(1)
torch.cuda.synchronize()

# PRE: perturb the process's streams / hardware queues BEFORE any capture (a graph exec's
# internal parallel streams are bound to hardware queues when it is instantiated)
#   streams:K   K more torch streams, each used once (round-robin over the GPU_MAX_HW_QUEUES queues)
#   cumask      one CU-masked stream (all CUs; a hardware queue of its own), used once
#   prio        one high-priority torch stream (a queue of its own), used once
_pre = os.environ.get("PRE", "")
_held = []
if _pre.startswith("streams:"):
    for _ in range(int(_pre.split(":")[1])):
        _held.append(torch.cuda.Stream(dev))
elif _pre == "cumask":
    eng.set_res_cumask(bench.cumask_words("all", torch.cuda.get_device_properties(dev).multi_processor_count))
    _held.append(eng._rstream)
    eng.res_external = False                         # the ResNet branch stays in the captured graph bodies
elif _pre == "prio":
    _held.append(torch.cuda.Stream(dev, priority=-1))
for st in _held:
    with torch.cuda.stream(st):
        tiny.add_(1)
torch.cuda.synchronize()


def timed(g, n=10):
    main = torch.cuda.current_stream(dev)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(main)
    for _ in range(n):
        g.replay()
    b.record(main)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / n, 3), round(t_issue * 1e3 / n, 3)


graphs = {}
for v in variants:
    print("capture", v, file=sys.stderr, flush=True)
    graphs[v] = capture(BODY[v])
# POST=SPEC[,SPEC...]: AFTER the graphs are instantiated, for each cumask spec (bench.py --res-cumask
# syntax; "plain" = an ordinary pooled stream) create that stream and time the pipelined step as
# "chain graph on the launch stream || the next batch's ResNet launched eagerly on that stream"
# (F4 <- F4N first, joined at the end), plus the chain and full graphs again beside it.
_post = [x for x in os.environ.get("POST", "").split(",") if x]
_rs = {}
for spec in _post:
    if spec == "plain":
        _rs[spec] = torch.cuda.Stream(dev)
    else:
        import ctypes
        words = bench.cumask_words(spec, torch.cuda.get_device_properties(dev).multi_processor_count)
        h = ctypes.c_void_p()
        arr = (ctypes.c_uint32 * len(words))(*words)
        rc = pkg.lib.hip_runtime().hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
        assert rc == 0, rc
        _rs[spec] = torch.cuda.ExternalStream(h.value, device=dev)
    with torch.cuda.stream(_rs[spec]):
        tiny.add_(1)
torch.cuda.synchronize()


class _Overlap:
    """replay(): the chain graph beside the ResNet on stream `rs` (eager launches)."""
    def __init__(self, g, rs):
        self.g, self.rs = g, rs

    def replay(self):
        main = torch.cuda.current_stream(dev)
        eng.copy_f4(pkg.lib.stream_handle(main))
        f = torch.cuda.Event()
        f.record(main)
        self.g.replay()
        self.rs.wait_event(f)
        h = pkg.lib.stream_handle(self.rs)
        for c in eng.res_calls:
            c(h)
        j = torch.cuda.Event()
        j.record(self.rs)
        main.wait_event(j)


if _post and "chain" in graphs:
    for spec, rs in _rs.items():
        graphs["chain||res@" + spec] = _Overlap(graphs["chain"], rs)
    variants = list(graphs)
out = {"env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_", "HIP_", "AMD_", "GPU_", "ROC_", "PRE", "POST"))}}
for rep in range(2):                              # interleaved twice
    for v in variants:
        ms, host = timed(graphs[v])
        out.setdefault(v, []).append(ms)
        out.setdefault(v + "_host_ms", []).append(host)
print(json.dumps(out), flush=True)
torch.cuda.synchronize()
for spec, rs in _rs.items():                      # the CU-masked streams are ours to destroy
    if spec != "plain":
        pkg.lib.hip_runtime().hipStreamDestroy(ctypes.c_void_p(rs.cuda_stream))
