"""Graph-capture investigation of the late-session hipGraphLaunch SIGSEGV.

  python tools/graph_probe.py audit            node-type census of every graph the engines capture
  python tools/graph_probe.py churn N          N build / capture / replay / rebuild / destroy cycles
                                               of small engines in ONE process, then the bench graph

audit: captures the benched step (R50, B=64, pipelined, deferred AdamW) and a small DP-style
engine with keep_graph=True, walks each hipGraph_t with hipGraphGetNodes / hipGraphNodeGetType
and prints how many nodes of each type it holds.  Any memcpy / memset / host node is a node the
runtime executes through its own blit path or host callback (not a library kernel).

churn: the product path's engine rebuilds (model.load_state_dict -> _build, the DP rebuild in
VQATrainer) and the test session's hundreds of captures, in one process: prints free device
memory and the per-cycle wall time, so a leak in the runtime's graph bookkeeping shows as a
trend, and a crash names the cycle it happened in."""
import ctypes
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "child_graph", 5: "empty", 6: "wait_event",
              7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free",
              12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


def census(graph_handle):
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(ctypes.c_void_p(graph_handle), None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(ctypes.c_void_p(graph_handle), nodes, ctypes.byref(n)) == 0
    out = {}
    for i in range(n.value):
        t = ctypes.c_int(-1)
        assert hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) == 0
        k = NODE_TYPES.get(t.value, str(t.value))
        out[k] = out.get(k, 0) + 1
    return out


def _capture_kept(fn, s):
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=s):
        fn()
    return g


def audit():
    pkg = load_package()
    E = pkg.engine
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    res = {}
    for name, kw in (("bench_b64", dict(batch=64, seq_len=32, image_size=224, pipeline=True)),
                     ("small_unpipelined", dict(batch=4, seq_len=16, image_size=64, pipeline=False))):
        eng = E.VQAEngine(sd, vision="resnet50", dropout=0.1, seed=0, **kw)
        nb = pkg.synthetic.make_batch(kw["batch"], kw["seq_len"], kw["image_size"], seed=1)
        if eng.pipeline:
            eng.prime(torch.as_tensor(nb["image_tensors"]).cuda())
        eng.load_batch(nb, next_images=nb["image_tensors"] if eng.pipeline else None)
        eng.forward()
        eng.backward()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with E.no_gc_capture():
            g = _capture_kept(eng._step_pipelined if eng.pipeline else eng._run_step_streams, s)
        res[name] = census(g.raw_cuda_graph())
        g.instantiate()
        g.replay()
        torch.cuda.synchronize()
        print(name, res[name], flush=True)
        del g, eng
        gc.collect()
    return res


def churn(n):
    pkg = load_package()
    E = pkg.engine
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    nb = pkg.synthetic.make_batch(4, 16, 64, seed=1)
    t0 = time.time()
    for i in range(n):
        t = time.time()
        eng = E.VQAEngine(sd, vision="resnet50", batch=4, seq_len=16, image_size=64, dropout=0.1, seed=0,
                          pipeline=(i % 2 == 0))
        if eng.pipeline:
            eng.prime(torch.as_tensor(nb["image_tensors"]).cuda())
        eng.load_batch(nb, next_images=nb["image_tensors"] if eng.pipeline else None)
        eng.forward()
        eng.backward()
        eng.capture()
        for _ in range(3):
            eng.train_step()
        torch.cuda.synchronize()
        lp = float(eng.LOSS.item())
        # rebuild from the engine's own state dict, as model.load_state_dict does, and replay
        # the new engine's graph while the old one is still alive
        eng2 = E.VQAEngine(eng.state_dict(), vision="resnet50", batch=4, seq_len=16, image_size=64, dropout=0.1,
                           seed=0)
        eng2.load_batch(nb)
        eng2.forward()
        eng2.backward()
        eng2.capture()
        eng2.train_step()
        torch.cuda.synchronize()
        del eng, eng2
        if i % 3 == 0:
            gc.collect()
        if i % 10 == 0 or i == n - 1:
            free, total = torch.cuda.mem_get_info()
            print(f"cycle {i}: loss {lp:.4f} free {free / 2**30:.1f} GiB  {time.time() - t:.2f} s/cycle "
                  f"({time.time() - t0:.0f} s)", flush=True)
    gc.collect()
    torch.cuda.empty_cache()
    # the benched graph after the churn (where the crash was seen)
    sdb = pkg.synthetic.make_state_dict("resnet50", seed=0)
    eng = E.VQAEngine(sdb, vision="resnet50", batch=64, seq_len=32, image_size=224, dropout=0.1, seed=0,
                      pipeline=True)
    nb64 = pkg.synthetic.make_batch(64, 32, 224, seed=1)
    img = torch.as_tensor(nb64["image_tensors"]).cuda()
    eng.prime(img)
    eng.load_batch(nb64, next_images=img)
    eng.forward()
    eng.backward()
    eng.capture()
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    print("bench graph after churn: loss", float(eng.LOSS.item()), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "audit":
        audit()
    else:
        churn(int(sys.argv[2]))
