"""Graph-capture hygiene of the step (the late-session hipGraphLaunch SIGSEGV).

* every captured step graph holds kernel nodes only: no runtime memcpy / memset / host node
  (a host node or a copy out of pageable memory would make a replay read host memory);
* every prepared call's `keep` owns every address the call passes (ops.uncovered_pointers):
  a buffer freed behind a captured node's back is exactly the kind of fault that shows up
  late in a long process;
* an engine rebuilt in the same process (ResnetVQAModel.load_state_dict -> _build, as the
  reference's init_model loads best-model.pt, train_faster_rcnn_vqa.py:40-45) captures and
  replays next to the old one, and the rebuilt step equals a fresh engine's bit for bit
  (trainer/faster_rcnn_vqa_trainer.py:391-406)."""
import ctypes
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "child_graph", 5: "empty", 6: "wait_event",
              7: "event_record", 10: "mem_alloc", 11: "mem_free"}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch


def census(graph_handle, pkg):
    # the runtime torch already runs: a CDLL by file name can map /opt/rocm's copy beside it, a
    # second HIP runtime in the process (its graph calls on the first one's objects; the replay
    # that followed segfaulted on the host in two suite runs)
    hip = pkg.lib.hip_runtime()
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


def _engine(pkg, torch, pipeline, B=4, L=16, H=64, sd=None, **kw):
    sd = sd if sd is not None else pkg.synthetic.make_state_dict("resnet50", seed=0)
    eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=L, image_size=H, dropout=0.1, seed=0,
                               pipeline=pipeline, **kw)
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    if pipeline:
        img = torch.as_tensor(nb["image_tensors"]).cuda()
        eng.prime(img)
        eng.load_batch(nb, next_images=img)
    else:
        eng.load_batch(nb)
    return eng, nb


@pytest.mark.parametrize("pipeline", [True, False])
def test_step_graph_is_kernel_only(torch_cuda, pkg, pipeline):
    torch = torch_cuda
    eng, _ = _engine(pkg, torch, pipeline)
    eng.capture(keep_graph=True)
    (g,) = eng.graph
    c = census(g.raw_cuda_graph(), pkg)
    assert set(c) == {"kernel"}, c
    n_calls = len(eng.fwd_calls) + len(eng.bwd_calls) + len(eng.opt_calls) + len(eng.adam_segs)
    assert c["kernel"] >= n_calls, (c, n_calls)
    eng.train_step()
    torch.cuda.synchronize()
    assert np.isfinite(float(eng.LOSS.item()))


def test_prepared_calls_keep_every_pointer(torch_cuda, pkg):
    torch = torch_cuda
    eng, _ = _engine(pkg, torch, True)
    calls = list(eng.res_calls) + eng.fwd_calls + eng.bwd_calls + eng.opt_calls + eng.zero_calls + \
        [c for _, c in eng.adam_segs] + [eng.clear_pending, eng.copy_f4, eng.adam_full]
    if eng.adam_embed is not None:
        calls.append(eng.adam_embed)
    calls += list(eng.emb_pre) + list(eng.tail_calls)      # the embedding rows' split update
    assert eng.emb_pre, "the stream step splits the embedding table's update by rows"
    bad = {}
    for c in calls:
        for sub in getattr(c, "calls", [c]):               # engine._Seq groups
            u = pkg.ops.uncovered_pointers(sub)
            if u:
                bad.setdefault(sub.name, []).extend(u)
    assert not bad, bad
    # after a tuning pass (split-K workspaces are attached to the calls) too
    eng.forward()
    eng.backward()
    eng.autotune(table=None, reps=1)
    for c in eng.fwd_calls + eng.bwd_calls:
        assert not pkg.ops.uncovered_pointers(c), (c.name, pkg.ops.uncovered_pointers(c))


def test_rebuild_recapture_replay_in_process(torch_cuda, pkg):
    """build -> capture -> replay -> model.load_state_dict rebuild -> recapture -> replay, with
    the old engine's graph still alive, in this process; the rebuilt engine's step equals a
    fresh engine built from the same state dict, bit for bit."""
    torch = torch_cuda
    B, L, H = 4, 16, 64
    m = pkg.model.ResnetVQAModel("resnet50", "t5-base", 170, device="cuda", batch_size=B, seq_len=L,
                                 image_size=H, dropout=0.1)
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    items = {k: (torch.as_tensor(v).cuda() if v is not None else None) for k, v in nb.items()}
    tr = pkg.trainer.VQATrainer(m, {"kwargs": {"weight_decay": 0.1}}, {"num_warmup_steps": 2}, num_training_steps=20)
    for _ in range(2):
        tr.train_one_step(items)
    old = m.engine                                          # keep the old engine and its graph alive
    sd = m.state_dict()
    m.load_state_dict(sd)
    assert m.engine is not old and old.graph is not None
    losses = [tr.train_one_step(items)[0] for _ in range(2)]
    lp = m.engine.LOGP.clone()
    old.train_step()                                        # the old graph still replays
    torch.cuda.synchronize()
    fresh = pkg.model.ResnetVQAModel("resnet50", "t5-base", 170, device="cuda", batch_size=B, seq_len=L,
                                     image_size=H, dropout=0.1, state_dict=sd)
    tr2 = pkg.trainer.VQATrainer(fresh, {"kwargs": {"weight_decay": 0.1}}, {"num_warmup_steps": 2},
                                 num_training_steps=20)
    losses2 = [tr2.train_one_step(items)[0] for _ in range(2)]
    assert losses == losses2
    assert torch.equal(lp, fresh.engine.LOGP)
    del old, fresh, tr2
    gc.collect()
