"""The data-parallel step (dp.DataParallelStep: the backward as stage graphs, the bucketed async
RCCL all-reduce of each stage's finished buckets issued between them on a comm stream and
overlapped with the later stages, + the (id, row) all-gather for the embedding) at world_size 1
on one MI355X: every exchange is then an identity, so it must reproduce the single-GPU graph step
bit for bit.  Multi-rank arithmetic is covered by tests/test_dp_cpu.py and
tests/test_a_dp2_gpu.py (gloo)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

# The world-1 RCCL group -- and the communicator's threads -- live only in a child process that runs
# this module's cases: one r06 full-suite run segfaulted inside hipGraphLaunch of a plain engine
# graph replayed in the same process as a live RCCL communicator (the next run of the same tree
# passed; DESIGN §3.8, "Graph hygiene").  The parent process never initialises RCCL.
_CHILD = os.environ.get("VQA_DP_CHILD") == "1"


def test_dp_world1_cases_in_a_child_process():
    if _CHILD:
        pytest.skip("the child runs the cases themselves")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", os.path.abspath(__file__), "-m", "gpu", "-x", "-v",
                        "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread"],
                       cwd=root, env={**os.environ, "VQA_DP_CHILD": "1"}, timeout=370, capture_output=True, text=True)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0, f"world-1 RCCL cases failed in the child (rc {r.returncode})"
    import re
    m = re.search(r"(\d+) passed", r.stdout)
    assert m and int(m.group(1)) == 6 and "failed" not in r.stdout, "the child must run and pass all 6 cases"


@pytest.fixture(scope="module")
def pg(pkg):
    if not _CHILD:
        pytest.skip("runs in the child process (test_dp_world1_cases_in_a_child_process)")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


# (r04: a form that captured the collectives INTO the backward graph segfaulted in capture_end
# when it followed eager async collectives on the same communicator, profiles/r04_rccl_capture.txt;
# no collective is captured any more -- the stage graphs hold kernels only -- so the cases run in
# their natural order)
@pytest.mark.parametrize("graph,pipe", [(False, False), (False, True), (True, False), (True, True)])
def test_dp_world1_matches_single_gpu(pg, pkg, graph, pipe):
    """World-1 DP (bucketed all-reduce, gathered-row embedding scatter, segmented graphs; with
    `pipe` also the separately replayed next-batch ResNet) == the single-GPU step, bit for bit,
    over distinct batches per step, and with a local backward run before the DP object exists
    (its embedding-gradient rows must not leak into the DP steps)."""
    B, L, H = 4, 32, 96
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    nbs = [pkg.synthetic.make_batch(B, L, H, seed=1 + i) for i in range(5)]
    dev = [{k: torch.as_tensor(v).cuda() for k, v in nb.items() if v is not None} for nb in nbs]
    e1 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, pipeline=pipe)
    # the DP engine batches the T5 weight gradients in groups of 4 layers (bench.py), the
    # single-GPU one over all 12: same bits, different bucket boundaries
    e2 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, t5_dw_group=(4, 4, 3, 1), pipeline=pipe)
    junk = dev[4]                                    # a local step on another batch, before DP exists
    for e in (e1, e2):
        if pipe:
            e.prime(junk["image_tensors"])
            e.F4.copy_(e.F4N)
            e.load_batch(junk, next_images=dev[0]["image_tensors"])
        else:
            e.load_batch(junk)
        e.forward()
        e.backward()
        e.RNG[1] = 0
    if graph:
        e1.capture()
    step = pkg.dp.DataParallelStep(e2, bucket_mb=8, use_graph=graph)
    assert len(step.buckets) >= 5
    for e in (e1, e2):
        if pipe:
            e.prime(dev[0]["image_tensors"])
    for i in range(3):
        for e in (e1, e2):
            if pipe:
                e.load_batch(dev[i], next_images=dev[i + 1]["image_tensors"])
            else:
                e.load_batch(dev[i])
        e1.train_step()
        step.step()
        torch.cuda.synchronize()
        assert float(e1.LOSS) == float(e2.LOSS), i
    assert torch.equal(e1.G32, e2.G32)
    e1.flush_optimizer()
    e2.flush_optimizer()
    assert torch.equal(e1.P32, e2.P32)


def test_dp_world1_sharded_optimizer_rccl(pg, pkg):
    """The sharded optimizer's RCCL path (reduce-scatter into the per-bucket output buffer, copy
    into the own chunk, sharded AdamW, all-gather of the fp32 masters and bf16 shadows) at world 1:
    the trajectory of the single-GPU step.  Multi-rank arithmetic: tests/test_a_dp2_gpu.py (gloo)."""
    B, L, H = 4, 32, 96
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    nbs = [pkg.synthetic.make_batch(B, L, H, seed=1 + i) for i in range(3)]
    dev = [{k: torch.as_tensor(v).cuda() for k, v in nb.items() if v is not None} for nb in nbs]
    e1 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20)
    e2 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, t5_dw_group=(4, 4, 3, 1))
    # e3: the same sharded step with bench.py's collective timing on -- its timing stream only
    # waits on the collectives (it once also re-ran the reduce-scatter's follow-up copy,
    # unordered with the next step's backward); bit-identical to e2
    e3 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, t5_dw_group=(4, 4, 3, 1))
    e1.capture()
    step = pkg.dp.DataParallelStep(e2, bucket_mb=8, use_graph=True, shard_optimizer=True)
    step3 = pkg.dp.DataParallelStep(e3, bucket_mb=8, use_graph=True, shard_optimizer=True)
    step3.timing = True
    for i in range(3):
        for e in (e1, e2, e3):
            e.load_batch(dev[i])
        e1.train_step()
        step.step()
        step3.step()
        torch.cuda.synchronize()
        assert float(e1.LOSS) == float(e2.LOSS) == float(e3.LOSS), i
        n1, n2 = e1.last_grad_norm(), e2.last_grad_norm()
        assert abs(n1 - n2) <= 1e-6 * abs(n1), (i, n1, n2)
        assert torch.equal(e2.G32, e3.G32), i
    assert step3.timing_report()["steps"] == 3
    for e in (e1, e2, e3):
        e.flush_optimizer()
    step.sync_optimizer_state()
    step3.sync_optimizer_state()
    rel = float((e1.P32 - e2.P32).norm() / e1.P32.norm())
    assert rel <= 1e-6, rel
    vrel = float((e1.VMAX - e2.VMAX).norm() / e1.VMAX.norm())
    assert vrel <= 1e-5, vrel
    assert torch.equal(e2.P32, e3.P32) and torch.equal(e2.M, e3.M) and torch.equal(e2.VMAX, e3.VMAX)


def test_dp_exchange_never_queues_stage_work_behind_a_collective(pg, pkg, monkeypatch):
    """The placement DESIGN §5 states, asserted on the issue order of one graphed, pipelined
    world-1 DP step: every collective is issued on the comm stream (never on the step's stream,
    whose packets the stage graphs follow), every wait on a collective is issued on the step's
    stream and only after the LAST stage graph has been replayed (a wait packet holds back every
    later packet of its hardware queue), and the finish graph comes after those waits.  The one
    exception is the step's opening exchange -- the valid-row count (engine.use_global_rows) and
    the token-id gather: issued before the forward graph, waited on between the forward and the
    first stage (the head backward reads the count, the first stage the ids) -- two small
    collectives that have had the whole forward to finish."""
    dpm = pkg.dp
    B, L, H = 4, 32, 96
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    nb = {k: torch.as_tensor(v).cuda() for k, v in pkg.synthetic.make_batch(B, L, H, seed=1).items() if v is not None}
    e = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, t5_dw_group=(4, 4, 3, 1),
                             pipeline=True)
    e.prime(nb["image_tensors"])
    e.F4.copy_(e.F4N)
    e.load_batch(nb, next_images=nb["image_tensors"])
    step = dpm.DataParallelStep(e, bucket_mb=8, use_graph=True)
    step.step()                                      # captured and run once
    torch.cuda.synchronize()
    log = []
    main = torch.cuda.current_stream()

    class _W:
        def __init__(self, w):
            self.w = w

        def wait(self):
            log.append(("wait", torch.cuda.current_stream() == main))
            return self.w.wait()

        def __getattr__(self, k):
            return getattr(self.w, k)
    real_ar, real_ag = dist.all_reduce, dist.all_gather_into_tensor

    def all_reduce(*a, **kw):
        log.append(("collective", torch.cuda.current_stream() == main))
        return _W(real_ar(*a, **kw))

    def all_gather_into_tensor(*a, **kw):
        log.append(("collective", torch.cuda.current_stream() == main))
        return _W(real_ag(*a, **kw))
    monkeypatch.setattr(dist, "all_reduce", all_reduce)
    monkeypatch.setattr(dist, "all_gather_into_tensor", all_gather_into_tensor)
    real_osw = dpm._OnStream.wait

    def on_stream_wait(self):                        # collectives enqueued on the comm stream (COMM_ON_STREAM)
        log.append(("wait", torch.cuda.current_stream() == main))
        return real_osw(self)
    monkeypatch.setattr(dpm._OnStream, "wait", on_stream_wait)
    for name, g in step.graphs.items():
        monkeypatch.setattr(g, "replay", (lambda n, r: (lambda: (log.append(("graph", n)), r())[1]))(name, g.replay))
    e.load_batch(nb, next_images=nb["image_tensors"])
    step.step()
    torch.cuda.synchronize()
    # the opening exchange -- the valid-row count and the token-id gather -- first (before the
    # forward graph), its waits right after it
    assert log[:5] == [("collective", False)] * 2 + [("graph", "fwd")] + [("wait", True)] * 2, log
    log = log[2:3] + log[5:]
    kinds = [k for k, _ in log]
    assert "collective" in kinds and "wait" in kinds, log
    assert all(not on_main for k, on_main in log if k == "collective"), log   # collectives: comm stream
    assert all(on_main for k, on_main in log if k == "wait"), log             # waits: the step's stream
    stages = [i for i, x in enumerate(log) if x[0] == "graph" and x[1].startswith("stage")]
    waits = [i for i, x in enumerate(log) if x[0] == "wait"]
    finish = [i for i, x in enumerate(log) if x == ("graph", "finish")]
    assert stages and finish and min(waits) > max(stages) and max(waits) < finish[0], log
