"""The data-parallel step with TWO ranks (tests/dp_worker.py, gloo, both on cuda:0):
every rank must end each step with bit-identical parameters, and the pair must
train like one engine on the global batch (2 x B samples): the per-rank NLL means
averaged equal the global mean, the summed-and-scaled gradients equal the
global-batch gradient up to fp32 summation order (trainer/faster_rcnn_vqa_trainer.py
:391-406 on the global batch).

The ranks are started before this process touches the GPU (this file sorts first in
the session; the skip check counts devices without initialising them)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return str(p)


def _ranks(tmp_path, world, steps, pipe, graph, mode="engine"):
    outs = [str(tmp_path / f"r{r}_{pipe}{graph}{mode}.npz") for r in range(world)]
    port = _port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), str(r), str(world), port, outs[r],
                               str(steps), str(int(pipe)), str(int(graph)), mode]) for r in range(world)]
    rcs = [p.wait(timeout=240 if mode == "c5" else 110) for p in procs]
    assert rcs == [0] * world, rcs
    return [np.load(o) for o in outs]


@pytest.fixture(scope="module")
def gpu():
    import torch
    if torch.cuda.device_count() < 1:                     # counts devices without initialising them
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("pipe,graph", [(False, True), (True, True)])
def test_dp_two_ranks_match_global_batch(gpu, pkg, tmp_path, parity_report, pipe, graph):
    world, steps = 2, 3
    res = _ranks(tmp_path, world, steps, pipe, graph)
    # ranks in lockstep: identical parameters, losses differ (their own samples)
    for r in res[1:]:
        assert np.array_equal(r["p32"], res[0]["p32"]), "DP ranks diverged"
        assert np.array_equal(r["norms"], res[0]["norms"]), "clip norms differ across ranks"
    # one engine on the global batch (2 x B samples), same schedule
    import torch
    B, L, H = 4, 32, 64
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    ref = pkg.engine.VQAEngine(sd, batch=world * B, seq_len=L, image_size=H, warmup=1, total=20, dropout=0.0)
    gloss, gnorm = [], []
    for i in range(steps):
        ref.load_batch(pkg.synthetic.make_batch(world * B, L, H, seed=40 + i))
        ref.train_step()
        torch.cuda.synchronize()
        gloss.append(float(ref.LOSS.item()))
        gnorm.append(ref.last_grad_norm())
    ref.flush_optimizer()
    p_ref = ref.P32.cpu().numpy()
    dloss = np.abs(np.mean([r["losses"] for r in res], axis=0) - gloss) / np.abs(gloss)
    dnorm = np.abs(res[0]["norms"] - gnorm) / np.array(gnorm)
    p0 = ref.lay.pack(sd)
    upd_err = float(np.linalg.norm(res[0]["p32"].astype(np.float64) - p_ref) /
                    np.linalg.norm(p_ref.astype(np.float64) - p0))
    parity_report[f"dp2_pipe{int(pipe)}"] = {"loss_rel": dloss.tolist(), "grad_norm_rel": dnorm.tolist(),
                                             "update_rel_l2": upd_err}
    # forward rows are batch-independent (same kernels per row); only the batch mean and the
    # gradient sums (two rank partials + an fp32 all-reduce vs one K = 2B*L sum) round differently
    # step 0 (same parameters on both sides): rounding only
    assert dloss[0] <= 1e-5 and dnorm[0] <= 1e-4, (dloss, dnorm)
    # later steps start from parameters whose AdamW updates differ where a gradient is ~0
    # (m / sqrt(v) amplifies its rounding): a loose bound on the trajectory
    assert (dloss <= 2e-3).all() and (dnorm <= 2e-2).all(), (dloss, dnorm)
    assert upd_err <= 5e-2, upd_err


@pytest.mark.parametrize("per,pipe", [((4, 1), False), ((4, 0), True), ((1, 3), True)])
def test_dp_unequal_rows_match_global_batch(gpu, pkg, tmp_path, parity_report, per, pipe):
    """Ranks holding unequal shares of the global batch (a contiguous split of a batch that does
    not divide evenly; (4, 0): rank 1 holds none).  The head divides by the all-reduced valid-row
    count over the world size (engine.use_global_rows, vqa_head_bwd ABI 18), so the summed,
    1/world-scaled gradients are the global batch's NLL mean (resnet_vqa_model.py:159), and each
    rank's loss is its share, whose mean over the ranks is the global loss.  Against one engine on
    the sum(per)-row global batch: ranks bitwise in lockstep, loss at step 0 within 1e-5."""
    world, steps = 2, 3
    res = _ranks(tmp_path, world, steps, pipe, True, mode="rows" + ".".join(map(str, per)))
    for r in res[1:]:
        assert np.array_equal(r["p32"], res[0]["p32"]), "DP ranks diverged"
        assert np.array_equal(r["norms"], res[0]["norms"]), "clip norms differ across ranks"
    if 0 in per:
        assert res[per.index(0)]["losses"].tolist() == [0.0] * steps, "an empty rank's loss share is 0"
    import torch
    B, L, H, n = 4, 32, 64, sum(per)
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    ref = pkg.engine.VQAEngine(sd, batch=world * B, seq_len=L, image_size=H, warmup=1, total=20, dropout=0.0)
    gloss, gnorm = [], []
    for i in range(steps):
        ref.load_batch(pkg.synthetic.make_batch(n, L, H, seed=40 + i))      # n < 2B rows: padded
        ref.train_step()
        torch.cuda.synchronize()
        gloss.append(float(ref.LOSS.item()))
        gnorm.append(ref.last_grad_norm())
    ref.flush_optimizer()
    p_ref = ref.P32.cpu().numpy()
    dloss = np.abs(np.mean([r["losses"] for r in res], axis=0) - gloss) / np.abs(gloss)
    dnorm = np.abs(res[0]["norms"] - gnorm) / np.array(gnorm)
    p0 = ref.lay.pack(sd)
    upd_err = float(np.linalg.norm(res[0]["p32"].astype(np.float64) - p_ref) /
                    np.linalg.norm(p_ref.astype(np.float64) - p0))
    parity_report["dp2_rows" + "_".join(map(str, per))] = {"loss_rel": dloss.tolist(), "grad_norm_rel": dnorm.tolist(),
                                                          "update_rel_l2": upd_err}
    assert dloss[0] <= 1e-5 and dnorm[0] <= 1e-4, (dloss, dnorm)
    assert (dloss <= 2e-3).all() and (dnorm <= 2e-2).all(), (dloss, dnorm)
    assert upd_err <= 5e-2, upd_err


@pytest.mark.parametrize("mode", ["trainer", "trainer_short"])
def test_trainer_data_parallel_two_ranks(gpu, pkg, tmp_path, parity_report, mode):
    """`VQATrainer` picks up the initialised process group (world 2) and drives
    dp.DataParallelStep: ranks stay bit-identical and train like one trainer on the
    global batch (the reference's train_one_step, faster_rcnn_vqa_trainer.py:391-406).
    trainer_short: the last step's batch is short (3 of the planned 4 rows per rank, as a
    DistributedSampler loader without drop_last gives every rank): each rank's padded rows
    are ignored, and the per-rank means averaged are the 6-row global mean."""
    sys.path.insert(0, HERE)
    import dp_worker
    world, steps = 2, 3
    res = _ranks(tmp_path, world, steps, False, True, mode=mode)
    assert all(bool(r["dp"]) for r in res), "the trainer did not switch to data parallel"
    for r in res[1:]:
        assert np.array_equal(r["p32"], res[0]["p32"]), "DP ranks diverged"
        assert np.array_equal(r["norms"], res[0]["norms"])
    B, L, H = 4, 32, 64
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    import torch
    rows = dp_worker.short_rows(B, steps) if mode == "trainer_short" else [B] * steps
    gb = [{k: torch.as_tensor(v).cuda() for k, v in pkg.synthetic.make_batch(world * rows[i], L, H, seed=40 + i).items()
           if v is not None} for i in range(steps)]
    ref = dp_worker.trainer_run(pkg, sd, world * B, L, H, gb, steps, True, data_parallel=False)
    dloss = np.abs(np.mean([r["losses"] for r in res], axis=0) - ref["losses"]) / np.abs(ref["losses"])
    dnorm = np.abs(res[0]["norms"] - ref["norms"]) / ref["norms"]
    p0 = pkg.layout.ParamLayout("resnet50").pack(sd)
    parity_report[f"dp2_{mode}"] = {"loss_rel": dloss.tolist(), "grad_norm_rel": dnorm.tolist()}
    assert dloss[0] <= 1e-5 and dnorm[0] <= 1e-4, (dloss, dnorm)
    assert (dloss <= 2e-3).all() and (dnorm <= 2e-2).all(), (dloss, dnorm)
    upd = float(np.linalg.norm(res[0]["p32"].astype(np.float64) - ref["p32"]) /
                np.linalg.norm(ref["p32"].astype(np.float64) - p0))
    parity_report[f"dp2_{mode}"]["update_rel_l2"] = upd
    assert upd <= 5e-2, upd


def test_dp_sharded_optimizer_matches_allreduce(gpu, tmp_path, parity_report):
    """DataParallelStep(shard_optimizer=True): reduce-scatter of the gradient buckets, AdamW on
    each rank's chunks only, all-gather of the fp32 masters and bf16 shadows.  The ranks stay
    bitwise in lockstep (parameters, shadows, gathered moments), and the result equals the
    all-reduce step's: the gradients are the same sums, only the clip norm's partial sums are
    grouped differently (fp64), so parameters agree to fp32 rounding."""
    world, steps = 2, 3
    ref = _ranks(tmp_path, world, steps, False, True)
    shd = _ranks(tmp_path, world, steps, False, True, mode="shard")
    for r in shd[1:]:
        for k in ("p32", "p16", "m", "vmax", "norms"):
            assert np.array_equal(r[k], shd[0][k]), f"sharded ranks diverged in {k}"
    assert np.array_equal(shd[0]["losses"], ref[0]["losses"]) or \
        np.abs(shd[0]["losses"] - ref[0]["losses"]).max() <= 1e-6 * np.abs(ref[0]["losses"]).max()
    dn = float(np.abs(shd[0]["norms"] - ref[0]["norms"]).max() / np.abs(ref[0]["norms"]).max())
    dp = float(np.abs(shd[0]["p32"].astype(np.float64) - ref[0]["p32"]).max() /
               np.abs(ref[0]["p32"]).max())
    dm = float(np.abs(shd[0]["m"].astype(np.float64) - ref[0]["m"]).max() / np.abs(ref[0]["m"]).max())
    parity_report["dp2_sharded_vs_allreduce"] = {"grad_norm_rel": dn, "p32_max_rel": dp, "exp_avg_max_rel": dm}
    assert dn <= 1e-6 and dp <= 1e-6 and dm <= 1e-5, (dn, dp, dm)


def test_dp_config5_two_ranks_match_global_batch(gpu, pkg, tmp_path, parity_report):
    """BASELINE configs[4]'s DP leg at its widths: two ranks of DataParallelStep on the T5-large +
    6 x SGA (width 1024) engine with e4m3 forward weight GEMMs and the DP weight-gradient groups
    (8, 8, 6, 2), pipelined and graphed, against one engine on the global batch.  The e4m3
    quantisation is row-wise (each activation row and weight row its own scale), so a rank's rows
    quantise exactly as they do inside the global batch; the gradient sums round differently."""
    world, steps = 2, 3
    res = _ranks(tmp_path, world, steps, True, True, mode="c5")
    for r in res[1:]:
        assert np.array_equal(r["p32"], res[0]["p32"]), "DP ranks diverged"
        assert np.array_equal(r["norms"], res[0]["norms"]), "clip norms differ across ranks"
    import torch
    B, L, H = 4, 32, 64
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=6, language_model="t5-large")
    ref = pkg.engine.VQAEngine(sd, batch=world * B, seq_len=L, image_size=H, warmup=1, total=20, dropout=0.0,
                               language_model="t5-large", num_blocks=6, fp8=True)
    gloss, gnorm = [], []
    for i in range(steps):
        ref.load_batch(pkg.synthetic.make_batch(world * B, L, H, seed=40 + i))
        ref.train_step()
        torch.cuda.synchronize()
        gloss.append(float(ref.LOSS.item()))
        gnorm.append(ref.last_grad_norm())
    ref.flush_optimizer()
    p_ref = ref.P32.cpu().numpy()
    dloss = np.abs(np.mean([r["losses"] for r in res], axis=0) - gloss) / np.abs(gloss)
    dnorm = np.abs(res[0]["norms"] - gnorm) / np.array(gnorm)
    p0 = ref.lay.pack(sd)
    upd_err = float(np.linalg.norm(res[0]["p32"].astype(np.float64) - p_ref) /
                    np.linalg.norm(p_ref.astype(np.float64) - p0))
    parity_report["dp2_config5"] = {"loss_rel": dloss.tolist(), "grad_norm_rel": dnorm.tolist(),
                                    "update_rel_l2": upd_err}
    assert dloss[0] <= 1e-5 and dnorm[0] <= 1e-4, (dloss, dnorm)
    assert (dloss <= 2e-3).all() and (dnorm <= 2e-2).all(), (dloss, dnorm)
    assert upd_err <= 5e-2, upd_err
