"""Data-parallel logic on CPU with the gloo backend, world_size 2 (the GPU path
uses the same functions over RCCL).  Covers: bucket planning over the flat
gradient arena, bucketed all-reduce == full all-reduce, the rank-major
(id, row) all-gather that replaces the dense embedding all-reduce, and the DP
semantics themselves (mean-NLL per rank + gradient average == global-batch
gradient) on the CPU oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from __graft_entry__ import load_package


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _spawn(fn, world, *args):
    port = _port()
    mp.spawn(fn, args=(world, port) + args, nprocs=world, join=True)


def test_plan_buckets_cover_prefix(pkg):
    lay = pkg.layout.ParamLayout("resnet50")
    emb = lay["t5.embed"].offset
    # marks as the engine emits them (DP: T5 weight gradients in groups): head, the SGA
    # blocks, scaler, final LN, T5 layers, relbias
    names = ["pool_b", "sga2.m1_b", "scaler_b", "t5.final_ln"] + \
        [f"t5.{i}.ln1" for i in reversed(range(12))] + ["t5.relbias"]
    marks = [(10 * (i + 1), lay[n].offset + (lay[n].numel + 63) // 64 * 64) for i, n in enumerate(names)]
    bks = pkg.dp.plan_buckets(marks, emb, 24 << 20)
    assert bks[0][1] == 0 and bks[-1][2] == emb
    for (c0, a0, b0), (c1, a1, b1) in zip(bks, bks[1:]):
        assert b0 == a1 and c0 < c1
    assert all(b - a >= (24 << 20) // 4 for _, a, b in bks[:-1])
    assert sum(b - a for _, a, b in bks) == emb


@pytest.mark.parametrize("world", [2, 3, 8])
def test_plan_shards_partition_the_prefix(pkg, world):
    """Sharded optimizer plan: per bucket, world equal 64-aligned owned chunks + a remainder
    shorter than world * 64; the owned chunks of all ranks and the remainders tile [0, emb)."""
    lay = pkg.layout.ParamLayout("resnet50")
    emb = lay["t5.embed"].offset
    names = ["pool_b", "sga2.m1_b", "scaler_b", "t5.final_ln"] + \
        [f"t5.{i}.ln1" for i in reversed(range(12))] + ["t5.relbias"]
    marks = [(10 * (i + 1), lay[n].offset + (lay[n].numel + 63) // 64 * 64) for i, n in enumerate(names)]
    bks = pkg.dp.plan_buckets(marks, emb, 24 << 20)
    shards = pkg.dp.plan_shards(bks, world)
    cover = np.zeros(emb, np.int32)
    for (_, a, b), (a2, c, b2) in zip(bks, shards):
        assert (a, b) == (a2, b2) and c % 64 == 0 and 0 <= b - a - world * c < world * 64
        for r in range(world):
            cover[a + r * c:a + (r + 1) * c] += 1
        cover[a + world * c:b] += 1
    assert (cover == 1).all()


def _allreduce_worker(rank, world, port, pkg_dir):
    _init(rank, world, port)
    from __graft_entry__ import load_package
    dp = load_package().dp
    g = torch.Generator().manual_seed(rank)
    flat = torch.randn(1000, generator=g)
    ref = flat.clone()
    dist.all_reduce(ref)
    bks = [(1, 0, 128), (2, 128, 640), (3, 640, 1000)]
    for w in dp.allreduce_buckets(flat, bks):
        w.wait()
    assert torch.equal(flat, ref)
    T, D = 6, 4
    ids = torch.tensor([5, 7, 5, 0, 0, 9]) + rank
    rows = torch.arange(T * D, dtype=torch.float32).reshape(T, D) + 100 * rank
    gi, gr = torch.zeros(world * T, dtype=torch.int64), torch.zeros(world * T, D)
    for w in dp.gather_rows(ids, rows, gi, gr):
        w.wait()
    for r in range(world):
        assert torch.equal(gi[r * T:(r + 1) * T], torch.tensor([5, 7, 5, 0, 0, 9]) + r)
        assert torch.equal(gr[r * T:(r + 1) * T], torch.arange(T * D, dtype=torch.float32).reshape(T, D) + 100 * r)
    # the step's opening id gather and the later row gather as separate collectives (r06)
    gi2, gr2 = torch.zeros(world * T, dtype=torch.int64), torch.zeros(world * T, D)
    for w in dp.gather_tensor(ids.reshape(2, 3), gi2) + dp.gather_tensor(rows, gr2):
        w.wait()
    assert torch.equal(gi2, gi) and torch.equal(gr2, gr)
    # gathered scatter == all-reduce of the per-rank dense scatters (what the reference computes)
    dense = torch.zeros(20, D).index_add_(0, ids, rows)
    dist.all_reduce(dense)
    assert torch.equal(torch.zeros(20, D).index_add_(0, gi, gr), dense)
    dist.destroy_process_group()


def test_allreduce_and_gather_gloo():
    _spawn(_allreduce_worker, 2, "")


def _semantics_worker(rank, world, port, tmp):
    _init(rank, world, port)
    from __graft_entry__ import load_package
    from oracle import vqa_oracle as orc
    torch.set_num_threads(2)
    pkg = load_package()
    B, L, H = 4, 16, 64
    sd = pkg.synthetic.make_state_dict("resnet34", seed=0)
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    half = {k: (None if v is None else v[rank * B // 2:(rank + 1) * B // 2]) for k, v in nb.items()}
    tr = orc.OracleTrainer(sd, "resnet34")
    tr.forward_backward(orc.to_torch_batch(half))
    grads = torch.cat([tr.sd[k].grad.reshape(-1) for k in tr.keys])
    dist.all_reduce(grads)
    grads /= world
    if rank == 0:
        np.save(os.path.join(tmp, "dp_grads.npy"), grads.numpy())
    dist.destroy_process_group()


@pytest.mark.slow
def test_dp_gradient_average_equals_global_batch(tmp_path):
    """Mean-NLL per rank + all-reduce average == the reference's single-device
    gradient of the global batch (faster_rcnn_vqa_trainer.py:391-406)."""
    from oracle import vqa_oracle as orc
    _spawn(_semantics_worker, 2, str(tmp_path))
    pkg = load_package()
    B, L, H = 4, 16, 64
    sd = pkg.synthetic.make_state_dict("resnet34", seed=0)
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    tr = orc.OracleTrainer(sd, "resnet34")
    tr.forward_backward(orc.to_torch_batch(nb))
    ref = torch.cat([tr.sd[k].grad.reshape(-1) for k in tr.keys]).numpy()
    got = np.load(tmp_path / "dp_grads.npy")
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < 1e-5, err


class _C:
    def __init__(self, seg, i, side):
        self.seg, self.i, self.side = seg, i, side


@pytest.mark.parametrize("dw_stream", [True, False])
def test_plan_stages_keep_order_and_finality(pkg, dw_stream):
    """dp.plan_stages: every backward call lands in exactly one stage; the chain calls keep
    their order; a segment's weight-gradient calls are forked only after that segment's chain
    calls (and after everything forked before them); every bucket becomes final exactly once, in
    a stage at or after the one running its last call; no stage ends without a final bucket."""
    rng = np.random.default_rng(0)
    sizes = [40, 9, 33, 26, 14, 6]                     # head+SGA, scaler dW, T5 groups, last layer
    segs = []
    for k, n in enumerate(sizes):
        segs.append([_C(k, i, (k == 1) or bool(rng.random() < 0.3)) for i in range(n)])
    scaler = (sizes[0], sizes[0] + sizes[1])
    stages, rows = pkg.dp.plan_stages(segs, scaler, dw_stream)
    seq = [(j, kd, c) for j, st in enumerate(stages) for kd, cs in st["ops"] for c in cs]
    allc = [c for s in segs for c in s]
    assert sorted(id(c) for _, _, c in seq) == sorted(id(c) for c in allc)
    mains = [c for _, kd, c in seq if kd == "main"]
    ref = [c for s in segs for c in s if not (c.seg == 1 or (dw_stream and c.side))]
    assert [id(c) for c in mains] == [id(c) for c in ref]
    pos = {id(c): p for p, (_, _, c) in enumerate(seq)}
    last_main = {}
    for c in mains:
        last_main[c.seg] = pos[id(c)]
    forks = [c for _, kd, c in seq if kd == "fork"]
    assert [(c.seg, c.i) for c in forks] == sorted((c.seg, c.i) for c in forks)
    for c in forks:
        assert pos[id(c)] > last_main.get(c.seg, -1)
    final_at = {k: j for j, st in enumerate(stages) for k in st["final"]}
    assert sorted(final_at) == list(range(len(segs)))
    assert sum(len(st["final"]) for st in stages) == len(segs)
    for c in allc:
        assert final_at[c.seg] >= next(j for j, _, x in seq if x is c)
    assert all(st["final"] for st in stages)
    assert len(stages) < len(segs) and rows == max(j for j, kd, _ in seq if kd == "main")
