"""Worker of tests/test_a_dp2_gpu.py: one DP rank of `dp.DataParallelStep` on cuda:0 over
the gloo backend (several ranks share the one GPU of the test box; RCCL refuses two ranks
on one device).  Rank r trains on samples [r*B, (r+1)*B) of each global batch.

  python tests/dp_worker.py RANK WORLD PORT OUT.npz STEPS PIPELINE GRAPH [trainer|trainer_short|shard|c5]

`trainer`: drive the step through model.ResnetVQAModel + trainer.VQATrainer (data_parallel
picked up from the initialised process group) instead of the engine directly; `trainer_short`:
the same with a short last batch (3 rows per rank, padded to the planned 4); `shard`: the
engine step with the sharded optimizer (reduce-scatter, AdamW on the own chunks, all-gather);
`c5`: the engine step at BASELINE configs[4] widths (T5-large, 6 SGA blocks, fp8 forward GEMMs,
T5 weight-gradient groups (8, 8, 6, 2)); `c5full` / `c2full`: config 5 / config 2 at the benched shape
(B = 64 per rank, 384^2 / 224^2, 24 MB buckets, tools/dp_full_parity.py); `rows<R0>.<R1>...`: unequal rows per rank (rank r takes
the next R_r samples of each sum(R)-row global batch; R_r = 0: an empty rank), the engine planned
for B = 4 rows with the global-batch NLL mean (engine.use_global_rows)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, out, steps, pipe, graph = sys.argv[1:8]
    rank, world, steps = int(rank), int(world), int(steps)
    pipe, graph = pipe == "1", graph == "1"
    import numpy as np
    import torch
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mode = sys.argv[8] if len(sys.argv) > 8 else "engine"
    c5 = mode in ("c5", "c5full")
    full = mode in ("c2full", "c5full")
    # c2full / c5full: the benched config-2 / config-5 shape itself (B = 64 per rank, 224^2 / 384^2,
    # 24 MB buckets, the DP weight-gradient groups bench.py uses; tools/dp_full_parity.py)
    B, L, H = (64, 32, 384) if mode == "c5full" else (64, 32, 224) if mode == "c2full" else (4, 32, 64)
    # c5: BASELINE configs[4] widths -- T5-large (24 layers, d 1024), 6 SGA blocks at 1024, e4m3
    # forward weight GEMMs, the DP weight-gradient groups dp.dp_t5_dw_groups(24) = (8, 8, 6, 2)
    ekw = dict(language_model="t5-large", num_blocks=6, fp8=True) if c5 else {}
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, **({"num_attention_blocks": 6, "language_model": "t5-large"}
                                                              if c5 else {}))
    rows = short_rows(B, steps) if mode == "trainer_short" else [B] * (steps + 1)
    if mode.startswith("rows"):                         # unequal rows: rank r's slice of each global batch
        per = [int(x) for x in mode[4:].split(".")]
        assert len(per) == world
        lo, hi = sum(per[:rank]), sum(per[:rank + 1])
        gb = [pkg.synthetic.make_batch(sum(per), L, H, seed=40 + i) for i in range(steps + 1)]
        mine = [{k: (None if v is None else v[lo:hi]) for k, v in nb.items()} for nb in gb]
    else:
        gb = [pkg.synthetic.make_batch(world * rows[i], L, H, seed=40 + i) for i in range(steps + 1)]
        mine = [{k: (None if v is None else v[rank * rows[i]:(rank + 1) * rows[i]]) for k, v in nb.items()}
                for i, nb in enumerate(gb)]
    dev = [{k: torch.as_tensor(v).cuda() for k, v in nb.items() if v is not None} for nb in mine]
    if mode in ("trainer", "trainer_short"):
        tr = trainer_run(pkg, sd, B, L, H, dev, steps, graph)
        np.savez(out, **tr)
        dist.barrier()
        dist.destroy_process_group()
        return
    groups = pkg.dp.dp_t5_dw_groups(24) if c5 else pkg.dp.dp_t5_dw_groups(12) if full else (4, 4, 3, 1)
    eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, dropout=0.0,
                               seed=rank, pipeline=pipe, t5_dw_group=groups, device="cuda:0", **ekw)
    assert not c5 or (eng.t5_dw_groups == [8, 8, 6, 2] and eng.fp8)
    if mode.startswith("rows"):
        eng.use_global_rows(world)                      # before the first load: a rank may hold 0 rows
    if pipe:
        eng.prime(dev[0]["image_tensors"])
        eng.F4.copy_(eng.F4N)
        eng.load_batch(dev[0], next_images=dev[1]["image_tensors"])
    else:
        eng.load_batch(dev[0])
    shard = mode == "shard"
    step = pkg.dp.DataParallelStep(eng, bucket_mb=24 if full else 8, use_graph=graph,
                                   shard_optimizer=shard)
    if pipe:
        eng.prime(dev[0]["image_tensors"])
    losses, norms = [], []
    step.timing = graph                                 # bench.py's collective timing
    for i in range(steps):
        if pipe:
            eng.load_batch(dev[i], next_images=dev[i + 1]["image_tensors"])
        else:
            eng.load_batch(dev[i])
        step.step()
        torch.cuda.synchronize()
        losses.append(float(eng.LOSS.item()))
        norms.append(eng.last_grad_norm())
    eng.flush_optimizer()
    step.sync_optimizer_state()                         # sharded: every chunk's moments on every rank
    torch.cuda.synchronize()
    rep = step.timing_report()
    if graph:                                           # one completion per bucket + the row gather
        assert rep["steps"] == steps and len(rep["buckets"]) == len(step.buckets), rep
        assert all(b["done_us_after_stage"] >= 0.0 for b in rep["buckets"]), rep
        assert rep["exposed_wait_us_total"] >= 0.0, rep
    np.savez(out, losses=np.array(losses), norms=np.array(norms), p32=eng.P32.cpu().numpy(),
             g32=eng.G32.cpu().numpy(), m=eng.M.cpu().numpy(), vmax=eng.VMAX.cpu().numpy(),
             p16=eng.P16.float().cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def short_rows(B, steps):
    """trainer_short: per-rank rows of each step -- full batches, then a short last one (a
    DistributedSampler loader without drop_last: every rank's last batch has the same 3 rows)."""
    return [B] * (steps - 1) + [3, B]


TRAINER_KW = dict(optimizer_kwargs={"type": "AdamW", "lm_encoder_lr": 1e-4, "classifier_lr": 1e-4,
                                    "kwargs": {"weight_decay": 0.1, "amsgrad": True}},
                  lr_scheduler_kwargs={"num_warmup_steps": 1}, num_training_steps=20, gradient_clipping=1.0)


def trainer_run(pkg, sd, B, L, H, batches, steps, graph, **kw):
    """VQATrainer steps over `batches`; returns losses, clip norms and the final fp32 params."""
    import numpy as np
    import torch
    model = pkg.model.ResnetVQAModel("resnet50", "t5-base", 170, batch_size=B, seq_len=L, image_size=H,
                                     state_dict=sd, dropout=0.0, device="cuda:0")
    tr = pkg.trainer.VQATrainer(model, use_graph=graph, logger=None, bucket_mb=8, **TRAINER_KW, **kw)
    losses, norms = [], []
    for i in range(steps):
        loss, _ = tr.train_one_step(batches[i])
        losses.append(loss)
        norms.append(tr.grad_norm())
    model.engine.flush_optimizer()
    torch.cuda.synchronize()
    return dict(losses=np.array(losses), norms=np.array(norms), p32=model.engine.P32.cpu().numpy(),
                dp=np.array(tr.data_parallel))


if __name__ == "__main__":
    main()
