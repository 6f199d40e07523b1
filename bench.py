"""Benchmark: question-image pairs/s of the ResNet50 + T5-base + 3xSGA training
step (fwd + bwd + [RCCL all-reduce] + clip + AdamW(amsgrad) + schedule) on
MI355X, bf16 MFMA / fp32 masters, B=64 per GPU, 224x224 images, 32-token
questions (BASELINE.json configs[1]; configs[2] when launched on 8 GPUs).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N ... bench.py --gpus N     (one process per GPU)

Synthetic data (no datasets offline): a pool of 4 batches per rank is made
resident in HBM before timing; each timed step copies one into the static input
buffers (device to device) and replays the captured step graph.
Prints ONE JSON line on rank 0.

`--gpus N` with N > 1 and no torchrun environment: this process starts N ranks
itself (one child process per GPU, before anything touches the GPU), waits for
them, and exits with the worst return code; rank 0 prints the line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

FLOP_PER_PAIR = 30.95e9        # fwd+bwd algorithmic FLOPs, R50 @224, L=32
MFMA_PEAK_TFLOPS = 2517.0      # bf16 dense: 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md)
FP8_PEAK_TFLOPS = 5034.0       # e4m3 dense, block-scaled MFMA (2x the bf16 rate per clock, MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
PMC_FILE = "r06_pmc.json"               # rocprofv3 PMC summary this bench quotes (tools/pmc_step.py)
PMC_FILE_C5 = "r06_pmc_c5.json"         # the same passes over the config-5 step (bench.py --config5)
DIGEST_SUFFIXES = (".py", ".hip", ".h", ".inl", ".json", "Makefile")


def tree_digest():
    """sha256 over the sources that decide which kernels one step launches and what they
    touch: the package (kernels, host code, tile table), bench.py and __graft_entry__.py.
    tools/pmc_step.py stamps it into the PMC summary; main() quotes the summary's counters
    only when the stamp equals this tree's digest (a PMC file from another tree is ignored)."""
    import hashlib
    h = hashlib.sha256()
    files = [os.path.join(ROOT, f) for f in ("bench.py", "__graft_entry__.py")]
    for d, dirs, fs in os.walk(os.path.join(ROOT, "t5-resnet-vqa_amd")):
        dirs[:] = sorted(x for x in dirs if x != "__pycache__" and not x.startswith("_build"))
        files += [os.path.join(d, f) for f in sorted(fs) if f.endswith(DIGEST_SUFFIXES)]
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def cpu_baseline(pkg, batch=64, steps=5, warm=2):
    """The CPU oracle (fp32 restatement of the reference step) on this host's cores, at the
    config-2 shapes (B=64, 224x224, L=32), median of 5 steps after 2 warm-up steps
    (SURVEY.md §8d / BASELINE.md)."""
    from oracle import vqa_oracle as orc
    threads = torch.get_num_threads()
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    tr = orc.OracleTrainer(sd, "resnet50", warmup=10, total=1000, dropout=0.1)
    nb = orc.to_torch_batch(pkg.synthetic.make_batch(batch, 32, 224, seed=1))
    times = []
    for i in range(warm + steps):
        t0 = time.perf_counter()
        tr.train_one_step(nb)
        if i >= warm:
            times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": round(batch / t, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"oracle fp32 train step (zero_grad+fwd+bwd+clip+AdamW amsgrad, dropout 0.1), R50+T5-base+3xSGA, "
                      f"B={batch}, 224x224, L=32, median of {steps} steps after {warm} warm-up "
                      f"({t:.2f} s/step), torch CPU {threads} threads"}


def calls_flop(eng, fp8_only=False):
    """MFMA work of one step from the engine's prepared calls (GEMMs / implicit-GEMM convs:
    2 m n k per batch item; attention: 4 lq lk dh forward, 8 backward, per (sample, head)).
    fp8_only: the e4m3 GEMMs' share."""
    tot = 0.0
    res = list(eng.res_calls) if eng.pipeline else []           # else they are in fwd_calls
    for c in res + eng.fwd_calls + eng.bwd_calls:
        if fp8_only and not (c.name == "vqa_gemm" and c.desc.fp8):
            continue
        if c.name == "vqa_gemm":
            d = c.desc
            tot += 2.0 * d.m * d.n * d.k * max(1, d.batch)
        elif c.name == "vqa_gemm_pair":
            tot += sum(2.0 * d.m * d.n * d.k for d in c.desc)
        elif c.name in ("vqa_attn_fwd", "vqa_attn_bwd"):
            d = c.desc
            tot += (4.0 if c.name == "vqa_attn_fwd" else 8.0) * d.batch * d.heads * d.lq * d.lk * d.dh
    return tot


def _flat_calls(calls):
    for c in calls:
        if hasattr(c, "calls"):                                    # engine._Seq (AdamW range + e4m3 copies)
            yield from _flat_calls(c.calls)
        else:
            yield c


def step_calls(eng):
    """Every prepared call one benched step launches: the next batch's frozen ResNet (pipelined),
    the F4 copy, the deferred AdamW ranges, forward, backward and the optimizer plan."""
    seq = []
    if eng.pipeline:
        seq += [eng.copy_f4] + list(eng.res_calls)
    if eng.defer_opt:
        seq += [c for _, c in eng.adam_segs] + [eng.clear_pending]
    seq += list(eng.fwd_calls) + list(eng.bwd_calls)
    if getattr(eng, "embed_split", False):                 # the stream step's embedding rows split
        seq += list(eng.emb_pre) + list(eng.opt_calls[:2]) + list(eng.tail_calls)
    else:
        seq += list(eng.opt_calls)
    return list(_flat_calls(seq))


ALG_TOUCHED_ROWS = 64 * 32     # embedding rows a step touches at most (B x L; main() sets it per config)


def call_bytes(c):
    """ALGORITHMIC HBM bytes of one prepared call: every operand read once and every result
    written once, at the precision the kernel stores it (SURVEY §8d's per-op byte model).
      GEMM: A (or, implicit im2col, the input activation itself) + B + C (fp32 and / or bf16, read
        too when beta != 0) + bias + residual + mask, per batch item where the stride is nonzero;
      attention: q, k, v (+ o, P) forward; q, k, v, P, dO, dq, dk, dv (+ dbias) backward, per
        (sample, head, group) + the shared bias / key mask;
      AdamW-amsgrad: 38 B per parameter (read p g m v vmax, write p m v vmax + bf16 shadow);
      embedding gather / scatter / row re-zeroing: the touched rows only (not the 98.7 MB table);
      grad sq-norm: the gradient range once;
      everything else (norms, column sums, copies, the image / pooling kernels, the head): the
        tensors the call is declared to read and write (its `keep`), each once."""
    n = c.name
    d = c.desc
    if n in ("vqa_gemm", "vqa_gemm_pair"):
        return sum(_gemm_bytes(x) for x in (d if isinstance(d, (tuple, list)) else (d,)))
    if n in ("vqa_attn_fwd", "vqa_attn_bwd"):
        g = max(1, d.groups)
        per = (d.lq + 2 * d.lk) * d.dh * 2                          # q, k, v (bf16)
        if n == "vqa_attn_fwd":
            per += d.lq * d.dh * 2 + (d.lq * d.lk * 4 if d.p else 0)  # o (+ saved P)
        else:
            per += d.lq * d.lk * 4 + d.lq * d.dh * 2 + (d.lq + 2 * d.lk) * d.dh * 2 + (d.lq * d.lk * 4 if d.dbias else 0)
        shared = (d.heads * d.lq * d.lk * 4 if d.bias else 0) + (d.batch * d.lk * 8 if d.key_mask else 0)
        return float(g * (d.batch * d.heads * per + shared))
    if n == "vqa_adamw_amsgrad":
        return 38.0 * d.n
    if n == "vqa_grad_sqnorm":
        return 4.0 * c.args[1]
    if n == "vqa_embed_mark":                                       # ids, tokens, rows, mark, state
        return float(c.args[1] * 8 + c.args[1] * 4)
    if n == "vqa_adamw_rows":                                       # desc, mark, rows, cols, touched, ...
        rows, cols, touched = c.args[2], c.args[3], c.args[4]
        t = min(rows, ALG_TOUCHED_ROWS)                             # the step's tokens bound the touched rows
        # touched == 1: the marked rows after finalize, 38 B each; 0 or > 1 (the grid size of the pass
        # beside the backward): the untouched rows, p m v vmax read + written and the bf16 shadow
        # written, no gradient read
        return float(rows * 4 + (t * cols * 38.0 if touched == 1 else (rows - t) * cols * 34.0))
    if n == "vqa_embedding_fwd":                                    # ids, table, out, tokens, d, ...
        t, dd = c.args[3], c.args[4]
        return float(t * 8 + 2 * t * dd * 4)
    if n == "vqa_embedding_bwd":                                    # ids, dh, dtable, tokens, d, ...
        t, dd = c.args[3], c.args[4]
        return float(t * 8 + 2 * t * dd * 4)
    if n == "vqa_embedding_zero_rows":                              # prev, cur, tokens, dtable, d, ...
        t, dd = c.args[2], c.args[4]
        return float(2 * t * 8 + t * dd * 4)
    # calls whose `keep` holds whole arenas or the ResNet's max-size ping-pong buffers: the bytes
    # they actually touch, from their arguments
    if n == "vqa_quant_rows_fp8":                                   # x, x_bf16, ldx, rows, cols, q, ldq, scale
        rows, cols = c.args[3], c.args[4]
        return float(rows * cols * (2 if c.args[1] else 4) + rows * cols + rows * 4)
    if n in ("vqa_stem_pool_s2d", "vqa_stem_s2d_conv"):             # z, w, bias, y, n, hz, oh
        nb, hz, oh = c.args[4], c.args[5], c.args[6]
        oy = oh // 2 if n == "vqa_stem_pool_s2d" else oh
        return float(nb * hz * hz * 16 * 2 + 64 * 256 * 2 + 64 * 4 + nb * oy * oy * 64 * 2)
    if n == "vqa_stem_pool_img":                                    # img, w, bias, y, n, h
        nb, h = c.args[4], c.args[5]
        return float(nb * 3 * h * h * 4 + 64 * 256 * 2 + 64 * 4 + nb * (h // 4) * (h // 4) * 64 * 2)
    if n == "vqa_subsample_nhwc":                                   # x, n, h, w, c, stride, y, ldy
        nb, h, w, ch, s = c.args[1:6]
        return float(2 * nb * ((h - 1) // s + 1) * ((w - 1) // s + 1) * ch * 2)
    if n == "vqa_maxpool3x3s2_nhwc":                                # x, y, n, h, w, c, oh, ow
        nb, h, w, ch, oh, ow = c.args[2:8]
        return float(nb * h * w * ch * 2 + nb * oh * ow * ch * 2)
    seen, tot = set(), 0
    for t in (c.keep or ()):
        if isinstance(t, torch.Tensor):
            key = (t.data_ptr(), t.numel(), t.element_size())
            if key not in seen:
                seen.add(key)
                tot += t.numel() * t.element_size()
    return float(tot)


def _gemm_bytes(d):
    e = 1 if d.fp8 else 2
    b = max(1, d.batch)
    m, n, k = d.m, d.n, d.k
    if d.a_conv:
        ga = d.ga
        a = ga.n * ga.h * ga.w * ga.c * 2
    else:
        a = m * k * e * (b if d.stride_a else 1)
    if d.b_conv:
        gb = d.gb
        bb = gb.n * gb.h * gb.w * gb.c * 2
    else:
        bb = n * k * e * (b if d.stride_b else 1)
    out = m * n * b * ((4 * (2 if d.beta else 1) if d.c32 else 0) + (2 if d.c16 else 0))
    extra = (n * 4 * (b if d.stride_bias else 1) if d.bias else 0)
    rb = b if d.stride_res else 1
    extra += m * n * rb * ((4 if d.res32 else 0) + (2 if d.res16 else 0) + (2 if d.mask16 else 0))
    return float(a + bb + out + extra)


def vit_flop_per_pair(lq, ld, nv=197, d=768, dff=3072, vff=3072, layers=12):
    """Algorithmic FLOPs of one config-4 pair (VitVQAModel, vit_vqa_model.py:166-225): the frozen
    ViT forward, the T5 encoder and decoder forward + backward (x3: the input and weight
    gradients), the fusing layer and classifier (2 FLOP per multiply-add)."""
    vit = 2 * (nv - 1) * d * d + layers * (2 * nv * d * 3 * d + 4 * nv * nv * d + 2 * nv * d * d
                                           + 4 * nv * d * vff) + 2 * d * d
    enc = layers * (2 * lq * d * 3 * d + 4 * lq * lq * d + 2 * lq * d * d + 4 * lq * d * dff)
    dec = layers * (2 * ld * d * 3 * d + 4 * ld * ld * d + 2 * ld * d * d + 2 * d * d + 2 * ld * d * d
                    + 4 * ld * d * dff)
    head = 2 * 2 * d * d + 2 * d * 170
    return float(vit + 3 * (enc + dec + head))


def bench_vit(args, pkg, dev):
    """BASELINE configs[3]: ViT-base + T5-base encoder-decoder (VitVQAModel) train step, 1 GPU."""
    B, L, Ld = args.batch, args.seq_len, 20
    vm = pkg.vit_model
    eng = pkg.vit_engine.VitVQAEngine(vm.make_state_dict(seed=0), batch=B, seq_len=L, dec_len=Ld, device=dev,
                                      warmup=10, total=100000, dropout=0.1)
    pool = [{k: (None if v is None else torch.as_tensor(v).to(dev)) for k, v in
             vm.make_batch(B, L, dec_len=Ld, seed=1 + i).items()} for i in range(4)]
    eng.load_batch(pool[0])
    eng.forward()
    eng.backward()
    eng.autotune(table=args.tune_table, save=args.tune_save)
    if not args.no_graph:
        eng.capture()

    def step(i):
        eng.load_batch(pool[i % len(pool)])
        eng.train_step()
    for i in range(args.warmup):
        step(i)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    t_issue = time.perf_counter() - t0             # host time to issue the K steps (< dt: the host ran ahead)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gpu_step = ev0.elapsed_time(ev1) * 1e-3 / args.steps
    fpp = vit_flop_per_pair(L, Ld)
    tf = fpp * B / gpu_step / 1e12
    out = {"metric": "question-image pairs/sec, ViT-base+T5-base encoder-decoder train step (BASELINE configs[3])",
           "value": round(B * args.steps / dt, 2), "unit": "pairs/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
           "config": {"workload": "VitVQAModel train step (vit_vqa_model.py:127-227), BASELINE configs[3]",
                      "model": "vit-base-patch16-224 (frozen) + t5-base encoder-decoder", "global_batch": B,
                      "seq_len": L, "dec_len": Ld, "image_size": 224, "answers": 170, "parallelism": "dp1",
                      "graph": not args.no_graph},
           "roofline": {"bound": "mfma", "kernel": "whole train step (one hipGraph replay)",
                        "achieved": round(tf, 1), "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / MFMA_PEAK_TFLOPS, 4), "traffic": None,
                        "flop_per_step": fpp * B, "step_gpu_ms": round(gpu_step * 1e3, 4)},
           "loss": round(float(eng.LOSS.item()), 5), "grad_norm": round(eng.last_grad_norm(), 4)}
    if not args.no_cpu_baseline:
        from oracle import vit_oracle as orc
        cb, steps, warm = 16, 3, 1
        tr = orc.VitOracleTrainer(vm.make_state_dict(seed=0), warmup=10, total=1000, dropout=0.1)
        nb = {k: (None if v is None else torch.as_tensor(v)) for k, v in vm.make_batch(cb, L, dec_len=Ld).items()}
        times = []
        for i in range(warm + steps):
            t1 = time.perf_counter()
            tr.train_one_step(nb)
            if i >= warm:
                times.append(time.perf_counter() - t1)
        t = float(np.median(times))
        out["cpu_baseline"] = {"value": round(cb / t, 3), "unit": "pairs/s", "cores": torch.get_num_threads(),
                               "kind": "port", "sample": f"config-4 oracle fp32 train step, B={cb}, L={L}, Ld={Ld}, "
                                                         f"224x224, median of {steps} after {warm} ({t:.2f} s/step)"}
    emit(out)


_OUT = None


def emit(out):
    """The bench's one JSON line, on the process's original stdout."""
    f = _OUT or sys.stdout
    f.write(json.dumps(out) + "\n")
    f.flush()


def spawn_ranks(n):
    """Start n ranks of this script (one per GPU) with a torchrun-style environment;
    called before any GPU call, so no process here ever initialises the GPU."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def time_kernel(call, reps, stream):
    """Average duration of one prepared launch, HIP events on the launch stream."""
    from vqa_amd import lib as L  # noqa
    h = L.stream_handle(stream)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        call(h)
    start.record(stream)
    for _ in range(reps):
        call(h)
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / reps * 1e-3


def make_step(args, pkg, dev, pool, use_dp, rank, lm):
    """The engine at the bench shapes, tuned and captured: the single-GPU graph step, or for
    `use_dp` the N > 1 code path (dp.DataParallelStep with the DP engine's weight-gradient
    groups).  Returns (engine, DataParallelStep or None, step(i) loading pool batch i)."""
    B, L, H, NB = args.batch, args.seq_len, args.image_size, args.blocks
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=NB,
                                       language_model=lm)      # identical init on every rank
    pipe = not args.no_pipeline
    dp_groups = pkg.dp.dp_t5_dw_groups(pkg.synthetic.lm_dims(lm).t5_layers)
    eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=L, image_size=H, device=dev, num_blocks=NB,
                               warmup=10, total=100000, dropout=0.1, seed=rank, pipeline=pipe,
                               t5_dw_group=dp_groups if (use_dp or args.dp_groups) else None, language_model=lm,
                               fp8=args.config5)
    del sd
    torch.cuda.synchronize()
    if pipe:
        # the frozen ResNet of batch k+1 runs beside step k (engine docstring): prime batch 0's features
        eng.prime(pool[0]["image_tensors"])
        eng.F4.copy_(eng.F4N)
        eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
    else:
        eng.load_batch(pool[0])
    eng.forward()
    eng.backward()
    eng.autotune(table=args.tune_table, save=args.tune_save if rank == 0 else None)   # tile choice: speed only
    dps = None
    if use_dp:
        dps = pkg.dp.DataParallelStep(eng, use_graph=not args.no_graph, shard_optimizer=args.shard_optimizer,
                                      **({} if args.dp_res_split is None else {"res_split": args.dp_res_split}))
        run_step = dps.step
    else:
        eng.res_order = getattr(args, "res_order", "first")
        eng.res_head = getattr(args, "res_head", 4)
        if args.res_cumask:
            eng.set_res_cumask(cumask_words(args.res_cumask, torch.cuda.get_device_properties(dev).multi_processor_count))
        if not args.no_graph:
            eng.capture()
        run_step = eng.train_step
    if pipe:                                       # the tuning passes above consumed nothing: restart at batch 0
        eng.prime(pool[0]["image_tensors"])
    k = [0]

    def step(_):
        i = k[0]
        k[0] += 1
        if pipe:
            eng.load_batch(pool[i % len(pool)], next_images=pool[(i + 1) % len(pool)]["image_tensors"])
        else:
            eng.load_batch(pool[i % len(pool)])
        run_step()
    return eng, dps, step


def cumask_words(spec, ncu):
    """--res-cumask SPEC -> CU mask words: 'lo:N' CUs 0..N-1, 'hi:N' the last N, 'st:K:R' the CUs
    i with i % K < R, 'all'."""
    kind, *v = spec.split(":")
    v = [int(x) for x in v]
    sel = {"all": lambda i: True, "lo": lambda i: i < v[0], "hi": lambda i: i >= ncu - v[0],
           "st": lambda i: i % v[0] < v[1]}[kind]
    words = [0] * ((ncu + 31) // 32)
    for i in range(ncu):
        if sel(i):
            words[i // 32] |= 1 << (i % 32)
    return words


def time_steps(args, step, dev, dist):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize on both sides;
    returns (wall seconds, GPU seconds per step from HIP events on the replay stream, host issue
    seconds), each the max over ranks."""
    for i in range(args.warmup):
        step(i)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    t_issue = time.perf_counter() - t0             # host time to issue the K steps (< dt: the host ran ahead)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gpu_step = ev0.elapsed_time(ev1) * 1e-3 / args.steps       # HIP events on the replay stream
    if dist:
        t = torch.tensor([dt, gpu_step], device="cpu" if args.rehearse else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, gpu_step = float(t[0].item()), float(t[1].item())
    return dt, gpu_step, t_issue


def init_world1(dev):
    """A world-1 RCCL group of this process (the N > 1 code path on one GPU)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    return dist


def dp_world1_line(args, pkg, dev, pool, lm, engine_dt):
    """The N > 1 code path at N = 1: the same workload through
    dp.DataParallelStep over a world-1 RCCL group -- forward graph, backward stage graphs with
    the bucketed all-reduce between them, finish graph -- timed exactly as the headline step,
    so SCALE's N = 1 point (the engine graph) can be read against the path N > 1 runs."""
    dist = init_world1(dev)
    try:
        eng, dps, step = make_step(args, pkg, dev, pool, True, 0, lm)
        dt, gpu_step, _ = time_steps(args, step, dev, dist)
        res = {"value": round(args.batch * args.steps / dt, 2), "unit": "pairs/s",
               "ms_per_step": round(dt / args.steps * 1e3, 3), "step_gpu_ms": round(gpu_step * 1e3, 4),
               "over_engine_step": round(dt / engine_dt, 4),
               "path": f"dp.DataParallelStep over a world-1 {dist.get_backend()} group: forward graph, "
                       f"{len(dps.stages)} backward stage graphs with the bucketed all-reduce between them, "
                       "finish graph (the code path bench.py runs for N > 1)",
               "loss": round(float(eng.LOSS.item()), 5)}
        del eng, dps, step
    finally:
        dist.destroy_process_group()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq-len", type=int, default=32)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--blocks", type=int, default=3, help="SGA blocks (3: the reference default; 6: BASELINE config 5)")
    ap.add_argument("--config5", action="store_true",
                    help="BASELINE configs[4]: ResNet50 + T5-large + 6xSGA at width 1024, 384x384 images, fp8 (e4m3) "
                         "forward weight GEMMs (per GPU; DP over N GPUs as for config 2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-kernel-rooflines", action="store_true", help="skip the per-kernel replays after the timed region")
    ap.add_argument("--shard-optimizer", action="store_true",
                    help="N > 1: reduce-scatter + sharded AdamW + all-gather instead of the bucketed all-reduce")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run the frozen ResNet inside each step instead of beside the previous one")
    ap.add_argument("--tune-table", default=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"),
                    help="measured GEMM tile choices (missing shapes are timed at start-up)")
    ap.add_argument("--tune-save", default=None, help="write the tile choices used to this file")
    ap.add_argument("--model", choices=("resnet", "vit"), default="resnet",
                    help="vit: BASELINE configs[3], ViT-base + T5 encoder-decoder (1 GPU)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4; set before the runtime starts)")
    ap.add_argument("--dp", action="store_true",
                    help="N = 1: run the N > 1 step (dp.DataParallelStep over a world-1 RCCL group, the DP engine's "
                         "weight-gradient groups) instead of the single-GPU engine graph")
    ap.add_argument("--dp-res-split", type=float, default=None,
                    help="DP, pipelined: share of the next batch's ResNet calls beside the forward graph (dp.RES_SPLIT)")
    ap.add_argument("--dp-groups", action="store_true",
                    help="the single-GPU engine step with the DP engine's T5 weight-gradient groups (A/B of --dp)")
    ap.add_argument("--res-cumask", default=None,
                    help="experiment: the next batch's ResNet on a CU-masked stream beside the chain graph "
                         "(lo:N | hi:N | st:K:R | all; bench.cumask_words)")
    ap.add_argument("--res-order", choices=("first", "last", "root", "interleave"), default="first",
                    help="experiment: capture the next batch's ResNet branch before (default) or after the chain; "
                         "root: F4 <- F4N issued before the replay, both branches graph roots")
    ap.add_argument("--res-head", type=int, default=4,
                    help="--res-order interleave: ResNet calls issued before the T5 encoder's first layer")
    ap.add_argument("--main-stream", choices=("default", "side"), default="default",
                    help="experiment: issue the step on torch's default stream or on a stream of its own")
    ap.add_argument("--no-dp-line", action="store_true",
                    help="N = 1: skip the second timing of the same workload through the N > 1 code path "
                         "(dp.DataParallelStep over a world-1 RCCL group; JSON key dp_world1)")
    ap.add_argument("--rehearse", action="store_true",
                    help="run every rank on cuda:0 over gloo: exercises the N-rank code path (bucketing, "
                         "gathers, capture, lockstep) on a one-GPU box; the timing is not a measurement")
    args = ap.parse_args()

    if args.hw_queues:                             # before anything starts the HIP runtime
        assert 1 <= args.hw_queues <= 16, args.hw_queues
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))          # one process per GPU, started before any GPU call

    # the one JSON line goes to the original stdout; anything native libraries print there (the
    # RCCL version banner at communicator creation) is sent to stderr instead
    global _OUT
    _OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse:
        local = 0                                          # every rank shares the one GPU (gloo, host-staged)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.main_stream == "side":
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    if args.model == "vit":
        if world != 1:
            raise SystemExit("bench --model vit: BASELINE configs[3] is a 1-GPU configuration")
        bench_vit(args, load_package(), dev)
        return
    dist = None
    use_dp = world > 1 or args.dp
    if use_dp:
        import torch.distributed as dist
        if world == 1:                                   # --dp: a world-1 RCCL group of this process
            init_world1(dev)
        elif args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    pkg = load_package()
    if args.config5:
        args.image_size, args.blocks = 384, 6
    lm = "t5-large" if args.config5 else "t5-base"
    B, L, H = args.batch, args.seq_len, args.image_size
    NB = args.blocks
    pipe = not args.no_pipeline
    pool = []
    for i in range(4):
        nb = pkg.synthetic.make_batch(B, L, H, seed=1 + rank * 16 + i)
        pool.append({k: torch.as_tensor(v).to(dev) for k, v in nb.items() if v is not None})
    eng, dps, step = make_step(args, pkg, dev, pool, use_dp, rank, lm)
    dt, gpu_step, t_issue = time_steps(args, step, dev, dist)
    loss = float(eng.LOSS.item())
    gnorm = eng.last_grad_norm()
    pairs = world * B * args.steps
    value = pairs / dt
    survey_cfg = (args.image_size, args.seq_len, NB) == (224, 32, 3) and not args.config5
    c5_cfg = args.config5 and (B, args.seq_len, args.image_size, NB) == (64, 32, 384, 6)
    pfile = PMC_FILE if survey_cfg else PMC_FILE_C5
    pmc, pmc_note = {}, f"profiles/{pfile} absent"
    pmc_path = os.path.join(ROOT, "profiles", pfile)
    if not (survey_cfg or c5_cfg):
        pmc_note = (f"profiles/{PMC_FILE} / {PMC_FILE_C5} cover the config-2 and config-5 steps only "
                    "(B=64, L=32; 224x224 / 3 blocks, 384x384 / 6 blocks)")
    elif os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        if args.no_pipeline or args.no_graph:
            pmc, pmc_note = {}, f"profiles/{pfile} was measured on the pipelined graph step: not quoted"
        elif use_dp or args.dp_groups:                     # other stage graphs / T5 weight-gradient groups
            pmc, pmc_note = {}, (f"profiles/{pfile} was measured on the single-GPU engine step, not on the "
                                 "DataParallelStep schedule: not quoted")
        elif pmc.get("tree_digest") != tree_digest():      # counters of another tree: not quoted
            pmc, pmc_note = {}, f"profiles/{pfile} was measured on another tree (digest mismatch): not quoted"
        else:
            pmc_note = (f"profiles/{pfile} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, all dispatches of one step; "
                        f"measured on this tree, commit {pmc.get('commit')})")

    # Headline roofline (the step is > 97 % GEMM FLOPs, so it is MFMA-bound): the whole
    # captured train step as one unit of work.  Algorithmic work per step = 30.95 GFLOP per
    # pair x B pairs; duration = the step's GPU time from HIP events on
    # the replay stream over the timed region; traffic = HBM bytes per step from the
    # committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes over every dispatch of one step.
    # Other shapes (--image-size / --seq-len): the MFMA work of the prepared calls.
    step_flop = FLOP_PER_PAIR * B if survey_cfg else calls_flop(eng)
    step_tflops = step_flop / gpu_step / 1e12
    st = pmc.get("step", {})
    global ALG_TOUCHED_ROWS
    ALG_TOUCHED_ROWS = eng.T                                     # tokens per step bound the touched rows
    alg = sum(call_bytes(c) for c in step_calls(eng))            # algorithmic HBM bytes of one step
    # config 5 mixes e4m3 (forward weight GEMMs) and bf16 MFMA work: the peak is the rate at which
    # the step's FLOP mix would run with every launch at its dtype's dense peak
    f8 = calls_flop(eng, fp8_only=True)
    peak = MFMA_PEAK_TFLOPS if f8 == 0 else calls_flop(eng) / (f8 / FP8_PEAK_TFLOPS + (calls_flop(eng) - f8) /
                                                               MFMA_PEAK_TFLOPS)
    if use_dp:
        replay = (f"DataParallelStep: forward graph, {len(dps.stages)} backward stage graphs with the "
                  f"{dist.get_backend()} exchange between them, finish graph")
        if args.no_graph:
            replay = f"DataParallelStep, eager: forward, {len(dps.stages)} backward stages, exchange, finish"
    else:
        replay = "eager stream launches (--no-graph)" if args.no_graph else "one hipGraph replay"
    roofline = {"bound": "mfma", "kernel": f"whole train step ({replay}: ResNet50 fwd, ConvT, {lm}, {NB}xSGA, "
                                           "head, backward, clip, AdamW)",
                "achieved": round(step_tflops, 1), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(step_tflops / peak, 4),
                **({"fp8_flop_per_step": f8, "peak_note": "e4m3 FLOPs at 5034, bf16 FLOPs at 2517 TFLOP/s"} if f8 else {}),
                "traffic": round(st["traffic_bytes"]) if "traffic_bytes" in st else None,
                "alg_bytes": round(alg),
                "traffic_over_alg": round(st["traffic_bytes"] / alg, 3) if "traffic_bytes" in st else None,
                "alg_bytes_model": "bench.call_bytes: every operand read once, every result written once "
                                   "(GEMM A/B/C/bias/residual; attention q/k/v/o/P; AdamW 38 B/param; "
                                   "touched embedding rows; the declared tensors of the other kernels)",
                "flop_per_step": step_flop, "flop_per_step_calls": calls_flop(eng),
                "step_gpu_ms": round(gpu_step * 1e3, 4),
                "traffic_source": pmc_note}
    out = {
        "metric": ("question-image pairs/sec, ResNet50+T5-large+6xSGA 384x384 fp8-weight train step (BASELINE configs[4])"
                   if args.config5 else "question-image pairs/sec, ResNet50+T5-base+SGA train step, 1/2/4/8 MI355X"),
        "value": round(value, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp8+bf16" if args.config5 else "bf16", "data": "synthetic",
        "config": {"workload": (f"ResNet50 + {lm} + {NB}xSGA train step"
                                + (" (BASELINE configs[1]; configs[2] at N=8)" if survey_cfg else "")
                                + (" (BASELINE configs[4]: e4m3 forward weight GEMMs)" if args.config5 else "")),
                   "model": f"resnet50+{lm}+{NB}xSGA", "global_batch": world * B, "per_gpu_batch": B,
                   "seq_len": L, "image_size": H, "answers": 170,
                   "parallelism": f"dp{world}" + (" (DataParallelStep, RCCL world 1)" if args.dp and world == 1 else ""),
                   "world_size": (dist.get_world_size() if dist else 1), "graph": not args.no_graph,
                   "resnet_pipelined": pipe},
        **({"rehearsal": "all ranks on cuda:0 over gloo: a code-path check, not a measurement"}
           if args.rehearse else {}),
        "roofline": roofline,
        "loss": round(loss, 5), "grad_norm": round(gnorm, 4),
        "host_issue_ms_per_step": round(t_issue * 1e3 / args.steps, 3),
    }
    if use_dp:                             # collective completion + exposed wait (HIP events), on 3
        dps.timing = True                  # steps after the timed region (its waits would perturb it)
        for i in range(3):
            step(args.steps + i)
        out["dp"] = dps.timing_report()
        out["dp"]["backend"] = dist.get_backend()
        out["dp"]["timing_steps"] = "3 steps after the timed region"
    if args.rehearse:                               # the N-rank path's results: lockstep across ranks
        eng.flush_optimizer()
        p = eng.P32[:: max(1, eng.P32.numel() // 65536)].cpu()
        ps = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(ps, p)
        out["rehearsal_lockstep"] = all(torch.equal(q, ps[0]) for q in ps)
    elif not args.no_kernel_rooflines:
        out.update(kernel_rooflines(eng, torch.cuda.current_stream(dev), pmc))   # PMC: the committed shapes only
    if world == 1 and not use_dp and not args.no_dp_line and not args.no_graph:
        # the N > 1 code path at N = 1, a second line beside the headline (same workload, same timing)
        del eng, dps, step
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        out["dp_world1"] = dp_world1_line(args, pkg, dev, pool, lm, dt)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pkg)
    if rank == 0:
        emit(out)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def kernel_rooflines(eng, stream, pmc):
    """Secondary per-kernel rooflines, each launch replayed alone between HIP events on its
    stream after the timed region (it only re-applies work the step already did)."""
    from vqa_amd import lib as VL
    out = {}
    # HBM: the fused AdamW-amsgrad pass over the whole arena (in-step it runs as parameter
    # ranges overlapped with the forward).  Algorithmic bytes per launch: read p, g, m, v,
    # vmax (20 B) + write p, m, v, vmax (16 B) + the bf16 shadow (2 B) per parameter.
    adam_call = eng.adam_full
    assert adam_call.name == "vqa_adamw_amsgrad"
    adam_bytes = 38.0 * eng.lay.total
    adam_dur = time_kernel(adam_call, 10, stream)
    adam_gbs = adam_bytes / adam_dur / 1e9
    out["roofline_hbm"] = {"bound": "hbm", "kernel": "adamw_kernel (fused clip-scaled AdamW-amsgrad + bf16 shadow)",
                           "achieved": round(adam_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(adam_gbs / HBM_PEAK_GBS, 4),
                           "traffic": (round(pmc["adamw_kernel"]["traffic_bytes"]) if "adamw_kernel" in pmc else None),
                           "algorithmic_bytes": adam_bytes, "kernel_avg_us": round(adam_dur * 1e6, 2)}
    # MFMA: the largest single launch, the ConvTranspose2d weight gradient as one GEMM batched
    # over the 9 taps (M=768, N=2048, K=B*49, batch 9 over vqa_tap_shift copies of dVIS;
    # 2*M*N*K*9 FLOP, the same work as the implicit-im2col form M=768, N=9*2048)
    wg_call = eng.scaler_dw_call
    assert wg_call.name == "vqa_gemm" and wg_call.desc.batch == 9
    cfg = VL.load().vqa_gemm_select(wg_call.desc)
    bm, bn, st = VL.GEMM_TILES[cfg]
    wm, wn = VL.GEMM_WAVES[cfg]
    kname = (f"gemm_kernel<{bm}, {bn}, {st}, {wm}, {wn}, false, false, false, false> (ConvTranspose2d dW, tap-batched "
             f"GEMM, batch 9, splitk={max(1, wg_call.desc.splitk)})")
    kdur = time_kernel(wg_call, 20, stream)
    kflop = 2.0 * wg_call.desc.m * wg_call.desc.n * wg_call.desc.k * wg_call.desc.batch
    k_tflops = kflop / kdur / 1e12
    out["roofline_gemm"] = {"bound": "mfma", "kernel": kname, "achieved": round(k_tflops, 1), "peak": MFMA_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(k_tflops / MFMA_PEAK_TFLOPS, 4),
                            "traffic": (round(pmc["convT_dW"]["traffic_bytes"]) if "convT_dW" in pmc else None),
                            "alg_bytes": call_bytes(wg_call),
                            "traffic_over_alg": (round(pmc["convT_dW"]["traffic_bytes"] / call_bytes(wg_call), 3)
                                                 if "convT_dW" in pmc else None),
                            "kernel_avg_us": round(kdur * 1e6, 2), "flop_per_launch": kflop}
    # north_star's SGA figure: MFMA utilisation of the SGA blocks' GEMM launches (the q/k/v,
    # merge and FFN linears of MHAtt / FFN, forward and backward; `gemm`) and of those plus
    # the attention cores (`all`): their FLOP per step over the sum of their launch times,
    # each replayed alone between HIP events (no neighbour overlap).  The committed PMC pass
    # (SQ_VALU_MFMA_BUSY_CYCLES over the same launches in the step) is quoted beside it.
    sga_calls = [c for c in eng.sga_vision_calls + eng.fwd_calls[eng._fsplit[2]:] + eng.bwd_calls[:eng._bsplit[0]]
                 if c.name in ("vqa_gemm", "vqa_gemm_pair", "vqa_attn_fwd", "vqa_attn_bwd")]

    def call_peak(c):                       # each launch's dense peak: e4m3 launches at the fp8 rate
        return FP8_PEAK_TFLOPS if c.name == "vqa_gemm" and c.desc.fp8 else MFMA_PEAK_TFLOPS

    def call_flop(c):
        if c.name == "vqa_gemm":
            return 2.0 * c.desc.m * c.desc.n * c.desc.k * max(1, c.desc.batch)
        if c.name == "vqa_gemm_pair":
            return sum(2.0 * d.m * d.n * d.k for d in c.desc)
        d = c.desc
        return (4.0 if c.name == "vqa_attn_fwd" else 8.0) * d.batch * d.heads * d.lq * d.lk * d.dh
    sga = {}
    times = {id(c): time_kernel(c, 10, stream) for c in sga_calls}
    for tag, names in (("gemm", ("vqa_gemm", "vqa_gemm_pair")), ("all", None)):
        cs = [c for c in sga_calls if names is None or c.name in names]
        fl = sum(call_flop(c) for c in cs)
        tm = sum(times[id(c)] for c in cs)
        # the peak of this mix: every launch at its own dtype's dense peak (config 5: the e4m3
        # forward GEMMs at 5,034, the rest at 2,517 TFLOP/s); config 2 is all bf16
        pk = fl / sum(call_flop(c) / call_peak(c) for c in cs)
        sga[tag] = {"launches": len(cs), "flop_per_step": fl, "kernel_us_per_step": round(tm * 1e6, 1),
                    "achieved": round(fl / tm / 1e12, 1), "peak": round(pk, 1), "frac": round(fl / tm / 1e12 / pk, 4)}
    gb = sum(call_bytes(c) for c in sga_calls if c.name in ("vqa_gemm", "vqa_gemm_pair"))
    sga["gemm"]["alg_bytes"] = gb
    if "sga_gemm" in pmc:
        sga["gemm"]["traffic"] = round(pmc["sga_gemm"]["traffic_bytes"])
        sga["gemm"]["traffic_over_alg"] = round(pmc["sga_gemm"]["traffic_bytes"] / gb, 3)
    out["sga_mfma"] = {"peak": sga["gemm"]["peak"], "unit": "TFLOP/s", "target_frac": 0.40, **sga,
                       "pmc_mfma_busy": pmc.get("sga_mfma_busy")}
    # e4m3 (config 5): the largest fp8 launch of the step against the fp8 dense peak
    f8 = [c for c in list(eng.res_calls) + eng.fwd_calls + eng.bwd_calls if c.name == "vqa_gemm" and c.desc.fp8]
    if f8:
        c = max(f8, key=call_flop)
        d = c.desc
        cfg = VL.load().vqa_gemm_select(d)
        bm, bn, st = VL.GEMM_TILES[cfg]
        kd = time_kernel(c, 20, stream)
        kt = call_flop(c) / kd / 1e12
        out["roofline_fp8"] = {"bound": "mfma", "kernel": f"gemm_kernel<{bm}, {bn}, {st}, ..., fp8> (e4m3 forward "
                                                          f"GEMM, m={d.m} n={d.n} k={d.k} batch={max(1, d.batch)}, "
                                                          f"splitk={max(1, d.splitk)})",
                               "achieved": round(kt, 1), "peak": FP8_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(kt / FP8_PEAK_TFLOPS, 4),
                               "traffic": (round(pmc["fp8_gemm"]["traffic_bytes"]) if "fp8_gemm" in pmc else None),
                               "kernel_avg_us": round(kd * 1e6, 2), "flop_per_launch": call_flop(c)}
    return out


if __name__ == "__main__":
    main()
