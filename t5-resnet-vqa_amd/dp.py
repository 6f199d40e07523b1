"""Data-parallel training step: one process per MI355X, gradients exchanged
with RCCL (torch.distributed backend "nccl") over xGMI, overlapped with the
backward pass.  (The reference trains on one device only,
trainer/faster_rcnn_vqa_trainer.py:61-62; this is the build's added strategy,
SURVEY.md §8e.)

Step on every rank (identical initial weights, rank-local batch):
  graph(forward) -> the backward as a few stage graphs (stage j: chain segment j beside the
  pending weight-gradient GEMMs of the segments before it), and after each stage an async
  all-reduce(SUM) of the buckets it finished, issued on a comm stream (they run while the next
  stages do) -> all-gather of (token id, dH row) pairs -> deterministic embedding scatter ->
  wait for the buckets -> graph(clip + AdamW), grads scaled by 1/world.

Buckets: the flat gradient arena is laid out in backward-completion order
(layout.py), so each finished bucket is a contiguous slice [a, b) of G32 and
RCCL works in place on it.  The dense 98.7 MB T5 embedding gradient is never
all-reduced: each rank ships only its <= B*L touched (id, row) pairs and every
rank rebuilds the identical summed rows with the sorted fixed-order scatter.
Because every exchange and kernel is deterministic, all ranks hold bit-identical
parameters after every step.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import lib as L
from . import ops
from . import synthetic as S
from .engine import no_gc_capture


# T5 weight-gradient groups of a DP engine (VQAEngine t5_dw_group), top layer first: the
# buckets of layers 11..8, 7..4 and 3..1 are all-reduced while the backward continues, and
# the last, exposed bucket holds one layer
DP_T5_DW_GROUPS = (4, 4, 3, 1)


def dp_t5_dw_groups(layers=12):
    """The DP grouping for a T5 stack of `layers` (t5-large: 24 -> (8, 8, 6, 2)): the same
    shape, scaled, with a short last group so the exposed bucket stays small."""
    if layers == 12:
        return DP_T5_DW_GROUPS
    g = [layers // 3, layers // 3, layers // 4]
    return tuple(g + [layers - sum(g)])


def plan_buckets(ready_marks, end, min_bytes=24 << 20):
    """Group the engine's ready marks (call index, prefix end) into buckets of
    at least `min_bytes` of fp32 gradient.  Returns [(call_index, start, stop)]."""
    out, start = [], 0
    for i, (ci, stop) in enumerate(ready_marks):
        stop = min(stop, end)
        last = i == len(ready_marks) - 1
        if stop - start >= min_bytes // 4 or (last and stop > start):
            if last and out and stop - start < min_bytes // 32:
                out[-1] = (ci, out[-1][1], stop)            # a tiny remainder joins the last bucket
            else:
                out.append((ci, start, stop))
            start = stop
    return out


def plan_shards(buckets, world, align=64):
    """Sharded optimizer (DataParallelStep(shard_optimizer=True)): each bucket [a, b) is cut
    into `world` equal chunks of a multiple of `align` elements, chunk r owned by rank r (its
    reduce-scatter target and the slice of the AdamW update it runs), plus a remainder
    [a + world*chunk, b) shorter than world*align that every rank all-reduces and updates.
    Returns [(a, chunk, b)] (chunk may be 0: the whole bucket is remainder)."""
    out = []
    for _, a, b in buckets:
        chunk = (b - a) // (world * align) * align
        out.append((a, chunk, b))
    return out


def _after(stream, other):
    """`stream` waits for everything issued so far on `other` (an event, no host sync)."""
    if stream is other:
        return
    ev = torch.cuda.Event()
    ev.record(other)
    stream.wait_event(ev)


def _wait_only(w):
    """The current stream waits for the collective of `w` alone -- never its follow-up copy
    (_Then): the timing stream only observes completions, it must not write anything."""
    return w.wait_only() if hasattr(w, "wait_only") else w.wait()


# RCCL collectives are issued with async_op=False from the comm stream: torch's ProcessGroupNCCL then
# launches them on the CURRENT stream (the comm stream, whose hardware queue the step chooses, DESIGN
# §5) instead of its own pooled stream, and the host does not block (no blocking-wait mode)
COMM_ON_STREAM = True


class _OnStream:
    """Collectives already enqueued on the current (comm) stream: wait() makes the waiting stream
    wait for an event recorded right after them (wait_only is the same: nothing follows)."""
    def __init__(self):
        self.ev = torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream())

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    wait_only = wait


class _Done:
    """A completed collective (host-staged gloo path): wait() is a no-op."""
    def wait(self):
        return True

    wait_only = wait


class _Then:
    """A collective followed by a device copy on the waiting stream (issued at wait(), once: the
    step's stream calls wait(); bench.py's timing stream calls wait_only())."""
    def __init__(self, work, then):
        self.work, self.then = work, then

    def wait(self):
        self.work.wait()
        self.then()
        return True

    def wait_only(self):
        return self.work.wait()


class _All:
    """Several collectives of one bucket waited on as one (the sharded exchange)."""
    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True

    def wait_only(self):
        for w in self.works:
            _wait_only(w)
        return True


def _staged(t, group):
    """gloo runs these collectives on host tensors only: stage device tensors through host
    memory (CPU tests and the single-GPU multi-process test; RCCL works on HBM in place)."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def allreduce_buckets(flat, buckets, group=None):
    """Launch one async SUM all-reduce per bucket slice of `flat`; returns works."""
    import torch.distributed as dist
    if _staged(flat, group):
        for _, a, b in buckets:
            h = flat[a:b].cpu()
            dist.all_reduce(h, group=group)
            flat[a:b].copy_(h)
        return [_Done() for _ in buckets]
    if COMM_ON_STREAM and flat.is_cuda:
        for _, a, b in buckets:
            dist.all_reduce(flat[a:b], group=group, async_op=False)
        return [_OnStream()]
    return [dist.all_reduce(flat[a:b], group=group, async_op=True) for _, a, b in buckets]


def gather_rows(ids, rows, out_ids, out_rows, group=None):
    """All-gather the rank-local (token id, gradient row) pairs (rank-major order)."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":                  # CPU tests: list form
        w = dist.get_world_size(group)
        if _staged(rows, group):
            hi, hr = torch.empty(out_ids.shape, dtype=out_ids.dtype), torch.empty(out_rows.shape, dtype=out_rows.dtype)
            dist.all_gather(list(hi.chunk(w)), ids.reshape(-1).cpu(), group=group)
            dist.all_gather(list(hr.chunk(w)), rows.cpu(), group=group)
            out_ids.copy_(hi)
            out_rows.copy_(hr)
            return [_Done(), _Done()]
        w1 = dist.all_gather(list(out_ids.chunk(w)), ids.reshape(-1), group=group, async_op=True)
        w2 = dist.all_gather(list(out_rows.chunk(w)), rows, group=group, async_op=True)
        return [w1, w2]
    if COMM_ON_STREAM:
        dist.all_gather_into_tensor(out_ids, ids.reshape(-1), group=group, async_op=False)
        dist.all_gather_into_tensor(out_rows, rows, group=group, async_op=False)
        return [_OnStream()]
    w1 = dist.all_gather_into_tensor(out_ids, ids.reshape(-1), group=group, async_op=True)
    w2 = dist.all_gather_into_tensor(out_rows, rows, group=group, async_op=True)
    return [w1, w2]


def gather_tensor(x, out, group=None):
    """All-gather one tensor per rank into `out` (rank-major): the step's token ids at its start,
    the (id-ordered) embedding-gradient rows after the backward.  gloo: staged through host memory."""
    import torch.distributed as dist
    w = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        if x.is_cuda:
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather(list(h.chunk(w)), x.reshape(-1, *out.shape[1:]).cpu(), group=group)
            out.copy_(h)
            return [_Done()]
        dist.all_gather(list(out.chunk(w)), x.reshape(-1, *out.shape[1:]), group=group)
        return [_Done()]
    if COMM_ON_STREAM:
        dist.all_gather_into_tensor(out, x.reshape(-1, *out.shape[1:]), group=group, async_op=False)
        return [_OnStream()]
    return [dist.all_gather_into_tensor(out, x.reshape(-1, *out.shape[1:]), group=group, async_op=True)]


# share of the next batch's frozen-ResNet calls forked beside the forward graph (pipelined
# engines; the rest go beside the first backward stage), DataParallelStep(res_split=...)
RES_SPLIT = 1.0


def plan_stages(segments, scaler, dw_stream=True):
    """The DP backward's stages (DataParallelStep._plan_schedule).  segments: the backward's
    calls cut at the bucket marks (bucket k final after segment k's calls); scaler: the
    (lo, hi) call range of the ConvTranspose2d scaler segment (all weight gradient); calls with
    `.side` set are weight-gradient calls.  Each stage is {"ops": [("main" | "fork", calls)],
    "final": [bucket]}: a segment's weight-gradient calls are forked beside the NEXT segment
    that has chain calls, a stage ends after a chain segment only where buckets become final,
    and the last segment's weight gradients end the last stage.  Returns (stages, index of the
    stage with the last chain call)."""
    stages, ops, fin, pend, pend_b, prev = [], [], [], [], [], 0
    for k, seg in enumerate(segments):
        lo, hi = prev, prev + len(seg)
        prev = hi
        if (lo, hi) == tuple(scaler):
            chain, dw = [], list(seg)
        elif dw_stream:
            chain, dw = [c for c in seg if not c.side], [c for c in seg if c.side]
        else:
            chain, dw = list(seg), []
        if chain:
            if pend:                                        # the pending dW, beside this chain
                ops.append(("fork", pend))
                fin, pend, pend_b = fin + pend_b, [], []
            ops.append(("main", chain))
        if dw:
            pend, pend_b = pend + dw, pend_b + [k]
        else:                                               # final with its own chain
            fin = fin + [k]
        if chain and fin:                                   # a stage ends where buckets become final
            stages.append({"ops": ops, "final": fin})
            ops, fin = [], []
    if pend:                           # the last dW: nothing left to overlap it with, no stage of its own
        if ops or not stages:
            ops.append(("fork", pend))
            fin = fin + pend_b
        else:
            stages[-1]["ops"].append(("fork", pend))
            stages[-1]["final"] = stages[-1]["final"] + pend_b
    if ops or fin:
        stages.append({"ops": ops, "final": fin})
    rows = max(j for j, st in enumerate(stages) if any(kd == "main" for kd, _ in st["ops"]))
    return stages, rows


class DataParallelStep:
    def __init__(self, engine, group=None, bucket_mb=24, use_graph=True, shard_optimizer=False, res_split=RES_SPLIT):
        import torch.distributed as dist
        self.eng, self.group = engine, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.shard = bool(shard_optimizer)
        e = engine
        e.set_grad_scale(1.0 / self.world)
        # the NLL mean over the global batch (ranks may hold unequal rows, or none): the head
        # backward divides by the all-reduced valid-row count over world (engine.use_global_rows)
        e.use_global_rows(self.world)
        emb = e.lay["t5.embed"]
        self.buckets = plan_buckets(e.ready_marks, emb.offset, bucket_mb << 20)
        calls = e.bwd_calls[:-1]                            # all but the local embedding scatter
        assert e.bwd_calls[-1] is e.emb_call
        T, D = e.T, e.D
        dev = e.dev
        # every rank's token ids, gathered at the start of the step (with the valid-row count): the
        # embedding rows the step touches on ANY rank are known before the backward, so the table's
        # untouched rows are updated beside it (engine.emb_pre) and only the gradient rows (GDH)
        # are gathered after the backward.  The rows to re-zero are the previous step's gathered
        # ids (every rank's rows were written): GIDS_PREV, then GIDS_PREV <- GIDS.
        self.GIDS = torch.zeros(self.world * T, dtype=torch.int64, device=dev)
        self.GIDS_PREV = torch.zeros(self.world * T, dtype=torch.int64, device=dev)
        assert calls[0] is e.zero_calls[0]
        g = e.g32["t5.embed"]
        calls = [ops.Call("vqa_embedding_zero_rows", self.GIDS_PREV.data_ptr(), self.GIDS.data_ptr(), self.world * T,
                          g.data_ptr(), D, S.T5_VOCAB, keep=(self.GIDS_PREV, self.GIDS, g))] + calls[1:]
        self.segments, prev = [], 0
        for ci, _, _ in self.buckets:
            self.segments.append(calls[prev:ci])
            prev = ci
        self.tail = calls[prev:]                            # nothing should remain after the last mark
        self.GDH = torch.zeros(self.world * T, D, dtype=torch.float32, device=dev)
        self.WS = torch.empty(3 * min(self.world * T, 16384), dtype=torch.int32, device=dev)   # per 16384-token slice
        self.emb_call = ops.Call("vqa_embedding_bwd", self.GIDS.data_ptr(), self.GDH.data_ptr(),
                                 e.g32["t5.embed"].data_ptr(), self.world * T, D, S.T5_VOCAB, self.WS.data_ptr(),
                                 keep=(self.GIDS, self.GDH, self.WS, e.g32["t5.embed"]))
        if self.shard:
            self._plan_sharded_optimizer()
        self._plan_schedule()
        # pipelined engines: the next batch's frozen ResNet (IMG -> F4N, read by the next step's
        # copy_f4 only) runs INSIDE the step's graphs, as on one GPU: its first `res_split` of the
        # calls forked beside the forward, the rest beside the first backward stage.  (Replayed as a
        # graph of its own on its stream it shared a hardware queue with the stage graphs' kernels,
        # one ResNet kernel holding back the chain kernels queued behind it.)
        r1 = int(round(len(e.res_calls) * float(res_split))) if e.pipeline else 0
        self._res_a = list(e.res_calls[:r1]) if e.pipeline else []
        if e.pipeline and r1 < len(e.res_calls):
            self.stages[0]["ops"].insert(0, ("res", list(e.res_calls[r1:])))
        self.graphs = None
        # exposed-communication timing (bench at N > 1): HIP events on the compute stream right
        # before and after each collective's wait, i.e. how long the step's stream stalls on it
        self.timing = False
        self._ev = []
        if use_graph:
            self.capture()
        # the dense embedding gradient must be zero outside the rows the scatter writes: the
        # zero-rows call only clears the PREVIOUS step's gathered ids (GIDS), so clear rows that
        # local backward passes (warm-ups, a train_step before this object) left behind
        e.g32["t5.embed"].zero_()

    def _plan_sharded_optimizer(self):
        """Reduce-scatter + sharded AdamW + all-gather (ZeRO stage 1):
        the buckets' gradients are reduce-scattered instead of all-reduced, rank r runs the
        clip-scaled AdamW-amsgrad on its chunk of every bucket only (m, v, vmax of other chunks
        are never touched here), and the updated fp32 masters and bf16 shadows of the chunks are
        all-gathered.  The remainders of the buckets and the embedding table (whose gradient rows
        every rank rebuilds identically) are updated by every rank.  The clip norm is the sum
        of per-range squared-norm partials, all-reduced (each owned chunk counted by its owner,
        the replicated ranges by rank 0 only), then finalized as usual."""
        e = self.eng
        self.shards = plan_shards(self.buckets, self.world)
        n, emb = e.lay.total, e.lay["t5.embed"].offset
        r, N = self.rank, self.world
        own = [(a + r * c, a + (r + 1) * c) for a, c, b in self.shards if c > 0]
        rep = [(a + N * c, b) for a, c, b in self.shards if b > a + N * c] + [(emb, n)]
        K = e.SQ_PARTS
        ranges = own + rep
        self.WS_SQN = torch.zeros(len(ranges) * K, dtype=torch.float64, device=e.dev)
        sq = []
        for i, (lo, hi) in enumerate(ranges):
            if i < len(own) or r == 0:                      # a replicated range is counted once
                sq.append(ops.Call("vqa_grad_sqnorm", ops.addr(e.G32, lo), hi - lo, ops.addr(self.WS_SQN, i * K), K,
                                   keep=(e.G32, self.WS_SQN)))
        self.sq_calls = sq
        fin = []
        e._call(fin, "vqa_optim_finalize", self.WS_SQN, len(ranges) * K, float(e.grad_scale), float(e.max_norm),
                int(e.warmup), int(e.total), float(e.betas[0]), float(e.betas[1]), e.opt_state)
        self.finalize_call = fin[0]
        self.adam_calls = [e.adam_range_call(lo, hi) for lo, hi in ranges]
        # reduce-scatter outputs, one slice per bucket (several are in flight at once); each is
        # copied into the rank's chunk of G32 once its collective is done
        offs = np.concatenate([[0], np.cumsum([c for _, c, _ in self.shards])]).astype(np.int64)
        self.rs_off = [int(o) for o in offs[:-1]]
        self.RS_OUT = torch.empty(max(int(offs[-1]), 1), dtype=torch.float32, device=e.dev)

    def _sharded_collectives_after(self, bk_index):
        """Reduce-scatter of bucket `bk_index`'s chunks (owner r receives the sum of chunk r)
        and all-reduce of its remainder; returns the works."""
        import torch.distributed as dist
        e = self.eng
        a, c, b = self.shards[bk_index]
        N, r = self.world, self.rank
        works = []
        if c > 0:
            full, mine = e.G32[a:a + N * c], e.G32[a + r * c:a + (r + 1) * c]
            if _staged(full, self.group) or dist.get_backend(self.group) == "gloo":
                h = full.cpu()                              # gloo: all-reduce, keep the own chunk
                dist.all_reduce(h, group=self.group)
                mine.copy_(h[r * c:(r + 1) * c])
                works.append(_Done())
            else:
                # into a separate buffer (no reliance on RCCL's in-place aliasing rule), then
                # copied into the own chunk on the NCCL work's completion (the wait below)
                out = self.RS_OUT[self.rs_off[bk_index]:self.rs_off[bk_index] + c]
                if COMM_ON_STREAM:                          # on the comm stream, the copy right behind it
                    dist.reduce_scatter_tensor(out, full, group=self.group, async_op=False)
                    mine.copy_(out)
                    works.append(_OnStream())
                else:
                    works.append(_Then(dist.reduce_scatter_tensor(out, full, group=self.group, async_op=True),
                                       lambda out=out, mine=mine: mine.copy_(out)))
        if b > a + N * c:
            works += allreduce_buckets(e.G32, [(None, a + N * c, b)], self.group)
        return [_All(works)]

    def _sharded_optimizer(self):
        """sqnorm partials -> all-reduce -> finalize -> AdamW on the own chunks + the replicated
        ranges -> clear the pending flag (the forward's deferred ranges then do nothing) ->
        all-gather the chunks' fp32 masters and bf16 shadows."""
        import torch.distributed as dist
        e = self.eng
        s = L.stream_handle()
        self.WS_SQN.zero_()
        for c in self.sq_calls:
            c(s)
        if _staged(self.WS_SQN, self.group):
            h = self.WS_SQN.cpu()
            dist.all_reduce(h, group=self.group)
            self.WS_SQN.copy_(h)
        else:
            dist.all_reduce(self.WS_SQN, group=self.group)
        self.finalize_call(s)
        for c in self.adam_calls:
            c(s)
        e.clear_pending(s)
        N, r = self.world, self.rank
        for a, c, b in self.shards:
            if c == 0:
                continue
            for t in (e.P32, e.P16):
                full, mine = t[a:a + N * c], t[a + r * c:a + (r + 1) * c]
                if _staged(full, self.group):
                    parts = [torch.empty(c, dtype=t.dtype) for _ in range(N)]
                    dist.all_gather(parts, mine.cpu(), group=self.group)
                    full.copy_(torch.cat(parts))
                else:
                    dist.all_gather_into_tensor(full, mine.clone(), group=self.group)
        if e.fp8 and not e.defer_opt:
            # the e4m3 weight copies follow the gathered masters (a deferred update requantizes
            # them range by range in the next forward: its _Seq(AdamW range, quant) calls)
            self._run(e.quant_all)

    def sync_optimizer_state(self):
        """Sharded optimizer: all-gather the AdamW moments of every chunk (each rank holds only
        its own chunks' up-to-date m, v, vmax) so optimizer_state() / checkpoints see them."""
        import torch.distributed as dist
        if not self.shard:
            return
        e = self.eng
        N, r = self.world, self.rank
        for a, c, b in self.shards:
            if c == 0:
                continue
            for t in (e.M, e.V, e.VMAX):
                full, mine = t[a:a + N * c], t[a + r * c:a + (r + 1) * c]
                if _staged(full, self.group):
                    parts = [torch.empty(c, dtype=t.dtype) for _ in range(N)]
                    dist.all_gather(parts, mine.cpu(), group=self.group)
                    full.copy_(torch.cat(parts))
                else:
                    dist.all_gather_into_tensor(full, mine.clone(), group=self.group)

    def _run(self, calls):
        s = L.stream_handle()
        for c in calls:
            c(s)

    # ------------------------------------------------------------------ schedule
    def _plan_schedule(self):
        """The backward as a short sequence of STAGES, each one graph: a stage runs chain
        segments (the input-gradient chain, the step's stream) with the weight-gradient calls
        of the segments before them forked beside them (`wside`) -- the same placement as the
        single-GPU step graph, where the batched dW GEMMs trail the chain on their own stream,
        software-pipelined across graph boundaries so no stage waits for its own last segment's
        weight gradients; a stage ends only where buckets become final, and the last segment's
        dW ends the last stage.  A bucket is final when the stage that ran its last call has ended;
        the host then issues its collective from a comm stream behind an event on the step's
        stream, so it runs while the next stages do.  (Measured in round 4: one graph per
        segment with the dW calls replayed as separate graphs on `wside` ran 14 % slower than the
        engine step at world 1 -- those launches shared a hardware queue with the chain; the
        collectives captured INTO one backward graph ran 11 % slower -- that graph executed
        with its captured streams on the step stream's hardware queue, profiles/r04_dp_trace.txt;
        ROCm's torch refuses external event records in a capture.)  The ConvTranspose2d scaler
        dW segment (engine: on `side`, beside the T5 backward) is all weight gradient, so it is
        deferred into the next stage like the others."""
        e = self.eng
        self.stages, self.rows_stage = plan_stages(self.segments, e._bsplit, e.dw_stream)
        assert sorted(k for st in self.stages for k in st["final"]) == list(range(len(self.buckets)))
        # after the last collective: the embedding scatter, then (unless sharded) the whole optimizer
        # plan (grad-norm partials, clip, AdamW).  The [0, a) partials once ran on a stream of their own
        # behind the early buckets' collectives: at world 1 they did not overlap anything (trace), and at
        # N > 1 that stream's wait on a running collective would hold back whatever stage kernels share
        # its hardware queue
        # the embedding table's update split by rows (engine.emb_pre; bit-identical to the dense
        # range): the rows no rank touched beside the first stage (marks from the gathered ids),
        # the rel-bias range and the touched rows in the finish graph.  The squared-norm partials of
        # [0, a) (engine._sq_split) run on the comm stream right behind the all-reduce that completes
        # that prefix, so the finish keeps only the later partials.
        self.emb_pre = []
        self._sq0_stage = None
        opt = list(e.opt_calls)
        if not self.shard:
            if e.embed_split:
                self.emb_pre = [ops.Call("vqa_embed_mark", self.GIDS.data_ptr(), self.world * e.T, S.T5_VOCAB,
                                         e.EMB_MARK.data_ptr(), e.opt_state.data_ptr(),
                                         keep=(self.GIDS, e.EMB_MARK, e.opt_state)), e.emb_pre[1]]
                self.stages[0]["ops"].insert(0, ("emb", self.emb_pre))
                opt = opt[:2] + list(e.tail_calls)
            a = e._sq_split[1] if e._sq_split is not None else None
            if a is not None:
                done = 0
                for j, st in enumerate(self.stages):
                    if st["final"]:
                        done = max(done, max(self.buckets[k][2] for k in st["final"]))
                    if done >= a and st["final"]:
                        self._sq0_stage = j
                        break
            if self._sq0_stage is not None:
                assert opt[0].name == "vqa_grad_sqnorm"
                self._sq0_call = opt[0]
                opt = opt[1:]
        self.finish_calls = self.tail + [self.emb_call] + ([] if self.shard else opt)
        # (high-priority streams -- hardware queues of their own -- measured 2.5x slower, r04)
        # issues the collectives behind the stage events (VQA_DP_COMM, an A/B switch: "own" a stream of
        # its own; "side" / "wside" the engine's capture-only fork streams, whose hardware queue the
        # replayed graphs do not use -- the graphs run on their execs' internal parallel streams)
        comm = os.environ.get("VQA_DP_COMM", "wside")
        self._comm = {"own": None, "side": e._side, "wside": e._wside}[comm] or torch.cuda.Stream(e.dev)
        self._tstream = torch.cuda.Stream(e.dev)            # timing mode: collective completions

    def stage_plan(self):
        """Per stage: its calls in order as ("chain" | "dw_fork", count), and the buckets final
        after it."""
        return [{"ops": [({"main": "chain", "fork": "dw_fork", "res": "resnet_fork", "emb": "embedding_rows_fork"}[kd],
                          len(c)) for kd, c in st["ops"]],
                 "final_buckets": st["final"]} for st in self.stages]

    def _run_stage(self, st):
        """One stage on the current stream: its chain calls, and at each fork point the pending
        weight-gradient calls on `wside` (after everything issued so far on the chain), joined
        at the end of the stage."""
        e = self.eng
        main = torch.cuda.current_stream(e.dev)
        forked = set()
        for kind, calls in st["ops"]:
            if kind == "main":
                self._run(calls)
            else:     # "fork": pending dW; "res": the next batch's ResNet; "emb": the untouched embedding rows
                side = {"fork": e._wside, "res": e._rstream, "emb": e._side}[kind]
                _after(side, main)
                with torch.cuda.stream(side):
                    self._run(calls)
                forked.add(side)
        for side in forked:
            _after(main, side)

    def _backward_exchange(self):
        """The staged backward with the exchange issued between the stages; the step's stream
        waits on the collectives only at the end, then runs the embedding scatter + (unless
        sharded) the optimizer plan as one graph.  The comm stream never waits on a collective
        (a wait packet there would hold back whatever stage kernels share its hardware queue);
        only the grad-norm stream and the final join do.  Returns the timing record (timing
        mode): stage-end and collective-done events, the final wait."""
        e = self.eng
        g = self.graphs
        main = torch.cuda.current_stream(e.dev)
        exchange = lambda i, bk: self._sharded_collectives_after(i)    # noqa: E731
        comm = self._comm
        tm = {"stage": {}, "done": {}} if self.timing else None
        works = {}

        def mark_done(key, ws):
            if tm is not None:                              # completion seen from a timing-only stream
                with torch.cuda.stream(self._tstream):      # (waits only: the copies stay on the step's stream)
                    for w in ws:
                        _wait_only(w)
                    tm["done"][key] = torch.cuda.Event(enable_timing=True)
                    tm["done"][key].record(self._tstream)
        for j, st in enumerate(self.stages):
            if g is not None:
                g[f"stage{j}"].replay()
            else:
                self._run_stage(st)
            if not (st["final"] or j == self.rows_stage):
                continue
            if tm is not None:
                tm["stage"][j] = torch.cuda.Event(enable_timing=True)
                tm["stage"][j].record(main)
            _after(comm, main)
            with torch.cuda.stream(comm):
                if j == self.rows_stage:
                    works["rows"] = gather_tensor(e.dH32, self.GDH, self.group)
                    mark_done("rows", works["rows"])
                if self.shard:
                    for k in st["final"]:
                        works[k] = exchange(k, self.buckets[k])
                        mark_done(k, works[k])
                else:                                       # the stage's buckets are contiguous: one all-reduce
                    ks = st["final"]
                    assert ks == list(range(ks[0], ks[-1] + 1))
                    ws = allreduce_buckets(e.G32, [(None, self.buckets[ks[0]][1], self.buckets[ks[-1]][2])], self.group)
                    for k in ks:
                        works[k] = ws if k == ks[-1] else []
                        mark_done(k, ws)
                    if j == self._sq0_stage and (COMM_ON_STREAM or _staged(e.G32, self.group)):
                        self._sq0_call(L.stream_handle(comm))     # behind the all-reduce of [0, a)
        if tm is not None:
            tm["wait"] = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            tm["wait"][0].record(main)
        for key, ws in works.items():
            for w in ws:
                w.wait()
        _after(main, comm)                                  # gloo: the staged copies ran on comm
        if tm is not None:
            tm["wait"][1].record(main)
        self._play("finish", self.finish_calls)
        return tm

    def _play(self, name, calls):
        if self.graphs is not None:
            self.graphs[name].replay()
        else:
            self._run(calls)

    def capture(self):
        e = self.eng
        e.flush_optimizer()              # the warm-up's backward must not overwrite a pending update's G
        e.ROWTOT.fill_(float(e.B * self.world))             # a finite divisor for the warm-up's head backward
        s = torch.cuda.Stream(e.dev)
        s.wait_stream(torch.cuda.current_stream(e.dev))
        saved_rng = e.RNG.clone()
        with torch.cuda.stream(s):                          # warm-up outside capture (no optimizer update)
            e._run(e.fwd_calls)
            e.backward()
        torch.cuda.current_stream(e.dev).wait_stream(s)
        torch.cuda.synchronize(e.dev)
        e.RNG.copy_(saved_rng)                              # the warm-up must not consume a dropout draw
        with no_gc_capture():
            self.graphs = self._capture_all(s)

    def _capture_all(self, s):
        e = self.eng
        gs = {}

        def cap(name, fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                fn()
            gs[name] = g
        cap("fwd", self._fwd)
        for j, st in enumerate(self.stages):
            cap(f"stage{j}", lambda st=st: self._run_stage(st))
        cap("finish", lambda: self._run(self.finish_calls))
        return gs

    def _fwd(self):
        """The forward (ConvTranspose2d || T5 encoder, then SGA; engine.run_forward_streams) with,
        when pipelined, the first part of the next batch's frozen ResNet forked beside it on
        `_rstream` -- captured first, as the single-GPU step graph captures it -- and joined at
        its end."""
        e = self.eng
        main = torch.cuda.current_stream(e.dev)
        if self._res_a:
            _after(e._rstream, main)
            with torch.cuda.stream(e._rstream):
                self._run(self._res_a)
        e.run_forward_streams()
        if self._res_a:
            _after(main, e._rstream)

    def _exchange_step_start(self):
        """The step's opening exchange, on the comm stream: this rank's valid-row count
        (vqa_count_targets, on the step's stream) summed over the ranks -- the head backward (first
        backward stage) divides by it -- and every rank's token ids gathered into GIDS (the
        embedding rows the step touches anywhere: the untouched rows' update in the first stage,
        the re-zeroing and the scatter).  Issued before the forward, waited on after it: the two
        small collectives run while the forward does."""
        e = self.eng
        main = torch.cuda.current_stream(e.dev)
        e.count_call(L.stream_handle(main))
        _after(self._comm, main)
        with torch.cuda.stream(self._comm):
            ws = allreduce_buckets(e.ROWTOT, [(None, 0, 1)], self.group)
            return ws + gather_tensor(e.IDS, self.GIDS, self.group)

    def step(self):
        e = self.eng
        rows = self._exchange_step_start()
        if e.pipeline:                                      # F4 <- F4N: this batch's features (last step's ResNet)
            e.copy_f4(L.stream_handle(torch.cuda.current_stream(e.dev)))
        if self.graphs is not None:
            self.graphs["fwd"].replay()
        else:
            self._fwd()
        for w in rows:                                      # long done: the forward ran meanwhile
            w.wait()
        _after(torch.cuda.current_stream(e.dev), self._comm)   # gloo: the staged copy ran on comm
        tev = self._backward_exchange()
        if self.shard:
            self._sharded_optimizer()
        if self.timing:
            self._ev.append(tev)

    def timing_report(self):
        """Over the steps run with `timing` on (HIP events): for the row gather and each gradient
        bucket, how long after the end of the stage that finished it its collective completed
        (queueing behind the earlier ones included), and the step stream's exposed wait on the
        exchange before the embedding scatter + optimizer."""
        torch.cuda.synchronize()
        if not self._ev:
            return None
        e = self.eng
        stage_of = {k: j for j, st in enumerate(self.stages) for k in st["final"]}
        stage_of["rows"] = self.rows_stage

        def mean(f):
            return round(float(np.mean([f(t) for t in self._ev])), 1)
        lag = {k: mean(lambda t, k=k: t["stage"][stage_of[k]].elapsed_time(t["done"][k]) * 1e3) for k in stage_of}
        return {"world_size": self.world, "steps": len(self._ev), "stages": self.stage_plan(),
                "embedding_rows_gather": {"bytes": int(self.world * e.T * (e.D * 4 + 8)),
                                          "done_us_after_stage": lag["rows"]},
                "buckets": [{"start": int(a), "stop": int(b), "bytes": int(4 * (b - a)), "stage": stage_of[k],
                             "done_us_after_stage": lag[k]} for k, (_, a, b) in enumerate(self.buckets)],
                "exposed_wait_us_total": mean(lambda t: t["wait"][0].elapsed_time(t["wait"][1]) * 1e3)}
