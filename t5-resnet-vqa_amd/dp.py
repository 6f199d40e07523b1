"""Data-parallel training step: one process per MI355X, gradients exchanged
with RCCL (torch.distributed backend "nccl") over xGMI, overlapped with the
backward pass.  (The reference trains on one device only,
trainer/faster_rcnn_vqa_trainer.py:61-62; this is the build's added strategy,
SURVEY.md §8e.)

Step on every rank (identical initial weights, rank-local batch):
  graph(forward) -> for each backward segment: graph(segment) ; async
  all-reduce(SUM) of the gradient bucket that segment finalised  ->
  all-gather of (token id, dH row) pairs -> deterministic embedding scatter ->
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
            out.append((ci, start, stop))
            start = stop
    return out


class _Done:
    """A completed collective (host-staged gloo path): wait() is a no-op."""
    def wait(self):
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
    w1 = dist.all_gather_into_tensor(out_ids, ids.reshape(-1), group=group, async_op=True)
    w2 = dist.all_gather_into_tensor(out_rows, rows, group=group, async_op=True)
    return [w1, w2]


class DataParallelStep:
    def __init__(self, engine, group=None, bucket_mb=24, use_graph=True):
        import torch.distributed as dist
        self.eng, self.group = engine, group
        self.world = dist.get_world_size(group)
        e = engine
        e.set_grad_scale(1.0 / self.world)
        emb = e.lay["t5.embed"]
        self.buckets = plan_buckets(e.ready_marks, emb.offset, bucket_mb << 20)
        calls = e.bwd_calls[:-1]                            # all but the local embedding scatter
        assert e.bwd_calls[-1] is e.emb_call
        T, D = e.T, e.D
        dev = e.dev
        self.GIDS = torch.zeros(self.world * T, dtype=torch.int64, device=dev)
        # the rows to re-zero are the previous step's GATHERED ids (every rank's rows were written);
        # GIDS still holds them when the backward starts (the gather runs after the first segment)
        assert calls[0] is e.zero_calls[0]
        g = e.g32["t5.embed"]
        calls = [ops.Call("vqa_embedding_zero_rows", self.GIDS.data_ptr(), None, self.world * T, g.data_ptr(), D,
                          S.T5_VOCAB, keep=(self.GIDS, g))] + calls[1:]
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

    def _run(self, calls):
        s = L.stream_handle()
        for c in calls:
            c(s)

    def capture(self):
        e = self.eng
        e.flush_optimizer()              # the warm-up's backward must not overwrite a pending update's G
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

        def cap(name, calls):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._run(calls)
            gs.setdefault(name, []).append(g)
        g = torch.cuda.CUDAGraph()                          # forward: ResNet || T5 encoder on two streams
        with torch.cuda.graph(g, stream=s):
            e.run_forward_streams()
        gs["fwd"] = [g]
        if e.pipeline:                                      # the next batch's ResNet, replayed beside the step
            cap("res", e.res_calls)
        for seg in self.segments:
            cap("seg", seg)
        cap("tail", self.tail + [self.emb_call])
        cap("opt", e.opt_calls)
        return gs

    def _res_begin(self):
        """Pipelined engines: F4 <- F4N, then the next batch's frozen ResNet on its own
        stream (graph or eager), overlapping this whole step; _res_end joins it."""
        e = self.eng
        if not e.pipeline:
            return
        main = torch.cuda.current_stream(e.dev)
        e.copy_f4(L.stream_handle(main))
        ev = torch.cuda.Event()
        ev.record(main)
        e._rstream.wait_event(ev)
        with torch.cuda.stream(e._rstream):
            if self.graphs is not None:
                self.graphs["res"][0].replay()
            else:
                self._run(e.res_calls)

    def _res_end(self):
        e = self.eng
        if e.pipeline:
            ev = torch.cuda.Event()
            ev.record(e._rstream)
            torch.cuda.current_stream(e.dev).wait_event(ev)

    def step(self):
        e = self.eng
        self._res_begin()
        if self.graphs is None:
            e.forward()
            works = []
            for seg, bk in zip(self.segments, self.buckets):
                self._run(seg)
                works += allreduce_buckets(e.G32, [bk], self.group)
            works += gather_rows(e.IDS, e.dH32, self.GIDS, self.GDH, self.group)
            for w in works[-2:]:
                w.wait()
            self._run(self.tail + [self.emb_call])
            for w in works[:-2]:
                w.wait()
            self._run(e.opt_calls)
            self._res_end()
            return
        g = self.graphs
        g["fwd"][0].replay()
        works = []
        for seg, bk in zip(g["seg"], self.buckets):
            seg.replay()
            works += allreduce_buckets(e.G32, [bk], self.group)
        works += gather_rows(e.IDS, e.dH32, self.GIDS, self.GDH, self.group)
        evs = []
        self._wait(works[-2:], evs)                         # the embedding rows: needed by the tail
        g["tail"][0].replay()
        for w in works[:-2]:
            self._wait([w], evs)
        g["opt"][0].replay()
        self._res_end()
        if self.timing:
            self._ev.append(evs)

    def _wait(self, works, evs):
        if not self.timing:
            for w in works:
                w.wait()
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for w in works:
            w.wait()
        b.record()
        evs.append((a, b))

    def timing_report(self):
        """Mean exposed wait per collective over the steps run with `timing` on: the row gather,
        then each gradient bucket (its bytes, the slice of G32 it covers)."""
        torch.cuda.synchronize()
        if not self._ev:
            return None
        waits = np.array([[a.elapsed_time(b) * 1e3 for a, b in evs] for evs in self._ev]).mean(0)
        e = self.eng
        return {"world_size": self.world, "steps": len(self._ev),
                "embedding_rows_gather": {"bytes": int(self.world * e.T * (e.D * 4 + 8)),
                                          "exposed_wait_us": round(float(waits[0]), 1)},
                "buckets": [{"start": int(a), "stop": int(b), "bytes": int(4 * (b - a)),
                             "exposed_wait_us": round(float(w), 1)} for (_, a, b), w in zip(self.buckets, waits[1:])],
                "exposed_wait_us_total": round(float(waits.sum()), 1)}
