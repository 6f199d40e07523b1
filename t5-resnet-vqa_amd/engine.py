"""VQAEngine: the MI355X training step of `ResnetVQAModel` as an explicit,
statically planned schedule of libvqa_hip kernel calls.

Mirrors, op for op:
  forward   ResnetVQAModel.forward            model/resnet_vqa_model.py:101-165
            SGA.forward                        model/multi_head_vision_text_attn.py:145-158
            T5Stack (encoder, eval)            TF/models/t5/modeling_t5.py:640-751
  backward  loss.backward()                    trainer/faster_rcnn_vqa_trainer.py:397
  step      clip_grad_norm_ + AdamW + sched    trainer/faster_rcnn_vqa_trainer.py:399-404

Design (MI355X-first, not a translation of eager PyTorch):
  * every trainable parameter, gradient and AdamW state lives in one flat fp32
    arena (layout.ParamLayout) + a bf16 shadow for GEMM operands, so the clip
    norm and AdamW are single HBM passes and DP all-reduces one contiguous
    buffer;
  * the frozen ResNet is BN-folded, bf16, NHWC, run as implicit-GEMM convs
    (no im2col buffers); the ConvTranspose2d scaler is an implicit GEMM over
    the layer4 map whose rows are already the [B, HW, 768] token order the
    reference obtains with view+permute (:142-143);
  * activations/workspaces are allocated once for a fixed (B, L, H), every
    kernel call is prepared once with fixed device addresses, and the whole
    step is replayed as one hipGraph (torch.cuda.CUDAGraph capture);
  * dropout (p = 0.1 at the reference's 12 sites per step) is
    applied inside the producing kernels from a stateless counter hash
    (include/vqa_hip.h "dropout"); the backward regenerates the masks, nothing
    is stored.  dropout=0 gives eval-mode numerics (golden-vector parity).
"""
from __future__ import annotations

import contextlib
import ctypes
import gc
import os
import math

import numpy as np
import torch

from . import lib as L
from . import ops
from . import synthetic as S
from .layout import ParamLayout, fold_bn, t5_bucket_map

BF16, F32, I64 = torch.bfloat16, torch.float32, torch.int64

# dropout site ids (the hash key of each nn.Dropout application of the step)
SITE_EMBED, SITE_FINAL = 1, 2                  # T5Stack: dropout(inputs_embeds) :725, dropout(final_ln) :745


def t5_site(layer, kind):
    """kind 0 attention probs (:168), 1 attention residual branch (:400), 2 FF inner (:86), 3 FF residual (:140)"""
    return 16 + 4 * layer + kind


def sga_site(block, kind):
    """kind 0 mhatt1 probs, 1 dropout1, 2 mhatt2 probs, 3 dropout2, 4 MLP inner, 5 dropout3
    (multi_head_vision_text_attn.py:84, 146, 84, 150, 99, 154)"""
    return 128 + 8 * block + kind


def stem_s2d_weight(wf):
    """The 7x7 stride-2 stem conv weight [Cout, 7, 7, 3] (NHWC order) as the 4x4 stride-1
    weight [Cout, 4, 4, 16] over vqa_image_to_s2d16's image:
    W'[o, a, e, (2p+q)*3 + c] = W[o, 2a+p, 2e+q, c], zero where 2a+p or 2e+q is 7."""
    co, kh, kw, ci = wf.shape
    w8 = np.zeros((co, 8, 8, ci), np.float32)
    w8[:, :kh, :kw] = wf
    w = w8.reshape(co, 4, 2, 4, 2, ci).transpose(0, 1, 3, 2, 4, 5).reshape(co, 4, 4, 4 * ci)
    return np.concatenate([w, np.zeros((co, 4, 4, 16 - 4 * ci), np.float32)], 3)


_TUNE_CACHE = {}
_TUNE_CACHE_COLD = {}            # autotune(cold=True): choices timed from cold caches
SPLITS = (1, 2, 3, 4, 6, 8)        # split-K counts the tuner tries for small grids


def lib_gemm_configs():
    import re
    return int(re.search(r"#define VQA_GEMM_CONFIGS (\d+)", open(L.HEADER).read()).group(1))


def _gemm_key(d):
    geo = lambda g: (g.n, g.h, g.w, g.c, g.oh, g.ow, g.kh, g.kw, g.stride, g.pad)
    return (d.m, d.n, d.k, d.batch, d.a_trans, d.b_trans, d.a_conv, d.b_conv,
            geo(d.ga) if d.a_conv else None, geo(d.gb) if d.b_conv else None,
            bool(d.c32), bool(d.c16), bool(d.bias), bool(d.res32), bool(d.res16), bool(d.mask16), d.relu,
            d.beta != 0.0, d.drop.p > 0.0) + (("fp8",) if d.fp8 else ())


class _Seq:
    """Several prepared calls issued as one (a deferred AdamW range and the e4m3 weight
    copies that follow it)."""
    def __init__(self, calls):
        self.calls = calls

    def __call__(self, stream):
        for c in self.calls:
            c(stream)


@contextlib.contextmanager
def no_gc_capture():
    """Stream capture with the cyclic garbage collector held off.  Engines (and the graphs /
    tensors they own) are reclaimed through reference cycles; a collection that lands inside
    a capture destroys another engine's graph execs and frees its blocks while the capture
    is being recorded (measured: the later replay of the captured graph crashed in the
    runtime).  Collect first, then keep the collector off until the capture has ended."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


_WARNED_ATTN = set()


def _check_attn_path(d, fn):
    """Say it loudly (once per shape) when a planned attention call would run the scalar VALU
    kernel (include/vqa_hip.h vqa_attn_path): it is correct but an order of magnitude slower
    than the MFMA kernels, which cover lq <= 32, lk <= 160 (key mask: lk <= 64)."""
    path = L.load().vqa_attn_path(ctypes.byref(d), int(fn == "vqa_attn_bwd"))
    if path == L.ATTN_VALU:
        key = (fn, d.lq, d.lk, d.dh, bool(d.key_mask))
        if key not in _WARNED_ATTN:
            _WARNED_ATTN.add(key)
            import warnings
            warnings.warn(f"{fn}: lq={d.lq} lk={d.lk} dh={d.dh} key_mask={bool(d.key_mask)} runs the scalar VALU "
                          "attention kernel (no MFMA kernel covers this shape)", RuntimeWarning, stacklevel=3)
    return path


def _h2d(dst, src):
    """dst <- src (numpy / torch, host or device).  Asynchronous only from device or pinned
    memory: an async copy out of a pageable temporary (freed when this returns) may be read
    by the runtime after the free."""
    src = torch.as_tensor(src).to(dst.dtype).reshape(dst.shape)
    dst.copy_(src, non_blocking=src.is_cuda or src.is_pinned())


IGNORE_INDEX = -100          # nn.NLLLoss's default ignore_index: the head skips rows with a target < 0


def batch_rows(batch, key, planned, allow_empty=False):
    """Rows of a collate batch (the reference's loaders have no drop_last, so an epoch's last
    batch is short: faster_rcnn_vqa_trainer.py:172-197); 1 <= rows <= the planned batch (0 rows
    only for a data-parallel rank whose share of the global batch is empty: allow_empty)."""
    n = int(torch.as_tensor(batch[key]).shape[0])
    if not (0 if allow_empty else 1) <= n <= planned:
        lo = 0 if allow_empty else 1
        raise ValueError(f"{key}: batch of {n} rows; this engine is planned for {lo}..{planned} rows")
    return n


def load_rows(dst, src, n, fill=None, empty_fill=0):
    """dst[:n] <- src (n rows); the planned rows past n are padding: copies of rows 0..n-1
    (real samples, so every activation stays finite) or `fill` (targets: IGNORE_INDEX, so the
    padded rows add nothing to the loss or to any gradient -- the NLL mean runs over the n
    real rows).  n = 0 (an empty data-parallel rank): every row is `fill`, else `empty_fill`
    (finite inputs whose targets are all ignored: the rank's gradient is exactly zero)."""
    if src is None:
        return
    B = dst.shape[0]
    if n == 0:
        dst.fill_(fill if fill is not None else empty_fill)
        return
    _h2d(dst[:n] if n < B else dst, src)
    if n == B:
        return
    if fill is not None:
        dst[n:].fill_(fill)
        return
    i = n
    while i < B:                                   # doubling copies of the real rows
        k = min(i, B - i)
        dst[i:i + k].copy_(dst[:k])
        i += k


class VQAEngine:
    def __init__(self, state_dict, vision="resnet50", batch=64, seq_len=32, image_size=224, device="cuda:0",
                 warmup=10, total=100, num_blocks=3, answer_spaces=170, grad_scale=1.0, max_norm=1.0,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1, dropout=0.1, seed=0, pipeline=False,
                 t5_dw_group=None, defer_optimizer=True, dw_stream=None, sga_dw_batch=True, pair_bwd=True,
                 language_model="t5-base", fp8=False, sga_attn_group=True):
        L.load()
        # pipeline: the frozen ResNet (no trainable input) of the NEXT batch runs on its own
        # stream beside this step's T5 / SGA / backward / optimizer (see train_step)
        self.pipeline = bool(pipeline)
        self.p_drop, self.seed = float(dropout), int(seed)
        self.dev = torch.device(device)
        self.vision, self.B, self.L, self.H = vision, batch, seq_len, image_size
        assert image_size % 2 == 0, "the space-to-depth stem needs an even image size"
        self.NB, self.A = num_blocks, answer_spaces
        # widths: t5-base (the reference) or t5-large (BASELINE configs[4]: the SGA blocks, scaler,
        # pooler and classifier at the language model's width, synthetic.LM_DIMS)
        self.dims = dm = S.lm_dims(language_model)
        self.D, self.nl, self.h5, self.dkv, self.dff = dm.d_model, dm.t5_layers, dm.t5_heads, dm.t5_dkv, dm.t5_dff
        self.sga_heads, self.sga_dh = dm.sga_heads, dm.sga_dhead
        assert self.h5 * self.dkv == self.D and self.sga_heads * self.sga_dh == self.D
        # fp8: the forward weight GEMMs of the T5 layers and SGA blocks on e4m3 operands (BASELINE
        # configs[4] "fp8 MFMA weights"): weights and their input activations quantised row-wise
        # (vqa_quant_rows_fp8), the backward on the bf16 shadows / saved bf16 activations
        self.fp8 = bool(fp8)
        # the answer head's log-softmax keeps one sample's answer logits in registers (head.hip:
        # A <= 1024; DAQUAR has 170) and the pooler one sample's tokens (L <= 64)
        if not 1 <= answer_spaces <= 1024:
            raise ValueError(f"answer_spaces={answer_spaces}: the fused answer head supports 1..1024 answers")
        if not 1 <= seq_len <= 64:
            raise ValueError(f"seq_len={seq_len}: the attention / pooler kernels support 1..64 question tokens")
        self.warmup, self.total, self.max_norm = warmup, total, max_norm
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.grad_scale = grad_scale
        self.group_lr = {}                # per-group LR overrides (trainer optimizer_kwargs)
        # dX + dW of a layer as one paired GEMM launch (pair_bwd=False: separate launches)
        self.pair_bwd = bool(pair_bwd)
        # T5 weight gradients: per weight ONE launch batched over a group of layers (the
        # layers' activations / gradients stacked at constant strides).  `t5_dw_group` is a
        # group size (1: dX + dW paired per layer; 12: one group) or a sequence of group sizes,
        # top layer first.  Default (single GPU): groups of 9 and 3 layers (3/4 and 1/4 of the
        # stack: 18 and 6 for t5-large), the batched weight
        # gradients on a side stream beside the remaining input-gradient chain (measured 6.66 vs
        # 6.78-6.84 ms per step against one group of 12 on the chain; tools/gpu/ab_env.sh).
        # DP passes (4, 4, 3, 1): the buckets become final, and are all-reduced, while the
        # backward runs, and the last, exposed bucket is one layer.
        if t5_dw_group is None:
            t5_dw_group = (3 * self.nl // 4, self.nl - 3 * self.nl // 4)
        if isinstance(t5_dw_group, (list, tuple)):
            self.t5_dw_groups = [int(x) for x in t5_dw_group]
            self.t5_dw_group = self.nl
            assert sum(self.t5_dw_groups) == self.nl and min(self.t5_dw_groups) >= 1
        else:
            self.t5_dw_groups = None
            self.t5_dw_group = int(t5_dw_group)
        # SGA blocks' q2 / m2 / fc1 / fc2 weight gradients batched over the blocks
        self.sga_dw_batch = bool(sga_dw_batch)
        # the SGA blocks' self-attentions as ONE launch forward and ONE backward
        # (vqa_attn_desc.groups; False: one launch per block)
        self.sga_attn_group = bool(sga_attn_group)
        # AdamW of step k applied inside step k+1's forward (see _plan_optimizer)
        self.defer_opt = bool(defer_optimizer)
        # weight-gradient GEMMs (calls tagged `side`) on a stream of their own beside the
        # input-gradient chain (single GPU and DP alike; dp.DataParallelStep keeps the placement)
        self.dw_stream = True if dw_stream is None else bool(dw_stream)
        self.T = batch * seq_len
        self.rows = batch                 # real rows of the loaded batch (a short last batch is padded)
        self.lay = ParamLayout(vision, answer_spaces, num_blocks, dm)
        sd = {k: np.asarray(v) for k, v in state_dict.items()}
        self._frozen = {k: v for k, v in sd.items() if k not in set(self.lay.trainable_keys)}
        with torch.cuda.device(self.dev):
            self._alloc_params(sd)
            self._plan_resnet(sd)
            self._alloc_activations()
            self.fwd_calls, self.bwd_calls, self.opt_calls, self.zero_calls = [], [], [], []
            self._plan_forward()
            self._plan_backward()
            self._plan_optimizer()
            self._run(self.quant_all)                     # e4m3 weights of the initial parameters
        self.graph = None
        self.allreduce = None            # set by the DP trainer: fn(G32 tensor) on the current stream
        self._side = torch.cuda.Stream(self.dev)
        self._wside = torch.cuda.Stream(self.dev)
        self._rstream = torch.cuda.Stream(self.dev)
        self.res_external = False        # set_res_cumask: the ResNet launched eagerly beside the graph
        self.allow_empty_rows = False     # use_global_rows (DP): a rank may get 0 rows
        self._img_rows_next = None        # pipelined: rows of the images whose features the next batch uses
        self.count_call = None
        self._scratch = None             # split-K workspace used while autotuning

    @classmethod
    def from_state_dict(cls, sd, **kw):
        return cls(sd, **kw)

    # ------------------------------------------------------------------ allocation
    def _t(self, shape, dtype=F32, zero=False):
        f = torch.zeros if zero else torch.empty
        return f(shape, dtype=dtype, device=self.dev)

    def _alloc_params(self, sd):
        lay = self.lay
        flat = lay.pack(sd)
        self.P32 = torch.from_numpy(flat).to(self.dev)
        self.P16 = self.P32.to(BF16)
        self.G32 = self._t(lay.total, zero=True)
        if self.fp8:
            # e4m3 weight shadow and its row scales, at the fp32 arena's element offsets: row r of
            # segment s is W8[s.offset + r*K :] with scale WSC[s.offset + r] (constant strides
            # between the blocks' segments, as the batched launches need)
            self.W8 = torch.empty(lay.total, dtype=torch.uint8, device=self.dev)
            self.WSC = torch.ones(lay.total, dtype=F32, device=self.dev)
            self._xq = {}
        self.M = self._t(lay.total, zero=True)
        self.V = self._t(lay.total, zero=True)
        self.VMAX = self._t(lay.total, zero=True)
        self.p32, self.p16, self.g32 = {}, {}, {}
        for s in lay.segments.values():
            sl = slice(s.offset, s.offset + s.numel)
            self.p32[s.name] = self.P32[sl].view(s.shape)
            self.p16[s.name] = self.P16[sl].view(s.shape)
            self.g32[s.name] = self.G32[sl].view(s.shape)
        self.opt_state = self._t(L.ST_FLOATS, zero=True)
        # dropout RNG state {seed, counter, training}; the forward's first call advances the counter
        self.RNG = torch.from_numpy(np.array([self.seed & 0xFFFFFFFF, 0, 1, 0], np.uint32).view(np.int32)).to(self.dev)
        self.bucket = torch.from_numpy(t5_bucket_map(self.L, self.L)).reshape(-1).to(self.dev)

    def _plan_resnet(self, sd):
        """Frozen torchvision ResNet (eval BN folded) as a list of implicit-GEMM convs."""
        B, H = self.B, self.H
        vm = "vision_model."
        self.res_calls = []
        self._res_keep = []
        convs = []                                   # (name_conv, name_bn, stride, pad, relu, role)

        def conv_w(cname, bname, s2d=False):
            w = sd[vm + cname + ".weight"].astype(np.float32)
            wf, bf = fold_bn(w, sd[vm + bname + ".weight"], sd[vm + bname + ".bias"],
                             sd[vm + bname + ".running_mean"], sd[vm + bname + ".running_var"])
            wf = wf.transpose(0, 2, 3, 1)            # [Cout, kh, kw, Cin]
            if s2d:
                wf = stem_s2d_weight(wf)
            w16 = torch.from_numpy(np.ascontiguousarray(wf)).to(self.dev).to(BF16)
            b32 = torch.from_numpy(bf).to(self.dev)
            self._res_keep += [w16, b32]
            return w16, b32

        # geometry walk to size the ping-pong buffers
        layers = S.RESNET_LAYERS[self.vision]
        bottleneck = self.vision == "resnet50"
        h1 = (H + 2 * 3 - 7) // 2 + 1
        h2 = (h1 + 2 - 3) // 2 + 1
        plan = []                                     # (kind, args)
        maxel = B * h1 * h1 * 64
        hh, cin = h2, 64
        for li, (planes, nblk) in enumerate(zip((64, 128, 256, 512), layers)):
            for bi in range(nblk):
                stride = (1 if li == 0 else 2) if bi == 0 else 1
                out = planes * 4 if bottleneck else planes
                ho = (hh + 2 - 3) // stride + 1
                maxel = max(maxel, B * hh * hh * planes, B * ho * ho * out)
                if bottleneck and bi == 0:            # the fused conv3 + downsample's [conv2 | x] rows
                    maxel = max(maxel, B * ho * ho * (planes + cin))
                plan.append((li, bi, stride, hh, ho, cin, planes, out))
                hh, cin = ho, out
        self.fh, self.fc = hh, cin                    # layer4 spatial size / channels
        self.V_TOK = B * hh * hh
        self.IMG = self._t((B, 3, H, H))
        hz = H // 2 + 1                               # space-to-depth stem image (vqa_image_to_s2d16)
        bufs = [self._t(maxel, BF16) for _ in range(5)]
        self.res_bufs = bufs
        self.F4 = self._t((B, hh, hh, cin), BF16)
        # pipelined: the ResNet writes the next batch's layer4 map here; each step first
        # moves it into F4 (read by the ConvTranspose2d forward and weight gradient)
        self.F4N = self._t((B, hh, hh, cin), BF16) if self.pipeline else self.F4
        # F4 <- F4N as a library kernel (a torch copy_ would put a runtime memcpy node in the graph)
        self.copy_f4 = ops.Call("vqa_copy", self.F4.data_ptr(), self.F4N.data_ptr(), self.F4.numel() * 2,
                                keep=(self.F4, self.F4N))

        # stem: conv7x7/2 + BN + ReLU, then maxpool 3x3/2
        # (as a 4x4 stride-1 conv over the space-to-depth image: K 256 instead of 7*7*8 = 392)
        w16, b32 = conv_w("conv1", "bn1", s2d=True)
        g = ops.conv_geom(B, hz, hz, 16, h1, h1, 4, 4, 1, 1)
        stem = os.environ.get("VQA_STEM", "img")            # img | pool | patch | gemm (A/B switches)
        fused_img = stem == "img" and H % 32 == 0 and hz == h1 + 1 and h2 == h1 // 2
        # the space-to-depth image only exists for the forms that read it (B x 113 x 113 x 16 bf16)
        self.IMG8 = None if fused_img else self._t((B, hz, hz, 16), BF16)
        if fused_img:
            # space-to-depth + stem + maxpool in one pass (csrc/stem.hip): patches staged from the
            # fp32 image, only the pooled map written; bit-identical to the three-kernel form below
            self.res_calls.append(ops.Call("vqa_stem_pool_img", self.IMG.data_ptr(), w16.data_ptr(), b32.data_ptr(),
                                           bufs[1].data_ptr(), B, H, keep=(self.IMG, w16, b32, bufs[1])))
            stem = None
        else:
            self.res_calls.append(ops.Call("vqa_image_to_s2d16", self.IMG.data_ptr(), self.IMG8.data_ptr(), B, H, H,
                                           keep=(self.IMG, self.IMG8)))
        if stem is None:
            pass
        elif stem in ("img", "pool") and h1 % 16 == 0 and hz == h1 + 1 and h2 == h1 // 2:
            # stem + maxpool in one pass from LDS input patches (csrc/stem.hip): only the pooled
            # map is written; bit-identical to the implicit GEMM + vqa_maxpool3x3s2_nhwc below
            self.res_calls.append(ops.Call("vqa_stem_pool_s2d", self.IMG8.data_ptr(), w16.data_ptr(), b32.data_ptr(),
                                           bufs[1].data_ptr(), B, hz, h1, keep=(self.IMG8, w16, b32, bufs[1])))
        else:
            if stem in ("pool", "patch") and h1 % 16 == 0 and hz == h1 + 1:
                self.res_calls.append(ops.Call("vqa_stem_s2d_conv", self.IMG8.data_ptr(), w16.data_ptr(),
                                               b32.data_ptr(), bufs[0].data_ptr(), B, hz, h1,
                                               keep=(self.IMG8, w16, b32, bufs[0])))
            else:
                self._gemm(self.res_calls, self.IMG8, w16, B * h1 * h1, 64, 256, lda=256, ldb=256, ga=g,
                           c16=bufs[0], ldc16=64, bias=b32, relu=True)
            self.res_calls.append(ops.Call("vqa_maxpool3x3s2_nhwc", bufs[0].data_ptr(), bufs[1].data_ptr(), B, h1,
                                           h1, 64, h2, h2, keep=(bufs[0], bufs[1])))
        x = bufs[1]
        free = [bufs[0], bufs[2], bufs[3], bufs[4]]
        nblocks_total = len(plan)
        for idx, (li, bi, stride, hi, ho, ci, planes, out) in enumerate(plan):
            p = f"layer{li + 1}.{bi}."
            t1, t2, ds, y = free[0], free[1], free[2], free[3]
            if idx == nblocks_total - 1:
                y = self.F4N
            fuse = bottleneck and (vm + p + "downsample.0.weight") in sd and os.environ.get("VQA_RES_FUSE_DS", "1") != "0"
            if fuse:
                # conv3 and the 1x1 downsample as ONE GEMM over the concatenated K (r05):
                # [conv2 out | x subsampled] . [W3 | Wd]^T + (b3 + bd), ReLU -- conv2 writes the
                # first `planes` columns of the `ds` buffer, vqa_subsample_nhwc the other `ci`;
                # the downsample's output never goes to HBM and one launch goes away
                kc = planes + ci
                w, b = conv_w(p + "conv1", p + "bn1")
                self._conv(x, (B, hi, hi, ci), w, b, 1, 0, t1, relu=True)
                w, b = conv_w(p + "conv2", p + "bn2")
                self._conv(t1, (B, hi, hi, planes), w, b, stride, 1, ds, relu=True, ldc16=kc)
                self.res_calls.append(ops.Call("vqa_subsample_nhwc", x.data_ptr(), B, hi, hi, ci, stride,
                                               ops.addr(ds, planes), kc, keep=(x, ds)))
                w3, b3 = conv_w(p + "conv3", p + "bn3")
                wd, bd = conv_w(p + "downsample.0", p + "downsample.1")
                wcat = torch.cat([w3.reshape(out, planes), wd.reshape(out, ci)], dim=1).contiguous()
                bcat = b3 + bd
                self._res_keep += [wcat, bcat]
                assert B * ho * ho * kc <= ds.numel(), "fused downsample: the [conv2 | x] rows exceed the buffer"
                self._gemm(self.res_calls, ds, wcat, B * ho * ho, out, kc, lda=kc, ldb=kc, c16=y, ldc16=out,
                           bias=bcat, relu=True)
                if y is not self.F4N:
                    free = [x, t1, t2, ds]
                    x = y
                continue
            if bottleneck:
                w, b = conv_w(p + "conv1", p + "bn1")
                self._conv(x, (B, hi, hi, ci), w, b, 1, 0, t1, relu=True)
                w, b = conv_w(p + "conv2", p + "bn2")
                self._conv(t1, (B, hi, hi, planes), w, b, stride, 1, t2, relu=True)
                last_in, last_c, last_h = t2, planes, ho
                w3, b3 = conv_w(p + "conv3", p + "bn3")
            else:
                w, b = conv_w(p + "conv1", p + "bn1")
                self._conv(x, (B, hi, hi, ci), w, b, stride, 1, t1, relu=True)
                last_in, last_c, last_h = t1, planes, ho
                w3, b3 = conv_w(p + "conv2", p + "bn2")
            res = x
            if (vm + p + "downsample.0.weight") in sd:
                w, b = conv_w(p + "downsample.0", p + "downsample.1")
                self._conv(x, (B, hi, hi, ci), w, b, stride, 0, ds, relu=False)
                res = ds
            k3 = 1 if bottleneck else 3
            self._conv(last_in, (B, last_h, last_h, last_c), w3, b3, 1, 1 if k3 == 3 else 0, y, relu=True,
                       res16=res)
            if y is not self.F4N:
                free = [x, t1, t2, ds]
                x = y

    def _conv(self, x, shape, w16, b32, stride, pad, out, relu, res16=None, ldc16=None):
        n, h, w, c = shape
        cout, kh, kw, _ = w16.shape
        oh = (h + 2 * pad - kh) // stride + 1
        g = ops.conv_geom(n, h, w, c, oh, oh, kh, kw, stride, pad)
        if kh == 1 and kw == 1 and stride == 1 and pad == 0:
            g = None                                   # a 1x1/1 conv is a plain GEMM over the NHWC rows
        # 3x3 / stride 1: the LDS-patch convolution (a_conv = 2), weights reordered to
        # [Cout][C/64][9][64]; any W <= 64 has a patch tile that fits (conv_patch.inl patch_fits)
        patch = kh == 3 and kw == 3 and stride == 1 and pad == 1 and c % 64 == 0 and 14 <= w <= 64
        if patch:
            w16 = w16.reshape(cout, 9, c // 64, 64).permute(0, 2, 1, 3).contiguous().reshape(cout, kh, kw, c)
            self._res_keep.append(w16)
        self._gemm(self.res_calls, x, w16, n * oh * oh, cout, kh * kw * c, lda=kh * kw * c, ldb=kh * kw * c, ga=g,
                   c16=out, ldc16=ldc16 or cout, bias=b32, relu=relu, res16=res16, ldres=cout, a_patch=patch)

    def _alloc_activations(self):
        D = self.D
        B, Lq, T, NB, V = self.B, self.L, self.T, self.NB, self.V_TOK
        t = self._t
        # inputs
        self.IDS = t((B, Lq), I64, zero=True)
        self.IDS_PREV = t((B, Lq), I64, zero=True)     # ids whose embedding-gradient rows are nonzero
        self.MASK = t((B, Lq), I64, zero=True)
        self.TGT = t((B,), I64, zero=True)
        # vision tokens
        self.VIS32, self.VIS16 = t((V, D)), t((V, D), BF16)
        # T5
        nl = self.nl
        self.PB = t((self.h5, Lq, Lq))
        self.HS = [t((T, D)) for _ in range(nl + 1)]
        # GEMM inputs the weight gradients read, stacked in backward order (slot = 11 - layer) so
        # a group of consecutive layers' dW is one batched launch with constant strides
        self.N0S, self.OS, self.N1S = t((nl, T, D), BF16), t((nl, T, D), BF16), t((nl, T, D), BF16)
        self.FFS = t((nl, T, self.dff), BF16)
        self.N0 = [self.N0S[nl - 1 - i] for i in range(nl)]
        self.QKV = [t((T, 3 * D), BF16) for _ in range(nl)]
        self.PT = [t((B, self.h5, Lq, Lq)) for _ in range(nl)]
        self.O = [self.OS[nl - 1 - i] for i in range(nl)]
        self.HM = [t((T, D)) for _ in range(nl)]
        self.N1 = [self.N1S[nl - 1 - i] for i in range(nl)]
        self.FF = [self.FFS[nl - 1 - i] for i in range(nl)]
        self.R0 = [t(T) for _ in range(nl)]
        self.R1 = [t(T) for _ in range(nl)]
        self.RF = t(T)
        self.TXT32, self.TXT16 = t((T, D)), t((T, D), BF16)
        # SGA blocks; the self-attention halves of all blocks share batched buffers:
        # q|k|v of block n in columns [n*2304, (n+1)*2304) of QKV1A, merge in/out in [n]
        self.QKV1A = t((T, NB * 3 * D), BF16)
        self.O1A, self.S1A = t((NB, T, D), BF16), t((NB, T, D))
        self.P1A = t((NB, B, self.sga_heads, Lq, Lq))         # their attention probabilities, stacked
        # inputs of the blocks' q2 / m2 / fc1 / fc2 weight gradients, stacked in backward order
        # (slot NB-1-n) for the batched dW launches
        self.X1hS, self.O2S, self.X2hS, self.FFhS = (t((NB, T, D), BF16) for _ in range(4))
        self.Q2S = t((NB, T, D), BF16)                 # the blocks' cross-attention queries (one batched GEMM)
        self.sga = []
        for n in range(NB):
            ly = V if n == 0 else T
            lk = self.fh * self.fh if n == 0 else Lq
            self.sga.append(dict(
                ly=ly, lk=lk,
                P1=self.P1A[n], O1=self.O1A[n], S1=self.S1A[n],
                X1=t((T, D)), X1h=self.X1hS[NB - 1 - n], MU1=t(T), RS1=t(T),
                Q2=self.Q2S[NB - 1 - n], KV2=t((ly, 2 * D), BF16), P2=t((B, self.sga_heads, Lq, lk)),
                O2=self.O2S[NB - 1 - n], S2=t((T, D)), X2=t((T, D)), X2h=self.X2hS[NB - 1 - n], MU2=t(T), RS2=t(T),
                FFh=self.FFhS[NB - 1 - n], S3=t((T, D)), OUT=t((T, D)), OUTh=t((T, D), BF16), MU3=t(T), RS3=t(T)))
        # head
        self.ATT, self.POOLED = t((B, Lq)), t((B, D))
        self.LOGP, self.NLL, self.LOSS = t((B, self.A)), t(B), t(1)
        self.ROWTOT = t(1, zero=True)     # DP: valid rows summed over the ranks (use_global_rows)
        # backward temporaries (reused layer to layer)
        mx = max(T, V)
        self.dY = [t((T, D)), t((T, D))]
        self.dA32 = t((T, D))
        self._gbufs = {}
        self.dC32 = t((T, D))
        self.dTA = [t((T, D)), t((T, D))]              # running text gradient of the SGA norm1s (ping-pong)
        self.dA1A, self.dO1A = t((NB, T, D), BF16), t((NB, T, D), BF16)
        self.dQKV1A = t((T, NB * 3 * D), BF16)
        self.dO16 = t((T, D), BF16)
        self.dTXT = t((T, D))
        self.dVIS32, self.dVIS16 = t((V, D)), t((V, D), BF16)
        self.dVIS9 = t((9, V, D), BF16)                 # its 3x3 tap-shifted copies (scaler dW)
        self.dH32 = t((T, D))
        self.dHM32 = t((T, D))
        self.dPB = t((self.h5, Lq, Lq), zero=True)
        self.dSB = t((self.nl, B, self.h5, Lq, Lq))   # per-layer, per-sample attention dS (rel-bias grad)
        self.WS_EMB = t(3 * T, torch.int32)
        lib = L.load()
        self.WS_COL2 = t(lib.vqa_colsum_workspace_floats(V, D))
        self.WS_HEAD = t(lib.vqa_head_workspace_floats(B, Lq, D, self.A))
        self.SQ_PARTS = 1024                              # per sqnorm range (three ranges, §3.7)
        self.WS_SQ = t(3 * self.SQ_PARTS, torch.float64)

    # ------------------------------------------------------------------ call helpers
    # Every helper records the tensors it bakes into a call (ops.Call.keep), so no
    # buffer can be freed while a prepared call still points at it.  Raw int
    # addresses (sub-views made with ops.addr) must come from tensors that are
    # passed too or are engine attributes.
    def _gemm(self, lst, a, b, m, n, k, keep=(), **kw):
        ts = [a, b] + [v for v in kw.values() if isinstance(v, torch.Tensor)] + list(keep)
        lst.append(ops.gemm_call(ops.gemm_desc(a, b, m, n, k, **kw), [t for t in ts if isinstance(t, torch.Tensor)]))

    def _sga_self_keep(self):
        """The flat-arena views the batched SGA self-attention launches read past: the
        blocks' q|k|v and merge weights, biases and gradients sit side by side (layout.py)."""
        names = [f"sga{n}.{w}" for w in ("qkv1_w", "qkv1_b", "m1_w", "m1_b") for n in range(self.NB)]
        for w in ("qkv1_w", "qkv1_b", "m1_w", "m1_b"):
            segs = [self.lay[f"sga{n}.{w}"] for n in range(self.NB)]
            assert all(b.offset == a.offset + a.numel for a, b in zip(segs, segs[1:])), w
        return tuple(self.p16[k] for k in names if k in self.p16) + tuple(self.p32[k] for k in names) + \
            tuple(self.g32[k] for k in names)

    def _sga_groups(self):
        """vqa_attn_desc group fields of the SGA blocks' self-attentions: all NB blocks in one
        launch (block n: q|k|v columns n*2304 of QKV1A, O1A[n] / dO1A[n], P1A[n], dropout site
        sga_site(n, 0)), or one block per launch (sga_attn_group=False)."""
        T, D = self.B * self.L, self.D
        if not self.sga_attn_group or self.NB == 1:
            return dict(groups=1)
        return dict(groups=self.NB, gstride_qkv=3 * D, gstride_o=T * D, gstride_dout=T * D,
                    gstride_p=self.P1A[0].numel(), gdrop_site_stride=sga_site(1, 0) - sga_site(0, 0))

    def _set_drop(self, call, site):
        d = self._drop(site)
        if d is not None:
            call.desc.drop = d
            call.keep = call.keep + (self.RNG,)

    def _call(self, lst, name, *args, extra=()):
        ts = tuple(a for a in args if isinstance(a, torch.Tensor)) + tuple(extra)
        lst.append(ops.Call(name, *[ops.addr(a) if isinstance(a, torch.Tensor) else a for a in args], keep=ts))

    def _attn(self, lst, fn, drop=None, keep=(), **kw):
        d = L.AttnDesc()
        for k, v in kw.items():
            setattr(d, k, ops.addr(v) if isinstance(v, torch.Tensor) else v)
        ts = tuple(v for v in kw.values() if isinstance(v, torch.Tensor)) + tuple(keep)
        dd = self._drop(drop) if drop is not None else None
        if dd is not None:
            d.drop = dd
            ts = ts + (self.RNG,)
        _check_attn_path(d, fn)
        lst.append(ops.Call(fn, ctypes.byref(d), keep=ts, desc=d))

    def _drop(self, site):
        """vqa_dropout for `site` (None when dropout is off)."""
        if self.p_drop <= 0.0:
            return None
        return L.Dropout(self.p_drop, site, self.RNG.data_ptr())

    def _dptr(self, site, keep):
        """`const vqa_dropout*` argument (0 = none); the struct is kept alive through `keep`."""
        d = self._drop(site)
        if d is None:
            return None
        keep.append(d)
        return ctypes.addressof(d)

    @property
    def drop_scale(self):
        """1/(1-p) in fp32, the multiplier of a kept element (as the kernels compute it)."""
        p = np.float32(self.p_drop)
        return float(np.float32(1.0) / (np.float32(1.0) - p))

    # ------------------------------------------------------------------ fp8 (config 5)
    FP8_T5 = ("qkv_w", "o_w", "wi", "wo")
    FP8_SGA = ("qkv1_w", "m1_w", "q2_w", "kv2_w", "m2_w", "fc1_w", "fc2_w")

    def _is_fp8(self, wname):
        return self.fp8 and wname.rsplit(".", 1)[-1] in (self.FP8_T5 + self.FP8_SGA)

    def _w8(self, wname):
        """(e4m3 weight view [n, k], its row scales [n]) of segment `wname` in the fp8 arenas."""
        sg = self.lay[wname]
        n, k = sg.shape
        return self.W8[sg.offset:sg.offset + n * k].view(n, k), self.WSC[sg.offset:sg.offset + n]

    def _quant_weight(self, lst, wname, rows=None):
        """Row-wise e4m3 copy of weight `wname` (its fp32 master, `rows` rows from its offset:
        several side-by-side segments quantised as one matrix)."""
        sg = self.lay[wname]
        k = sg.shape[1]
        rows = sg.shape[0] if rows is None else rows
        self._call(lst, "vqa_quant_rows_fp8", ops.addr(self.P32, sg.offset), 0, k, rows, k, ops.addr(self.W8, sg.offset),
                   k, ops.addr(self.WSC, sg.offset), extra=(self.P32, self.W8, self.WSC))

    def _quant_act(self, lst, key, x16, rows):
        """e4m3 copy (+ row scales) of a bf16 GEMM input, into a buffer private to call site `key`."""
        k = x16.shape[-1]
        if key not in self._xq:
            self._xq[key] = (torch.empty(rows, k, dtype=torch.uint8, device=self.dev), self._t(rows))
        x8, xs = self._xq[key]
        self._call(lst, "vqa_quant_rows_fp8", x16, 1, k, rows, k, x8, k, xs)
        return x8, xs

    def _linear(self, lst, x16, wname, m, out32=None, out16=None, bias=True, relu=False, res32=None, drop=None):
        if getattr(self, "fp8", False) and self._is_fp8(wname):          # (borrowed by VitVQAEngine: no fp8)
            x8, xs = self._quant_act(lst, (wname, "x"), x16, m)
            w8, ws = self._w8(wname)
            n, k = w8.shape
            self._gemm(lst, x8, w8, m, n, k, lda=k, ldb=k, c32=out32, ldc32=n, c16=out16, ldc16=n,
                       bias=self.p32[wname[:-1] + "b"] if bias else None, relu=relu, res32=res32, ldres=n, fp8=True,
                       scale_a=xs, scale_b=ws, keep=(self.W8, self.WSC))
            d = self._drop(drop) if drop is not None else None
            if d is not None:
                lst[-1].desc.drop = d
                lst[-1].keep = lst[-1].keep + (self.RNG,)
            return
        w = self.p16[wname]
        n, k = w.shape
        self._gemm(lst, x16, w, m, n, k, lda=k, ldb=k, c32=out32, ldc32=n, c16=out16, ldc16=n,
                   bias=self.p32[wname[:-1] + "b"] if bias else None, relu=relu, res32=res32, ldres=n)
        d = self._drop(drop) if drop is not None else None
        if d is not None:
            lst[-1].desc.drop = d
            lst[-1].keep = lst[-1].keep + (self.RNG,)

    def _dx(self, lst, dy16, wname, m, out32=None, out16=None, res32=None, mask16=None, beta=0.0, alpha=1.0):
        """dX[m, k] = alpha * dY[m, n] W[n, k]  (+res) (*mask>0) (+beta*out32)"""
        w = self.p16[wname]
        n, k = w.shape
        self._gemm(lst, dy16, w, m, k, n, lda=n, ldb=k, b_trans=True, c32=out32, ldc32=k, c16=out16, ldc16=k,
                   res32=res32, ldres=k, mask16=mask16, ldmask=k, beta=beta, alpha=alpha)

    def _dxdw(self, lst, dy16, x16, wname, rows, bias_from=None, **dxkw):
        """A layer's input gradient and weight gradient (they share dY) as ONE paired
        launch (vqa_gemm_pair), then the bias column sum."""
        tmp = []
        self._dx(tmp, dy16, wname, rows, **dxkw)
        self._dw(tmp, dy16, x16, wname, rows, bias_from=bias_from)
        if not self.pair_bwd:
            lst.extend(tmp)
            return
        gx, gw = tmp[0], tmp[1]
        lst.append(ops.Call("vqa_gemm_pair", ctypes.byref(gx.desc), ctypes.byref(gw.desc), keep=gx.keep + gw.keep,
                            desc=(gx.desc, gw.desc)))
        lst.extend(tmp[2:])

    def _defer(self, ws, parts, stride, cols, out, beta=0.0, offset=0):
        """Queue the final reduction out = beta*out + sum_p ws[offset + p*stride + c] (a norm
        weight/bias or Linear bias gradient whose per-block partial rows a backward kernel
        wrote); _flush() finishes every queued one in a single vqa_colsum_batched launch."""
        self._jobs.append((ops.addr(ws) + 4 * offset, ops.addr(out), stride, parts, cols, beta, (ws, out)))

    def _flush(self, lst):
        if not self._jobs:
            return
        arr = (L.ColsumJob * len(self._jobs))()
        blk = 0
        keep = []
        for j, (ws, out, stride, parts, cols, beta, k) in enumerate(self._jobs):
            arr[j] = L.ColsumJob(ws, out, stride, parts, cols, beta, blk)
            blk += -(-cols // 64)
            keep += list(k)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.dev)
        lst.append(ops.Call("vqa_colsum_batched", raw.data_ptr(), len(self._jobs), blk, keep=tuple(keep) + (raw,)))
        self._jobs = []

    def _norm_ws(self):
        """A private partial-row workspace for one deferred norm backward."""
        D = self.D
        return self._t(L.load().vqa_norm_bwd_workspace_floats(self.T, D))

    def _gbuf(self, name, shape):
        """A bf16 backward buffer private to one use (see _plan_backward)."""
        if name not in self._gbufs:
            self._gbufs[name] = self._t(shape, BF16)
        return self._gbufs[name]

    def _bias_colsum(self, lst, dy16, rows, bname):
        """A Linear bias gradient = column sums of its bf16 output gradient (deferred)."""
        lib = L.load()
        n = dy16.shape[-1]
        ws = self._t(lib.vqa_colsum_workspace_floats(rows, n))
        self._call(lst, "vqa_colsum", dy16, 1, rows, n, n, None, 0.0, ws)
        self._defer(ws, lib.vqa_colsum_parts(rows), n, n, self.g32[bname])

    def _dw(self, lst, dy16, x16, wname, rows, bias_from=None, bias_bf16=True):
        """dW[n, k] = dY[rows, n]^T X[rows, k]; optional bias grad = colsum(dY).
        Tagged `side`: nothing on the dX chain reads them, so the step graph runs
        them on a third stream beside the chain (joined before the optimizer)."""
        g = self.g32[wname]
        n, k = g.shape
        self._gemm(lst, dy16, x16, n, k, rows, lda=n, ldb=k, a_trans=True, b_trans=True, c32=g, ldc32=k)
        lst[-1].side = True
        if bias_from is not None:                   # partial column sums now, final sum deferred (_flush)
            lib = L.load()
            ws = self._t(lib.vqa_colsum_workspace_floats(rows, n))
            self._call(lst, "vqa_colsum", bias_from, int(bias_bf16), rows, n, n, None, 0.0, ws)
            self._defer(ws, lib.vqa_colsum_parts(rows), n, n, self.g32[wname[:-1] + "b"])

    # ------------------------------------------------------------------ forward plan
    def _plan_forward(self):
        D = self.D
        f = self.fwd_calls
        B, Lq, T = self.B, self.L, self.T
        if self.p_drop > 0.0:                                # fresh dropout masks every step
            self._call(f, "vqa_rng_advance", self.RNG)
        self._fsplit = [len(f)]                              # [pre | vision | text | fusion]
        if not self.pipeline:                                # pipelined: res_calls run beside the step
            f += self.res_calls
        self._fvis_param = len(f)                            # first vision-branch call reading parameters
        # ConvTranspose2d scaler as implicit GEMM over the layer4 map (+bias) -> vision tokens
        cin, fh = self.fc, self.fh
        g = ops.conv_geom(B, fh, fh, cin, fh, fh, 3, 3, 1, 1)
        self._gemm(f, self.F4, self.p16["scaler_w"], self.V_TOK, D, 9 * cin, lda=9 * cin, ldb=9 * cin, ga=g,
                   c32=self.VIS32, ldc32=D, c16=self.VIS16, ldc16=D, bias=self.p32["scaler_b"])
        # SGA block 0's key/value projection reads only the vision tokens: it runs here, on the
        # vision branch beside the T5 encoder, instead of on the chain after it
        self._linear(f, self.VIS16, "sga0.kv2_w", self.sga[0]["ly"], out16=self.sga[0]["KV2"])
        self.sga_vision_calls = [f[-1]]                    # SGA work outside the fusion segment (bench)
        # T5 encoder (independent of the vision branch until the SGA blocks)
        self._fsplit.append(len(f))
        kp = []
        self._call(f, "vqa_embedding_fwd", self.IDS, self.p32["t5.embed"], self.HS[0], T, D, S.T5_VOCAB,
                   self._dptr(SITE_EMBED, kp), extra=kp + [self.RNG])
        self._call(f, "vqa_t5_relbias_fwd", self.p32["t5.relbias"], self.bucket, self.PB, self.h5, Lq, Lq)
        self._t5_layer_start = []
        for i in range(self.nl):
            self._t5_layer_start.append(len(f))
            self._call(f, "vqa_rmsnorm_fwd", self.HS[i], self.p32[f"t5.{i}.ln0"], None, self.N0[i], self.R0[i], T,
                       D, 1e-6, None)
            self._linear(f, self.N0[i], f"t5.{i}.qkv_w", T, out16=self.QKV[i], bias=False)
            q = self.QKV[i]
            self._attn(f, "vqa_attn_fwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, o=self.O[i], ldo=D, p=self.PT[i], bias=self.PB, key_mask=self.MASK, batch=B,
                       heads=self.h5, lq=Lq, lk=Lq, dh=self.dkv, scale=1.0, drop=t5_site(i, 0))
            # h + dropout(attention output)   (T5LayerSelfAttention :400)
            self._linear(f, self.O[i], f"t5.{i}.o_w", T, out32=self.HM[i], bias=False, res32=self.HS[i],
                         drop=t5_site(i, 1))
            # dropout(relu(wi h)) (T5DenseActDense :86), then h + dropout(wo .) (T5LayerFF :140)
            self._call(f, "vqa_rmsnorm_fwd", self.HM[i], self.p32[f"t5.{i}.ln1"], None, self.N1[i], self.R1[i], T,
                       D, 1e-6, None)
            self._linear(f, self.N1[i], f"t5.{i}.wi", T, out16=self.FF[i], bias=False, relu=True,
                         drop=t5_site(i, 2))
            self._linear(f, self.FF[i], f"t5.{i}.wo", T, out32=self.HS[i + 1], bias=False, res32=self.HM[i],
                         drop=t5_site(i, 3))
        kp = []
        self._call(f, "vqa_rmsnorm_fwd", self.HS[-1], self.p32["t5.final_ln"], self.TXT32, self.TXT16, self.RF, T, D,
                   1e-6, self._dptr(SITE_FINAL, kp), extra=kp + [self.RNG])
        self._fsplit.append(len(f))
        # SGA blocks: x = text always, y chained
        y16 = self.VIS16
        sc = 1.0 / math.sqrt(self.sga_dh)
        # self-attention halves of all blocks first (they only read the T5 output): one q|k|v
        # projection with N = 3 * 2304, the blocks' attentions, one batched merge
        NB, W3 = self.NB, 3 * D
        if self.fp8:                                          # the blocks' q|k|v weights as one [NB*2304, D] matrix
            x8, xs = self._quant_act(f, ("sga.qkv1", "x"), self.TXT16, T)
            w8 = self.W8[self.lay["sga0.qkv1_w"].offset:]
            self._gemm(f, x8, w8, T, NB * W3, D, lda=D, ldb=D, c16=self.QKV1A, ldc16=NB * W3,
                       bias=self.p32["sga0.qkv1_b"], fp8=True, scale_a=xs,
                       scale_b=ops.addr(self.WSC, self.lay["sga0.qkv1_w"].offset),
                       keep=self._sga_self_keep() + (self.W8, self.WSC))
        else:
            self._gemm(f, self.TXT16, self.p16["sga0.qkv1_w"], T, NB * W3, D, lda=D, ldb=D, c16=self.QKV1A,
                       ldc16=NB * W3, bias=self.p32["sga0.qkv1_b"], keep=self._sga_self_keep())
        grp = self._sga_groups()
        for n in range(0, NB, grp["groups"]):
            s, c0 = self.sga[n], n * W3
            q = self.QKV1A
            self._attn(f, "vqa_attn_fwd", q=ops.addr(q, c0), ldq=NB * W3, k=ops.addr(q, c0 + D), ldk=NB * W3,
                       v=ops.addr(q, c0 + 2 * D), ldv=NB * W3, o=s["O1"], ldo=D, p=s["P1"], batch=B,
                       heads=self.sga_heads, lq=Lq, lk=Lq, dh=self.sga_dh, scale=sc, drop=sga_site(n, 0),
                       keep=(q, self.O1A, self.P1A), **grp)
        m1kw = dict(c32=self.S1A, ldc32=D, bias=self.p32["sga0.m1_b"], res32=self.TXT32, ldres=D, batch=NB,
                    stride_a=T * D, stride_b=D * D, stride_c32=T * D, stride_res=0, stride_bias=D,
                    drop_site_stride=sga_site(1, 1) - sga_site(0, 1))
        if self.fp8:
            x8, xs = self._quant_act(f, ("sga.m1", "x"), self.O1A.view(NB * T, D), NB * T)
            o0 = self.lay["sga0.m1_w"].offset
            self._gemm(f, x8, self.W8[o0:], T, D, D, lda=D, ldb=D, fp8=True, scale_a=xs, stride_scale_a=T,
                       scale_b=ops.addr(self.WSC, o0), stride_scale_b=D * D,
                       keep=self._sga_self_keep() + (self.W8, self.WSC), **m1kw)
        else:
            self._gemm(f, self.O1A, self.p16["sga0.m1_w"], T, D, D, lda=D, ldb=D, keep=self._sga_self_keep(), **m1kw)
        self._set_drop(f[-1], sga_site(0, 1))
        for n in range(NB):
            s, p = self.sga[n], f"sga{n}."
            self._call(f, "vqa_layernorm_fwd", s["S1"], self.p32[p + "ln1_g"], self.p32[p + "ln1_b"], s["X1"],
                       s["X1h"], s["MU1"], s["RS1"], T, D, 1e-5)
        # the blocks' cross-attention queries read only their norm1 outputs: one launch
        # batched over the blocks (stack slot NB-1-n = the blocks' order in the arena)
        segs = [self.lay[f"sga{n}.q2_w"] for n in reversed(range(NB))]
        bsegs = [self.lay[f"sga{n}.q2_b"] for n in reversed(range(NB))]
        wst = segs[1].offset - segs[0].offset if NB > 1 else 0
        assert all(b_.offset - a_.offset == wst for a_, b_ in zip(segs, segs[1:]))
        assert all(b_.offset - a_.offset == wst for a_, b_ in zip(bsegs, bsegs[1:]))
        q2kw = dict(c16=self.Q2S, ldc16=D, bias=self.p32[f"sga{NB - 1}.q2_b"], batch=NB, stride_a=T * D,
                    stride_b=wst, stride_c16=T * D, stride_bias=wst)
        if self.fp8:
            x8, xs = self._quant_act(f, ("sga.q2", "x"), self.X1hS.view(NB * T, D), NB * T)
            o0 = self.lay[f"sga{NB - 1}.q2_w"].offset
            self._gemm(f, x8, self.W8[o0:], T, D, D, lda=D, ldb=D, fp8=True, scale_a=xs, stride_scale_a=T,
                       scale_b=ops.addr(self.WSC, o0), stride_scale_b=wst, keep=(self.P16, self.P32, self.W8, self.WSC),
                       **q2kw)
        else:
            self._gemm(f, self.X1hS, self.p16[f"sga{NB - 1}.q2_w"], T, D, D, lda=D, ldb=D, keep=(self.P16, self.P32),
                       **q2kw)
        for n in range(NB):
            s, p = self.sga[n], f"sga{n}."
            if n > 0:
                self._linear(f, y16, p + "kv2_w", s["ly"], out16=s["KV2"])
            kv = s["KV2"]
            self._attn(f, "vqa_attn_fwd", q=s["Q2"], ldq=D, k=kv, ldk=2 * D, v=ops.addr(kv, D), ldv=2 * D,
                       o=s["O2"], ldo=D, p=s["P2"], batch=B, heads=self.sga_heads, lq=Lq, lk=s["lk"], dh=self.sga_dh,
                       scale=sc, drop=sga_site(n, 2))
            self._linear(f, s["O2"], p + "m2_w", T, out32=s["S2"], res32=s["X1"], drop=sga_site(n, 3))
            self._call(f, "vqa_layernorm_fwd", s["S2"], self.p32[p + "ln2_g"], self.p32[p + "ln2_b"], s["X2"],
                       s["X2h"], s["MU2"], s["RS2"], T, D, 1e-5)
            self._linear(f, s["X2h"], p + "fc1_w", T, out16=s["FFh"], relu=True, drop=sga_site(n, 4))
            self._linear(f, s["FFh"], p + "fc2_w", T, out32=s["S3"], res32=s["X2"], drop=sga_site(n, 5))
            self._call(f, "vqa_layernorm_fwd", s["S3"], self.p32[p + "ln3_g"], self.p32[p + "ln3_b"], s["OUT"],
                       s["OUTh"], s["MU3"], s["RS3"], T, D, 1e-5)
            y16 = s["OUTh"]
        last = self.sga[-1]["OUT"]
        self._call(f, "vqa_head_fwd", last, self.p32["pool_w"], self.p32["pool_b"], self.p32["cls_w"],
                   self.p32["cls_b"], self.TGT, self.ATT, self.POOLED, self.LOGP, self.NLL, self.LOSS, B, Lq, D, self.A)

    # ------------------------------------------------------------------ backward plan
    def _plan_backward(self):
        D = self.D
        b = self.bwd_calls
        B, Lq, T, NB = self.B, self.L, self.T, self.NB
        nparts = L.load().vqa_norm_bwd_parts(T)
        # the dense embedding gradient only ever gets the touched rows written: re-zero the rows
        # the previous step wrote (IDS_PREV) instead of all 32128 x 768 floats (DP: dp.py swaps in
        # the gathered ids of every rank)
        z = self.g32["t5.embed"]
        self._call(self.zero_calls, "vqa_embedding_zero_rows", self.IDS_PREV, self.IDS, T, z, D, S.T5_VOCAB)
        b += self.zero_calls
        # head: log_softmax + NLL + classifier + attention pooler
        last = self.sga[-1]["OUT"]
        self._call(b, "vqa_head_bwd", last, self.ATT, self.POOLED, self.LOGP, self.TGT, self.p32["pool_w"],
                   self.p32["cls_w"], self.dY[(NB - 1) & 1], None, self.g32["pool_w"], self.g32["pool_b"],
                   self.g32["cls_w"], self.g32["cls_b"], self.WS_HEAD, B, Lq, D, self.A, self.NLL, self.LOSS,
                   None, 1.0)
        # ready marks: (number of backward calls issued, end of the gradient prefix now final).
        # The flat layout is in backward-completion order, so finished gradients always form
        # a prefix of G32: DP all-reduces bucket [prev_end, end) as soon as it is final.
        self.ready_marks = []
        self._sq_split = None        # (call index, prefix end) where the grad-norm pass can start early

        self._jobs = []

        def mark(seg):
            self._flush(b)                          # finish this segment's deferred reductions first
            sg = self.lay[seg]
            self.ready_marks.append((len(b), sg.offset + (sg.numel + 63) // 64 * 64))
        mark("pool_b")
        sc = 1.0 / math.sqrt(self.sga_dh)
        ks = self.drop_scale if self.p_drop > 0.0 else 1.0      # relu-mask dX: kept elements carry 1/(1-p)
        # the blocks' q2 / m2 / fc1 / fc2 weight gradients (768 x 768, K = 2048 each) are left
        # out of the sequential block chain and computed after it as one launch per weight
        # batched over the blocks (the block chain then runs its input gradients alone)
        self.dA3S, self.dBS, self.dA2S, self.dQS = (self._t((NB, T, D), BF16) for _ in range(4))
        batched = self.sga_dw_batch
        dxdw = (lambda lst, dy, x, w, rows, **kw: self._dx(lst, dy, w, rows, **kw)) if batched else self._dxdw
        for n in reversed(range(NB)):
            s, p = self.sga[n], f"sga{n}."
            dy = self.dY[n & 1]
            y16 = self.VIS16 if n == 0 else self.sga[n - 1]["OUTh"]
            # every bf16 gradient a weight-gradient GEMM reads gets its own buffer, so the dW
            # GEMMs can trail the dX chain on another stream without write-after-read hazards
            g = lambda nm, shape: self._gbuf(f"{p}{nm}", shape)
            slot = NB - 1 - n
            dA3, dA2, dB, dQ = self.dA3S[slot], self.dA2S[slot], self.dBS[slot], self.dQS[slot]
            dKV = g("dKV", (s["ly"], 2 * D))
            # norm3 + FFN: dA32 = grad of x + dropout3(ffn(x)) (the residual), dA16 = its dropout3 branch;
            # the fc2 bias gradient (column sums of the branch) is fused into the LayerNorm backward
            kp = []
            ws = self._norm_ws()
            self._call(b, "vqa_layernorm_bwd", dy, s["S3"], s["MU3"], s["RS3"], self.p32[p + "ln3_g"], None,
                       self.dA32, dA3, None, None, ws, T, D,
                       self._dptr(sga_site(n, 5), kp), self.g32[p + "fc2_b"], extra=kp + [self.RNG])
            for j, nm in enumerate(("ln3_g", "ln3_b", "fc2_b")):      # ws = [parts][dgamma | dbeta | dsum]
                self._defer(ws, nparts, 3 * D, D, self.g32[p + nm], offset=j * D)
            dxdw(b, dA3, s["FFh"], p + "fc2_w", T, out16=dB, mask16=s["FFh"], alpha=ks)
            if batched:
                self._dx(b, dB, p + "fc1_w", T, out32=self.dC32, res32=self.dA32)
                self._bias_colsum(b, dB, T, p + "fc1_b")
            else:
                self._dxdw(b, dB, s["X2h"], p + "fc1_w", T, bias_from=dB, out32=self.dC32, res32=self.dA32)
            # norm2 + cross attention (q from x, k/v from y)
            kp = []
            ws = self._norm_ws()
            self._call(b, "vqa_layernorm_bwd", self.dC32, s["S2"], s["MU2"], s["RS2"], self.p32[p + "ln2_g"], None,
                       self.dA32, dA2, None, None, ws, T, D,
                       self._dptr(sga_site(n, 3), kp), self.g32[p + "m2_b"], extra=kp + [self.RNG])
            for j, nm in enumerate(("ln2_g", "ln2_b", "m2_b")):      # ws = [parts][dgamma | dbeta | dsum]
                self._defer(ws, nparts, 3 * D, D, self.g32[p + nm], offset=j * D)
            dxdw(b, dA2, s["O2"], p + "m2_w", T, out16=self.dO16)
            kv = s["KV2"]
            self._attn(b, "vqa_attn_bwd", q=s["Q2"], ldq=D, k=kv, ldk=2 * D, v=ops.addr(kv, D), ldv=2 * D,
                       p=s["P2"], batch=B, heads=self.sga_heads, lq=Lq, lk=s["lk"], dh=self.sga_dh, scale=sc,
                       dout=self.dO16, lddo=D, dq=dQ, lddq=D, dk=dKV, lddk=2 * D,
                       dv=ops.addr(dKV, D), lddv=2 * D, drop=sga_site(n, 2))
            if batched:
                self._dx(b, dQ, p + "q2_w", T, out32=self.dC32, res32=self.dA32)
                self._bias_colsum(b, dQ, T, p + "q2_b")
            else:
                self._dxdw(b, dQ, s["X1h"], p + "q2_w", T, bias_from=dQ, out32=self.dC32, res32=self.dA32)
            if n == 0:
                self._dxdw(b, dKV, y16, p + "kv2_w", s["ly"], bias_from=dKV, out32=self.dVIS32, out16=self.dVIS16)
            else:
                self._dxdw(b, dKV, y16, p + "kv2_w", s["ly"], bias_from=dKV, out32=self.dY[(n - 1) & 1])
            # norm1: its residual input is the T5 output, so the text gradient of the blocks
            # accumulates here (dres = the running sum); the merge branch goes to dA1A[n]
            kp = []
            ws = self._norm_ws()
            self._call(b, "vqa_layernorm_bwd", self.dC32, s["S1"], s["MU1"], s["RS1"], self.p32[p + "ln1_g"],
                       None if n == NB - 1 else self.dTA[(n + 1) & 1], self.dTA[n & 1], self.dA1A[n], None, None,
                       ws, T, D, self._dptr(sga_site(n, 1), kp), self.g32[p + "m1_b"], extra=kp + [self.RNG])
            for j, nm in enumerate(("ln1_g", "ln1_b", "m1_b")):      # ws = [parts][dgamma | dbeta | dsum]
                self._defer(ws, nparts, 3 * D, D, self.g32[p + nm], offset=j * D)
            if not batched:
                mark(f"sga{n}.ln3_b")
        if batched:
            for w, dys, xs in (("fc2_w", self.dA3S, self.FFhS), ("fc1_w", self.dBS, self.X2hS),
                               ("m2_w", self.dA2S, self.O2S), ("q2_w", self.dQS, self.X1hS)):
                segs = [self.lay[f"sga{n}.{w}"] for n in reversed(range(NB))]
                lstride = segs[1].offset - segs[0].offset if NB > 1 else 0
                assert all(b_.offset - a_.offset == lstride for a_, b_ in zip(segs, segs[1:])), w
                self._gemm(b, dys, xs, D, D, T, lda=D, ldb=D, a_trans=True, b_trans=True,
                           c32=self.g32[f"sga{NB - 1}.{w}"], ldc32=D, batch=NB, stride_a=T * D, stride_b=T * D,
                           stride_c32=lstride, keep=(self.G32,))
                b[-1].side = True
        # the blocks' self-attention halves, batched: merge dX / dW (batch NB), the
        # attentions, then ONE q|k|v dX GEMM over K = NB * 2304 (it also sums the blocks'
        # text gradients, plus the norm1 residual sum as res32) paired with ONE q|k|v dW GEMM
        W3 = 3 * D
        keep = self._sga_self_keep()
        self._gemm(b, self.dA1A, self.p16["sga0.m1_w"], T, D, D, lda=D, ldb=D, b_trans=True, c16=self.dO1A,
                   ldc16=D, batch=NB, stride_a=T * D, stride_b=D * D, stride_c16=T * D, keep=keep)
        self._gemm(b, self.dA1A, self.O1A, D, D, T, lda=D, ldb=D, a_trans=True, b_trans=True,
                   c32=self.g32["sga0.m1_w"], ldc32=D, batch=NB, stride_a=T * D, stride_b=T * D,
                   stride_c32=D * D, keep=keep)
        b[-1].side = True
        dq = self.dQKV1A
        grp = self._sga_groups()
        for n in reversed(range(0, NB, grp["groups"])):
            s, c0 = self.sga[n], n * W3
            q = self.QKV1A
            self._attn(b, "vqa_attn_bwd", q=ops.addr(q, c0), ldq=NB * W3, k=ops.addr(q, c0 + D), ldk=NB * W3,
                       v=ops.addr(q, c0 + 2 * D), ldv=NB * W3, p=s["P1"], batch=B, heads=self.sga_heads, lq=Lq, lk=Lq,
                       dh=self.sga_dh, scale=sc, dout=self.dO1A[n], lddo=D, dq=ops.addr(dq, c0), lddq=NB * W3,
                       dk=ops.addr(dq, c0 + D), lddk=NB * W3, dv=ops.addr(dq, c0 + 2 * D), lddv=NB * W3,
                       drop=sga_site(n, 0), keep=(q, dq, self.P1A, self.dO1A), **grp)
        tmp = []
        self._gemm(tmp, dq, self.p16["sga0.qkv1_w"], T, D, NB * W3, lda=NB * W3, ldb=D, b_trans=True,
                   c32=self.dTXT, ldc32=D, res32=self.dTA[0], ldres=D, keep=keep)
        self._gemm(tmp, dq, self.TXT16, NB * W3, D, T, lda=NB * W3, ldb=D, a_trans=True, b_trans=True,
                   c32=self.g32["sga0.qkv1_w"], ldc32=D, keep=keep)
        tmp[1].side = True                         # not paired: the K = NB * 2304 dX wants split-K
        b.extend(tmp)
        lib = L.load()
        ws = self._t(lib.vqa_colsum_workspace_floats(T, NB * W3))
        self._call(b, "vqa_colsum", dq, 1, T, NB * W3, NB * W3, None, 0.0, ws)
        self._defer(ws, lib.vqa_colsum_parts(T), NB * W3, NB * W3, self.g32["sga0.qkv1_b"])
        self._jobs[-1] = self._jobs[-1][:-1] + (self._jobs[-1][-1] + keep,)
        mark(f"sga{NB - 1}.m1_b")
        # ConvTranspose2d scaler weight/bias gradient (vision branch: independent of the T5
        # backward below; its own colsum workspace).  The flipped-conv weight column t*C + c
        # (tap t = ky*3 + kx) is sum_pos dVIS[pos] * F4[pos shifted by tap t]; shifting dVIS
        # the other way instead makes the 9 taps ONE batched GEMM over plain operands:
        # dW[:, t*C:(t+1)*C] = shift_t(dVIS)^T @ F4 (vqa_tap_shift; no implicit im2col gather)
        self._bsplit = [len(b)]
        cin, fh = self.fc, self.fh
        self._call(b, "vqa_tap_shift", self.dVIS16, self.dVIS9, B, fh, fh, D, 3, 3, 1)
        self._gemm(b, self.dVIS9, self.F4, D, cin, self.V_TOK, lda=D, ldb=cin, a_trans=True, b_trans=True,
                   c32=self.g32["scaler_w"], ldc32=9 * cin, batch=9, stride_a=self.V_TOK * D, stride_b=0,
                   stride_c32=cin, keep=(self.G32,))
        self.scaler_dw_call = b[-1]                       # bench roofline_gemm: the step's largest launch
        self._call(b, "vqa_colsum", self.dVIS32, 0, self.V_TOK, D, D, self.g32["scaler_b"], 0.0, self.WS_COL2)
        mark("scaler_b")
        self._bsplit.append(len(b))
        # T5 encoder backward.  dH32 is the gradient of the residual stream h_i; dH16 the
        # dropout-masked gradient of the FF branch that produced it (T5LayerFF :140).
        nl = self.nl
        # per-layer bf16 gradients the weight gradients read, stacked like the inputs (slot 11 - i)
        self.dH16S, self.dHMS = self._t((nl, T, D), BF16), self._t((nl, T, D), BF16)
        self.dFS, self.dQKVS = self._t((nl, T, self.dff), BF16), self._t((nl, T, 3 * D), BF16)
        dH16 = [self.dH16S[nl - 1 - i] for i in range(nl)]               # FF-branch grad of layer i
        G = self.t5_dw_group
        kp = []
        ws = self._norm_ws()
        self._call(b, "vqa_rmsnorm_bwd", self.dTXT, self.HS[-1], self.RF, self.p32["t5.final_ln"], None, self.dH32,
                   dH16[-1], None, 0.0, ws, T, D,
                   self._dptr(SITE_FINAL, kp), None, self._dptr(t5_site(self.nl - 1, 3), kp),
                   extra=kp + [self.RNG])
        self._defer(ws, nparts, D, D, self.g32["t5.final_ln"])
        mark("t5.final_ln")
        # G > 1: the layers' input gradients chain alone and every G layers ONE batched launch
        # per weight (wo, wi, o, qkv) computes the group's weight gradients (4 x G GEMMs of
        # K = 2048 as 4 launches); G == 1: each layer's dX + dW as paired launches
        dxdw = self._dxdw if (G == 1 and not self.t5_dw_groups) else \
            (lambda lst, dy, x, w, rows, **kw: self._dx(lst, dy, w, rows, **kw))
        for i in reversed(range(nl)):
            dF, dHM, dQKV = self.dFS[nl - 1 - i], self.dHMS[nl - 1 - i], self.dQKVS[nl - 1 - i]
            dxdw(b, dH16[i], self.FF[i], f"t5.{i}.wo", T, out16=dF, mask16=self.FF[i], alpha=ks)
            dxdw(b, dF, self.N1[i], f"t5.{i}.wi", T, out32=self.dC32)
            kp = []
            ws = self._norm_ws()
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HM[i], self.R1[i], self.p32[f"t5.{i}.ln1"], self.dH32,
                       self.dHM32, dHM, None, 0.0, ws, T, D,
                       None, None, self._dptr(t5_site(i, 1), kp), extra=kp + [self.RNG])
            self._defer(ws, nparts, D, D, self.g32[f"t5.{i}.ln1"])
            dxdw(b, dHM, self.O[i], f"t5.{i}.o_w", T, out16=self.dO16)
            q = self.QKV[i]
            dq = dQKV
            self._attn(b, "vqa_attn_bwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, p=self.PT[i], bias=self.PB, key_mask=self.MASK, batch=B, heads=self.h5, lq=Lq,
                       lk=Lq, dh=self.dkv, scale=1.0, dout=self.dO16, lddo=D, dq=dq, lddq=3 * D,
                       dk=ops.addr(dq, D), lddk=3 * D, dv=ops.addr(dq, 2 * D), lddv=3 * D, dbias=self.dSB[i],
                       drop=t5_site(i, 0))
            dxdw(b, dq, self.N0[i], f"t5.{i}.qkv_w", T, out32=self.dC32)
            # layer 0: dH32 becomes the embedding gradient (masked by the embedding dropout :725);
            # otherwise dH16 is the FF branch gradient of layer i-1
            kp = []
            d32 = self._dptr(SITE_EMBED, kp) if i == 0 else None
            d16 = self._dptr(t5_site(i - 1, 3), kp) if i > 0 else None
            ws = self._norm_ws()
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HS[i], self.R0[i], self.p32[f"t5.{i}.ln0"], self.dHM32,
                       self.dH32, dH16[i - 1] if i > 0 else None, None, 0.0, ws, T, D,
                       None, d32, d16, extra=kp + [self.RNG])
            self._defer(ws, nparts, D, D, self.g32[f"t5.{i}.ln0"])
            done = nl - i                                   # layers finished so far (11 .. i)
            ends = (np.cumsum(self.t5_dw_groups) if self.t5_dw_groups else None)
            if G == 1 and ends is None:
                mark(f"t5.{i}.ln1")
            elif ends is not None and done in ends:
                k = int(np.searchsorted(ends, done))
                self._t5_group_dw(b, i + self.t5_dw_groups[k] - 1, i)
                mark(f"t5.{i}.ln1")
                if self._sq_split is None and i > 0:      # the first T5 dW group is final
                    self._sq_split = self.ready_marks[-1]
            elif ends is None and (done % G == 0 or i == 0):
                self._t5_group_dw(b, i + (done - 1) % G, i)
                mark(f"t5.{i}.ln1")
                if self._sq_split is None and i > 0:
                    self._sq_split = self.ready_marks[-1]
        # the relative-position bias is shared by all 12 layers: dPB = sum over (layer, sample) of dS,
        # one fixed-order reduction after the last layer instead of one per layer
        self._call(b, "vqa_batch_sum", self.dSB, self.nl * B, self.h5 * Lq * Lq, self.dPB, 0.0)
        self._call(b, "vqa_t5_relbias_bwd", self.dPB, self.bucket, self.g32["t5.relbias"], self.h5, Lq, Lq,
                   S.T5_BUCKETS)
        mark("t5.relbias")
        self._flush(b)
        # embedding rows last (DP replaces this call by an all-gather of (id, dH row) pairs)
        self._call(b, "vqa_embedding_bwd", self.IDS, self.dH32, self.g32["t5.embed"], T, D, S.T5_VOCAB, self.WS_EMB)
        self.emb_call = b[-1]

    def _t5_group_dw(self, lst, i_hi, i_lo):
        """Weight gradients of T5 layers i_hi >= .. >= i_lo: per weight one launch batched over
        the layers (stack slot 11 - i, consecutive gradient segments at a constant stride)."""
        nl, T = self.nl, self.T
        cnt, s0 = i_hi - i_lo + 1, nl - 1 - i_hi
        for w, dys, xs in (("wo", self.dH16S, self.FFS), ("wi", self.dFS, self.N1S), ("o_w", self.dHMS, self.OS),
                           ("qkv_w", self.dQKVS, self.N0S)):
            nout, kin = self.g32[f"t5.{i_hi}.{w}"].shape
            segs = [self.lay[f"t5.{i}.{w}"] for i in range(i_hi, i_lo - 1, -1)]
            lstride = segs[1].offset - segs[0].offset if cnt > 1 else 0
            assert all(b.offset - a.offset == lstride for a, b in zip(segs, segs[1:])), w
            self._gemm(lst, ops.addr(dys, s0 * T * nout), ops.addr(xs, s0 * T * kin), nout, kin, T, lda=nout,
                       ldb=kin, a_trans=True, b_trans=True, c32=self.g32[f"t5.{i_hi}.{w}"], ldc32=kin, batch=cnt,
                       stride_a=T * nout, stride_b=T * kin, stride_c32=lstride, keep=(dys, xs, self.G32))
            lst[-1].side = True

    # ------------------------------------------------------------------ optimizer plan
    def _plan_optimizer(self):
        o = self.opt_calls
        n = self.lay.total
        # squared-norm partials over two ranges: [0, rel-bias) is final once the backward's
        # deferred column sums are flushed, so graph steps run it beside the embedding-gradient
        # scatter (run_backward_streams); the rel-bias + embedding-table range follows it
        # [0, a) is final once the first T5 weight-gradient group is (graph steps run that part
        # beside the backward's last layers), [a, rel-bias) with the last group
        e0 = self.lay["t5.relbias"].offset
        a = self._sq_split[1] if self._sq_split is not None else e0
        assert a % 4 == 0 and e0 % 4 == 0 and (n - e0) % 4 == 0 and a <= e0
        K = self.SQ_PARTS
        self._call(o, "vqa_grad_sqnorm", self.G32, a, self.WS_SQ, K)
        self._call(o, "vqa_grad_sqnorm", ops.addr(self.G32, a), e0 - a, ops.addr(self.WS_SQ, K), K,
                   extra=[self.G32, self.WS_SQ])
        self._call(o, "vqa_grad_sqnorm", ops.addr(self.G32, e0), n - e0, ops.addr(self.WS_SQ, 2 * K), K,
                   extra=[self.G32, self.WS_SQ])
        self._call(o, "vqa_optim_finalize", self.WS_SQ, 3 * K, float(self.grad_scale), float(self.max_norm),
                   int(self.warmup), int(self.total), float(self.betas[0]), float(self.betas[1]), self.opt_state)
        d = L.AdamWDesc()
        d.param, d.grad = self.P32.data_ptr(), self.G32.data_ptr()
        d.exp_avg, d.exp_avg_sq, d.max_exp_avg_sq = self.M.data_ptr(), self.V.data_ptr(), self.VMAX.data_ptr()
        d.param16 = self.P16.data_ptr()
        d.n = n
        ends, lrs = self.lay.group_of_element()
        lrs = [self.group_lr.get(g, lr) for g, lr in zip(self.lay.groups, lrs)]
        d.ngroups = len(ends)
        for i, (e, lr) in enumerate(zip(ends, lrs)):
            d.group_end[i], d.group_lr[i] = e, lr
        d.beta1, d.beta2, d.eps, d.weight_decay = self.betas[0], self.betas[1], self.eps, self.wd
        d.grad_scale = self.grad_scale
        d.state = self.opt_state.data_ptr()
        self._adam_desc = d
        keep = (self.P32, self.G32, self.M, self.V, self.VMAX, self.P16, self.opt_state)
        self.adam_full = ops.Call("vqa_adamw_amsgrad", ctypes.byref(d), desc=d, keep=keep)
        # Deferred update (defer_opt): step k's AdamW runs inside step k+1's forward, one
        # parameter range at a time on its own stream, each range just before its first use
        # (the forward reads the layout back to front: T5 layers 0..11, then the scaler / SGA /
        # head).  The embedding table + rel-bias range is read by the forward's very first
        # calls, so it is applied at the end of step k instead (the T5 chain would otherwise
        # start behind its 0.9 GB pass).  Same arithmetic, same order of updates vs uses.
        lay = self.lay
        cuts = [("embed", lay["t5.relbias"].offset, n)]
        for i in range(self.nl):
            lo = lay[f"t5.{i}.qkv_w"].offset if i < self.nl - 1 else lay["t5.final_ln"].offset
            hi = lay[f"t5.{i - 1}.qkv_w"].offset if i > 0 else lay["t5.relbias"].offset
            cuts.append((f"t5.{i}", lo, hi))
        cuts.append(("scaler", lay["scaler_w"].offset, lay["t5.final_ln"].offset))
        cuts.append(("head", 0, lay["scaler_w"].offset))     # classifier, pooler, SGA
        assert sum(hi - lo for _, lo, hi in cuts) == n
        # fp8: the e4m3 copies of the range's weights follow every AdamW range (and the whole
        # update when it is not deferred)
        quant = {name: [] for name, _, _ in cuts}
        self.quant_all = []
        if self.fp8:
            jobs = [(f"t5.{i}.{w}", None) for i in range(self.nl) for w in self.FP8_T5]
            jobs.append(("sga0.qkv1_w", self.NB * 3 * self.D))          # the blocks' side-by-side q|k|v
            jobs += [(f"sga{n}.{w}", None) for n in range(self.NB) for w in self.FP8_SGA if w != "qkv1_w"]
            for wname, rows in jobs:
                off = self.lay[wname].offset
                nm = next(name for name, lo, hi in cuts if lo <= off < hi)
                self._quant_weight(quant[nm], wname, rows)
                self.quant_all += quant[nm][-1:]
        self.adam_segs = []
        self.adam_embed = None
        for name, lo, hi in cuts:
            ds = L.AdamWDesc()
            ctypes.memmove(ctypes.addressof(ds), ctypes.addressof(d), ctypes.sizeof(d))
            ds.param, ds.grad = ops.addr(self.P32, lo), ops.addr(self.G32, lo)
            ds.exp_avg, ds.exp_avg_sq = ops.addr(self.M, lo), ops.addr(self.V, lo)
            ds.max_exp_avg_sq, ds.param16 = ops.addr(self.VMAX, lo), ops.addr(self.P16, lo)
            ds.n = hi - lo
            for i, e in enumerate(ends):
                ds.group_end[i] = e - lo
            c = ops.Call("vqa_adamw_amsgrad", ctypes.byref(ds), desc=ds, keep=keep)
            if quant[name]:
                c = _Seq([c] + quant[name])
            if name == "embed":
                self.adam_embed = c
            else:
                self.adam_segs.append((name, c))
        lst = []
        self._call(lst, "vqa_zero", ops.addr(self.opt_state, L.ST_PENDING), 16, extra=[self.opt_state])
        self.clear_pending = lst[0]
        if not self.defer_opt:
            o.append(self.adam_full)
            o += self.quant_all
        elif self.adam_embed is not None:
            o.append(self.adam_embed)
        # The embedding table's update split by rows (vqa_adamw_rows): the rows no
        # token of the step touched have a zero gradient, so their update runs beside the
        # backward (emb_pre: mark the step's ids, then those rows), and the step's exposed tail
        # keeps only the rel-bias range and the touched rows (tail_calls).  Bit-identical to the
        # dense range; used by the stream / graph step (run_backward_streams with sq_overlap),
        # while opt_calls keeps the dense form (eager steps, dp.DataParallelStep's finish graph).
        self.embed_split = self.defer_opt and os.environ.get("VQA_EMBED_SPLIT", "1") != "0"
        self.tail_calls = o[2:]
        self.emb_pre = []
        if self.embed_split:
            emb = lay["t5.embed"]
            assert emb.offset + emb.numel == n and self.adam_embed is o[-1]
            if getattr(self, "EMB_MARK", None) is None:
                self.EMB_MARK = torch.full((S.T5_VOCAB,), -1, dtype=torch.int32, device=self.dev)
            dt = L.AdamWDesc()
            ctypes.memmove(ctypes.addressof(dt), ctypes.addressof(d), ctypes.sizeof(d))
            lo = emb.offset
            dt.param, dt.grad = ops.addr(self.P32, lo), ops.addr(self.G32, lo)
            dt.exp_avg, dt.exp_avg_sq = ops.addr(self.M, lo), ops.addr(self.V, lo)
            dt.max_exp_avg_sq, dt.param16 = ops.addr(self.VMAX, lo), ops.addr(self.P16, lo)
            dt.n = emb.numel
            for i in range(d.ngroups):                     # as adam_range_call: ends relative to the table
                dt.group_end[i] = d.group_end[i] - lo
            self._emb_desc = dt
            keep = (self.P32, self.G32, self.M, self.V, self.VMAX, self.P16, self.opt_state, self.EMB_MARK)
            rows_call = lambda touched: ops.Call("vqa_adamw_rows", ctypes.byref(dt), self.EMB_MARK.data_ptr(),  # noqa: E731
                                                 S.T5_VOCAB, self.D, touched, int(self.warmup), int(self.total),
                                                 desc=dt, keep=keep)
            self.emb_pre = [ops.Call("vqa_embed_mark", self.IDS.data_ptr(), self.T, S.T5_VOCAB,
                                     self.EMB_MARK.data_ptr(), self.opt_state.data_ptr(),
                                     keep=(self.IDS, self.EMB_MARK, self.opt_state)),
                            # the untouched rows' pass as 256 workgroups striding over the rows: a
                            # 32k-block grid beside the chain cost what it saved at the tail (A/B:
                            # 6.47-6.48 ms either way), 256 measured 6.44-6.47
                            rows_call(int(os.environ.get("VQA_EMB_GRID", "256")))]
            self.tail_calls = o[2:-1] + [self.adam_range_call(lay["t5.relbias"].offset, lo), rows_call(1)]

    def adam_range_call(self, lo, hi):
        """The fused AdamW-amsgrad pass over flat parameters [lo, hi) only (the step's device
        state: clip coefficient, schedule, bias corrections; no-op unless an update is pending)."""
        d = self._adam_desc
        ds = L.AdamWDesc()
        ctypes.memmove(ctypes.addressof(ds), ctypes.addressof(d), ctypes.sizeof(d))
        ds.param, ds.grad = ops.addr(self.P32, lo), ops.addr(self.G32, lo)
        ds.exp_avg, ds.exp_avg_sq = ops.addr(self.M, lo), ops.addr(self.V, lo)
        ds.max_exp_avg_sq, ds.param16 = ops.addr(self.VMAX, lo), ops.addr(self.P16, lo)
        ds.n = hi - lo
        for i in range(d.ngroups):
            ds.group_end[i] = d.group_end[i] - lo
        return ops.Call("vqa_adamw_amsgrad", ctypes.byref(ds), desc=ds,
                        keep=(self.P32, self.G32, self.M, self.V, self.VMAX, self.P16, self.opt_state))

    def flush_optimizer(self):
        """Apply a deferred AdamW update now (before reading the parameters outside a step)."""
        if self.defer_opt:
            self._run([c for _, c in self.adam_segs] + [self.clear_pending])

    def set_training(self, mode=True):
        """model.train() / model.eval(): the dropout kernels read this device flag at run
        time, so captured graphs stay valid."""
        self.RNG[2].fill_(1 if mode else 0)

    def configure_optimizer(self, group_lr=None, warmup=None, total=None, max_norm=None, weight_decay=None,
                            betas=None, eps=None):
        """Re-plan the clip + AdamW + schedule tail (faster_rcnn_vqa_trainer.py:231-287 knobs)."""
        if group_lr:
            self.group_lr.update(group_lr)
        if warmup is not None:
            self.warmup = int(warmup)
        if total is not None:
            self.total = int(total)
        if max_norm is not None:
            self.max_norm = float(max_norm)
        if weight_decay is not None:
            self.wd = float(weight_decay)
        if betas is not None:
            self.betas = tuple(betas)
        if eps is not None:
            self.eps = float(eps)
        self.opt_calls = []
        self._plan_optimizer()
        self.graph = None

    def set_grad_scale(self, s):
        """DP: grads are summed over ranks; the average enters as a scale."""
        self.grad_scale = float(s)
        self.opt_calls = []
        self._plan_optimizer()
        self.graph = None

    # ------------------------------------------------------------------ execution
    def _run(self, calls):
        s = L.stream_handle()
        for c in calls:
            c(s)

    def load_batch(self, batch, next_images=None):
        """Copy a batch dict (numpy or torch, host or device) into the static input buffers.
        Pipelined engines take the batch's text and targets, and `next_images` = the image
        tensors of the batch that the FOLLOWING step trains on (this batch's images went
        in one step earlier, or through prime())."""
        ae = self.allow_empty_rows
        n = batch_rows(batch, "question_input_ids", self.B, ae)
        if self.pipeline:
            # this batch's images went in one step earlier (or through prime()): their row count
            # must be the text's, else the rows past the shorter one would pair other samples'
            # features with real targets
            if self._img_rows_next is not None and self._img_rows_next != n:
                raise ValueError(f"pipelined engine: this batch has {n} question rows but its images "
                                 f"(loaded one step earlier) had {self._img_rows_next}")
            if next_images is not None:
                ni = batch_rows({"image_tensors": next_images}, "image_tensors", self.B, ae)
                load_rows(self.IMG, next_images, ni)
                self._img_rows_next = ni
            else:
                self._img_rows_next = None
        else:
            load_rows(self.IMG, batch["image_tensors"], n)
        self.rows = n
        load_rows(self.IDS, batch["question_input_ids"], n)
        load_rows(self.MASK, batch["question_attention_masks"], n, empty_fill=1)
        load_rows(self.TGT, batch.get("annotation_ids"), n, fill=IGNORE_INDEX)

    def prime(self, images):
        """Pipelined engines: compute the layer4 features of the first batch's images, so
        that the first train_step has them (later steps produce their successor's)."""
        assert self.pipeline, "prime() is for pipelined engines"
        ni = batch_rows({"image_tensors": images}, "image_tensors", self.B, self.allow_empty_rows)
        load_rows(self.IMG, images, ni)
        self._img_rows_next = ni
        self._run(self.res_calls)

    def use_global_rows(self, world):
        """Data parallel (dp.DataParallelStep): the head backward divides by the valid-row count
        summed over the `world` ranks (ROWTOT, which the DP step fills each step: count_call, then
        an all-reduce) over `world` instead of by the rank's own count, and rewrites LOSS as the
        rank's share (vqa_head_bwd, ABI 18), so the summed, 1/world-scaled gradients are the
        global batch's NLL mean however the global batch is split -- unequal rows per rank, or a
        rank with none (allowed from here on: its gradient is zero).  The reference's mean is
        over the whole batch (resnet_vqa_model.py:159, loaders without drop_last,
        trainer/faster_rcnn_vqa_trainer.py:172-197)."""
        i = next(k for k, c in enumerate(self.bwd_calls) if c.name == "vqa_head_bwd")
        old = self.bwd_calls[i]
        if self.count_call is not None:
            assert old.args[-1] == float(world), "use_global_rows: already set for another world size"
            return
        new = ops.Call("vqa_head_bwd", *old.args[:-2], ops.addr(self.ROWTOT), float(world),
                       keep=tuple(old.keep) + (self.ROWTOT,))
        new.side = old.side
        self.bwd_calls[i] = new
        self.count_call = ops.Call("vqa_count_targets", ops.addr(self.TGT), self.B, ops.addr(self.ROWTOT),
                                   keep=(self.TGT, self.ROWTOT))
        self.allow_empty_rows = True
        self.graph = None

    def forward(self):
        if self.defer_opt:                              # the previous step's update, then the forward
            self._run([c for _, c in self.adam_segs] + [self.clear_pending])
        self._run(self.fwd_calls)

    def backward(self):
        self._run(self.bwd_calls)

    def optimizer_step(self):
        self._run(self.opt_calls)

    def _run_step_streams(self, optimizer=True):
        """One step with graph-level concurrency: the frozen-ResNet + ConvTranspose2d
        branch and the T5 encoder run on two streams in the forward (they meet at
        SGA block 0), and the scaler weight gradient overlaps the T5 backward.
        Buffers of the two branches are disjoint, so the result is the same as
        the sequential order (and bit-identical: no cross-branch reductions)."""
        self.run_forward_streams()
        if optimizer:
            self.run_backward_streams(sq_overlap=True)
            self._run(self.tail_calls)
        else:
            self.run_backward_streams()

    def run_forward_streams(self):
        main = torch.cuda.current_stream(self.dev)
        side = self._side
        f = self.fwd_calls
        p0, p1, p2 = self._fsplit
        self._run(f[:p0])                                  # rng advance
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        # Issue the two branches interleaved (ResNet + ConvTranspose2d on `main`,
        # T5 encoder on `side`): a replayed graph submits its nodes in capture
        # order, so capturing one branch whole would hold the other back until
        # all of its nodes were submitted (measured: the ResNet branch started
        # ~1 ms into the step).
        hm, hs = L.stream_handle(main), L.stream_handle(side)
        vis, txt = f[p0:p1], f[p1:p2]
        if self.defer_opt:
            self._forward_branches_deferred(fork, main, side, vis, txt)
        else:
            j = 0
            for i, c in enumerate(vis):
                c(hm)
                upto = (i + 1) * len(txt) // len(vis)
                while j < upto:
                    txt[j](hs)
                    j += 1
            for c in txt[j:]:
                c(hs)
            join = torch.cuda.Event()
            join.record(side)
            main.wait_event(join)
        self._run(f[p2:])                                  # SGA + head

    def _forward_branches_deferred(self, fork, main, side, vis, txt):
        """The two forward branches with the previous step's AdamW ranges on a third stream.
        Capture order is submission order for a replayed graph, so the ranges are issued
        two T5 layers ahead of the layer calls that wait for them (issuing all of them
        first held the T5 chain back ~0.47 ms); the vision branch's parameter-reading
        calls wait for the scaler range, the SGA / head for the last range."""
        hm, hs = L.stream_handle(main), L.stream_handle(side)
        # the ranges run on the vision-branch stream: a fourth concurrent stream shares a
        # hardware queue with one of the others anyway (measured 6.85 vs 6.81 ms)
        ost = main
        hs_o = L.stream_handle(ost)
        segs = dict(self.adam_segs)
        order = [n for n, _ in self.adam_segs]
        ev = {}

        def issue(name):
            segs[name](hs_o)
            ev[name] = torch.cuda.Event()
            ev[name].record(ost)
        p0, p1 = self._fsplit[0], self._fsplit[1]
        starts = [at - p1 for at in self._t5_layer_start]
        nl = len(starts)
        # ranges in issue order: layers 0, 1, the scaler, the SGA / head range (the vision
        # branch's SGA block-0 k/v projection reads it), then layer i+2 at layer i
        ahead = 2                                          # layers a range runs ahead of its use
        for i in range(min(ahead, nl)):
            issue(f"t5.{i}")
        issue("scaler")
        issue("head")
        vpre = vis[:self._fvis_param - p0]                 # frozen ResNet calls (unpipelined engines)
        vpost = vis[self._fvis_param - p0:]                # ConvTranspose2d + SGA block 0 k/v
        bounds = starts + [len(txt)]
        j = 0
        feed = getattr(self, "_res_feed", None)            # the next batch's ResNet (res_order interleave)
        nres = len(feed[0]) if feed else 0
        head = min(nres, getattr(self, "res_head", 4))

        def res_upto(n):
            while feed and feed[0] and nres - len(feed[0]) < n:
                feed[0].pop(0)(feed[1])
        res_upto(head)
        for t in range(bounds[0]):                         # embedding + rel-bias
            txt[t](hs)
        for i in range(nl):
            if i + ahead < nl:
                issue(f"t5.{i + ahead}")
            side.wait_event(ev[f"t5.{i}"])
            for t in range(bounds[i], bounds[i + 1]):
                txt[t](hs)
            res_upto(head + (i + 1) * (nres - head) // nl)
            # the ResNet calls spread over the layers (as in the plain interleave); the
            # parameter-reading vision calls follow the last of them (they read its output)
            while j < (i + 1) * len(vpre) // nl:
                vpre[j](hm)
                j += 1
            if j == len(vpre) and vpost:
                main.wait_event(ev["scaler"])
                main.wait_event(ev["head"])
                for c in vpost:
                    c(hm)
                vpost = []
        join = torch.cuda.Event()
        join.record(side)
        main.wait_event(join)
        main.wait_event(ev[f"t5.{nl - 1}"])               # the last range issued (stream order)
        self.clear_pending(hm)                             # the update is applied: once only
        assert set(ev) == set(order)

    def run_backward_streams(self, sq_overlap=False):
        """sq_overlap: also run the optimizer plan's first two calls (the squared-norm partials
        of [0, a), final once the first T5 weight-gradient group is, and of [a, rel-bias),
        final before the embedding scatter) on `side`, beside the backward's tail; the caller
        then runs tail_calls (opt_calls[2:], the embedding table's dense update split by rows:
        emb_pre runs here, on `side`)."""
        main = torch.cuda.current_stream(self.dev)
        side, wside = self._side, self._wside
        b = self.bwd_calls
        q0, q1 = self._bsplit
        self._run_tagged(b[:q0], main, wside)              # head + SGA backward
        fork2 = torch.cuda.Event()
        fork2.record(main)
        side.wait_event(fork2)
        with torch.cuda.stream(side):
            self._run(b[q0:q1])                            # scaler dW / db
            if sq_overlap:                                 # a full step: the untouched embedding rows'
                self._run(self.emb_pre)                    # update, beside the T5 backward
        if sq_overlap:
            assert b[-1] is self.emb_call

            def to_side(calls):                            # after everything issued so far on main / wside
                for st in ((main, wside) if self.dw_stream else (main,)):
                    ev = torch.cuda.Event()
                    ev.record(st)
                    side.wait_event(ev)
                with torch.cuda.stream(side):
                    self._run(calls)
            m1 = self._sq_split[0] if self._sq_split is not None else None
            if m1 is not None and q1 < m1 < len(b) - 1:
                self._run_tagged(b[q1:m1], main, wside)    # T5 backward up to the first dW group
                to_side(self.opt_calls[:1])                # grad-norm partials of [0, a), beside the rest
                self._run_tagged(b[m1:-1], main, wside)
                to_side(self.opt_calls[1:2])               # ... and of [a, rel-bias)
            else:
                self._run_tagged(b[q1:-1], main, wside)    # T5 backward (+ deferred column sums)
                to_side(self.opt_calls[:2])
            self._run(b[-1:])                              # embedding rows
        else:
            self._run_tagged(b[q1:], main, wside)          # T5 backward + embedding
        for st in (side, wside):
            join2 = torch.cuda.Event()
            join2.record(st)
            main.wait_event(join2)

    def _run_tagged(self, calls, main, wside):
        """Run `calls` in order on `main`, except runs of side-tagged calls (weight
        gradients), which go to `wside` after an event on `main` at that point
        (`dw_stream`, on by default): the batched T5 dW launches trail the input-gradient chain
        (6.66 vs 6.78-6.84 ms per step).  dp.DataParallelStep keeps this placement across its
        stage graphs (dp.plan_stages: a segment's side-tagged calls forked beside the next
        chain segment, its gradient bucket all-reduced once that stage has ended).  Every
        bf16 gradient a side-tagged call reads has its own buffer (_gbuf), so no later chain
        call overwrites it (tests: test_dw_stream_matches_single_stream_bitwise)."""
        if not self.dw_stream:
            self._run(calls)
            return
        i, n = 0, len(calls)
        while i < n:
            j = i
            while j < n and calls[j].side == calls[i].side:
                j += 1
            if calls[i].side:
                ev = torch.cuda.Event()
                ev.record(main)
                wside.wait_event(ev)
                with torch.cuda.stream(wside):
                    self._run(calls[i:j])
            else:
                self._run(calls[i:j])
            i = j

    def set_res_cumask(self, words):
        """Experiment (bench.py --res-cumask): run the next batch's ResNet on a stream restricted
        to the CUs whose bits are set in `words` (hipExtStreamCreateWithCUMask, 32 CUs per word),
        launched eagerly beside the step graph, which then holds the chain only.  Call before
        capture().  Ordering as in the graph: F4 <- F4N, then the ResNet may overwrite F4N; the
        next step's inputs wait for it."""
        hip = L.hip_runtime()
        s = ctypes.c_void_p()
        arr = (ctypes.c_uint32 * len(words))(*words)
        with torch.cuda.device(self.dev):
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        self.reset_res_cumask()                       # one masked stream at a time
        self._rstream_plain = self._rstream           # restored by reset_res_cumask
        self._rstream_handle = s
        self._rstream = torch.cuda.ExternalStream(s.value, device=self.dev)
        self.res_external = True

    def reset_res_cumask(self, destroy=True):
        """End the set_res_cumask experiment: the ResNet goes back to the engine's own stream and
        into the captured step (re-capture needed: the graph is dropped).  destroy=False keeps the
        masked stream alive and returns it (tools/queue_probe.py times the step while it exists);
        the caller then owns the handle (hipStreamDestroy)."""
        h = getattr(self, "_rstream_handle", None)
        if h is None:
            return None
        torch.cuda.synchronize(self.dev)
        masked = self._rstream
        self._rstream = self._rstream_plain
        self._rstream_handle = None
        if self.res_external:
            self.res_external = False
            self.graph = None
        if destroy:
            rc = L.hip_runtime().hipStreamDestroy(h)
            if rc != 0:
                raise RuntimeError(f"hipStreamDestroy failed ({rc})")
            return None
        return masked, h

    def _res_external_step(self):
        main = torch.cuda.current_stream(self.dev)
        self.copy_f4(L.stream_handle(main))
        fork = torch.cuda.Event()
        fork.record(main)
        for g in self.graph:
            g.replay()
        self._rstream.wait_event(fork)
        with torch.cuda.stream(self._rstream):
            self._run(self.res_calls)
        join = torch.cuda.Event()
        join.record(self._rstream)
        main.wait_event(join)

    def _step_pipelined(self):
        """One pipelined step: F4 <- F4N (features of this batch, made last step), then the
        ResNet of the next batch (IMG -> F4N) on its own stream, concurrently with this
        step's whole chain on the current stream; joined at the end.  The two sides share
        no buffer, so every result equals the unpipelined step's bit for bit."""
        main = torch.cuda.current_stream(self.dev)
        if self.res_external:                              # the chain only (set_res_cumask)
            self.run_forward_streams()
            self.run_backward_streams(sq_overlap=True)
            self._run(self.tail_calls)
            return
        if not (torch.cuda.is_current_stream_capturing() and getattr(self, "res_order", "first") == "root"):
            self.copy_f4(L.stream_handle(main))            # ("root": issued before the replay, train_step)
        fork = torch.cuda.Event()
        fork.record(main)
        self._rstream.wait_event(fork)

        # the ResNet branch is captured first: a replayed graph submits nodes in capture order,
        # and issuing it after T5 layer 0 / 1 / 3 measured 0.7 ms slower
        # (res_order "last": the same dependencies, the ResNet's nodes created after the chain's)
        last = getattr(self, "res_order", "first") == "last"
        inter = getattr(self, "res_order", "first") == "interleave"
        if inter:                    # issued between the T5 encoder layers (_forward_branches_deferred)
            self._res_feed = [list(self.res_calls), L.stream_handle(self._rstream)]
        elif not last:
            with torch.cuda.stream(self._rstream):
                self._run(self.res_calls)
        self.run_forward_streams()                         # ConvTranspose2d || T5 encoder, then SGA
        if inter:
            assert not self._res_feed[0], "every ResNet call issued"
            self._res_feed = None
        self.run_backward_streams(sq_overlap=True)
        self._run(self.tail_calls)
        if last:
            with torch.cuda.stream(self._rstream):
                self._run(self.res_calls)
        join = torch.cuda.Event()
        join.record(self._rstream)
        main.wait_event(join)

    def train_step(self):
        """zero_grad -> forward -> backward -> (all-reduce) -> clip -> AdamW -> sched, all on-device."""
        if self.graph is not None and self.res_external:
            self._res_external_step()
            return
        if self.graph is not None and self.pipeline and getattr(self, "res_order", "first") == "root":
            self.copy_f4(L.stream_handle(torch.cuda.current_stream(self.dev)))
        if self.graph is not None:
            for g in self.graph:
                if callable(g):
                    g()
                else:
                    g.replay()
            return
        if self.pipeline:
            assert self.allreduce is None, "pipelined DP steps go through dp.DataParallelStep"
            self._step_pipelined()
            return
        self.forward()
        self.backward()
        if self.allreduce is not None:
            self.allreduce(self.G32)
        self.optimizer_step()

    def capture(self, warm=True, keep_graph=False):
        """Capture the step as hipGraph(s): one graph when single-GPU; with a DP
        all-reduce hook, graph(fwd+bwd) -> eager collective -> graph(optimizer).
        keep_graph: keep the hipGraph_t of each part (torch CUDAGraph keep_graph) so tests can
        walk its nodes (raw_cuda_graph); the exec is instantiated here either way."""
        self._keep_graph = bool(keep_graph)
        self.flush_optimizer()           # the warm-up's backward must not overwrite a pending update's G
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        saved, saved_rng = self.opt_state.clone(), self.RNG.clone()
        with torch.cuda.stream(s):
            if warm:                                    # warm-up launch outside capture (no update)
                self._run(self.fwd_calls)
                self.backward()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with no_gc_capture():
            parts = self._capture_parts(s)
        self.opt_state.copy_(saved)
        self.RNG.copy_(saved_rng)                       # the warm-up launch must not consume a dropout draw
        for g in parts:
            if self._keep_graph and not callable(g):
                g.instantiate()
        self.graph = parts

    def _new_graph(self):
        return torch.cuda.CUDAGraph(keep_graph=getattr(self, "_keep_graph", False))

    def _capture_parts(self, s):
        if self.allreduce is None:
            g = self._new_graph()
            with torch.cuda.graph(g, stream=s):
                if self.pipeline:
                    self._step_pipelined()
                else:
                    self._run_step_streams()
            parts = [g]
        else:
            g1, g2 = self._new_graph(), self._new_graph()
            with torch.cuda.graph(g1, stream=s):
                self.forward()
                self.backward()
            with torch.cuda.graph(g2, stream=s):
                self.optimizer_step()
            ar = self.allreduce
            parts = [g1, lambda: ar(self.G32), g2]
        return parts

    # ------------------------------------------------------------------ GEMM autotuning
    def _tune_scratch(self, d):
        """Zero-filled split-K workspace shared by every candidate timed during tuning
        (one stream, one launch at a time; each launch leaves its counters zero)."""
        need = int(L.load().vqa_gemm_workspace_bytes(ctypes.byref(d)))
        if self._scratch is None or self._scratch.numel() * 4 < need:
            self._scratch = torch.zeros(need // 4 + 4, dtype=torch.int32, device=self.dev)
        return self._scratch

    def _apply_choice(self, c, choice):
        """Tuning-table value = tile config + 100 * splitk (splitk 0/1 = no split).  A split
        call gets its own zero-filled workspace, kept alive by the call."""
        d = c.desc
        d.config, sk = choice % 100, choice // 100
        if sk > 1:
            ops.set_splitk(d, sk)
            ws = ops.splitk_workspace(d, self.dev)
            ops.set_splitk(d, sk, ws)
            c.keep = tuple(c.keep or ()) + (ws,)
        else:
            ops.set_splitk(d, 0)

    def autotune(self, reps=5, table=None, save=None, cold=False):
        """Pick the fastest (tile config, split-K) for every prepared GEMM by timing
        them in place (HIP events).  Tile configs differ only in speed: each output
        element is accumulated in the same K order whatever the tile.  Split-K
        (tried only for grids < 512 tiles) re-associates the K sum in a fixed slice
        order, so a given choice is deterministic; DP ranks stay in lockstep either
        way because they apply the same all-reduced gradient.  The committed table
        (`table`) pins the choices of known shapes.  Run after a batch is loaded and
        one forward/backward has filled the activations; it scribbles only on
        buffers the next step recomputes.

        cold: time every candidate from cold caches (a 512 MiB write evicts L2 and the
        Infinity Cache before each timed launch), as the launches run inside the step,
        where operands were written by another kernel or last read a step ago; warm
        back-to-back replays favour shallow rings.  Uses (and fills) its own cache."""
        import json
        import os
        cache = _TUNE_CACHE_COLD if cold else _TUNE_CACHE
        if table and os.path.exists(table):                # measured table (tools: bench --tune-save)
            for k, v in json.load(open(table)).items():
                cache.setdefault(k, int(v))
        s = L.stream_handle()
        lib = L.load()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        flush = torch.empty(128 << 20, dtype=torch.float32, device=self.dev) if cold else None
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]

        def time_call(c):
            c(s)
            if not cold:
                st.record()
                for _ in range(reps):
                    c(s)
                en.record()
                en.synchronize()
                return st.elapsed_time(en)
            for a, b in evs:
                flush.fill_(1.0)
                a.record()
                c(s)
                b.record()
            evs[-1][1].synchronize()
            return sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]
        chosen = {}
        timed = []                                         # shapes not in the table: timed here
        extra = self.res_calls if self.pipeline else []
        for c in extra + self.fwd_calls + self.bwd_calls:
            if c.name == "vqa_gemm_pair":
                d1, d2 = c.desc
                key = repr(("pair", _gemm_key(d1), _gemm_key(d2)))
                if key not in cache:
                    timed.append(key)
                    best = None
                    for c1 in (3, 4, 6, 7):
                        for c2 in (3, 4, 6, 7):
                            d1.config, d2.config = c1, c2
                            t = time_call(c)
                            if best is None or t < best[0]:
                                best = (t, c1 * 10 + c2)
                    cache[key] = best[1]
                d1.config, d2.config = cache[key] // 10, cache[key] % 10
                chosen[key] = cache[key]
                continue
            if c.name != "vqa_gemm" or c.desc.relu >= 2:        # GELU / tanh: one fixed kernel
                continue
            d = c.desc
            key = repr(_gemm_key(d))
            if key not in cache:
                timed.append(key)
                best = None
                nk = -(-d.k // 64)
                for cfg in range(1, lib_gemm_configs() + 1):
                    if (cfg in L.GEMM_KC_B_ONLY and d.b_trans) or ((cfg in L.GEMM_PATCH_ONLY) != (d.a_conv == 2)):
                        continue
                    if d.fp8 and cfg not in L.GEMM_FP8:
                        continue
                    bm, bn, _ = L.GEMM_TILES[cfg]
                    tiles = -(-d.m // bm) * -(-d.n // bn) * max(1, d.batch)
                    if cfg in L.GEMM_BK128 and (d.a_conv or d.b_conv):
                        continue                           # 128-deep k-tiles: plain operands only
                    if cfg in L.GEMM_K64_ONLY and (d.k > 64 or d.a_conv or d.b_conv):
                        continue                           # one k-tile, plain operands only
                    for sk in SPLITS:
                        # split only grids that leave CUs idle, with >= 2 k-tiles per slice
                        if sk > 1 and (tiles >= 512 or nk < 2 * sk or tiles > 16384 or d.a_conv == 2
                                       or cfg in L.GEMM_BK128 or cfg in L.GEMM_K64_ONLY):
                            continue
                        d.config = cfg
                        ops.set_splitk(d, sk)
                        ops.set_splitk(d, sk, self._tune_scratch(d) if sk > 1 else None)
                        t = time_call(c)
                        if best is None or t < best[0]:
                            best = (t, cfg + 100 * sk)
                ops.set_splitk(d, 0)
                cache[key] = best[1]
            self._apply_choice(c, cache[key])
            chosen[key] = cache[key]
        torch.cuda.synchronize(self.dev)
        if timed:
            import sys
            print(f"autotune: {len(timed)} GEMM shapes not in the table, timed at start-up "
                  f"(their choice, and with split-K the rounding, can vary by box): {timed}", file=sys.stderr)
        self._scratch = None
        self.graph = None
        if save:
            json.dump(dict(sorted(chosen.items())), open(save, "w"), indent=0)
        return chosen

    # ------------------------------------------------------------------ readouts (tests / API)
    def forward_backward(self, batch):
        self.load_batch(batch)
        self.forward()
        self.backward()
        torch.cuda.synchronize(self.dev)
        return self.LOGP[:self.rows].cpu().numpy(), float(self.LOSS.item())

    def log_probs(self):
        return self.LOGP[:self.rows]

    def loss(self):
        return self.LOSS

    def grad_norm(self):
        return float(self.G32.double().norm()) * self.grad_scale

    def group_grad_norms(self):
        out = {}
        for g, (a, e) in self.lay.groups.items():
            out[g] = float(self.G32[a:e].double().norm()) * self.grad_scale
        return out

    def last_grad_norm(self):
        return float(self.opt_state[L.ST_GRAD_NORM].item())

    def state_dict(self):
        """Reference-layout state_dict (SURVEY Appendix B keys), fp32 numpy."""
        self.flush_optimizer()
        sd = dict(self._frozen)
        sd.update(self.lay.unpack(self.P32.cpu().numpy()))
        specs = S.model_specs(self.vision, self.A, self.NB, self.dims)
        return {k: sd[k] for k in specs}

    def optimizer_state(self):
        """AdamW(amsgrad) state in reference layout: ({key: exp_avg}, {key: exp_avg_sq},
        {key: max_exp_avg_sq}, step, dropout RNG {seed, counter, training}).  The pending
        deferred update is applied first, as state_dict() does."""
        self.flush_optimizer()
        torch.cuda.synchronize(self.dev)
        unpack = lambda t: self.lay.unpack(t.cpu().numpy())
        return (unpack(self.M), unpack(self.V), unpack(self.VMAX), float(self.opt_state[L.ST_STEP].item()),
                self.RNG.cpu().numpy().copy())

    def load_optimizer_state(self, exp_avg, exp_avg_sq, max_exp_avg_sq, step, rng=None):
        """Restore what optimizer_state() returned (keys missing from the dicts: zero state)."""
        self.flush_optimizer()
        zeros = {k: np.zeros(sg, np.float32) for k, sg in S.model_specs(self.vision, self.A, self.NB, self.dims).items()
                 if k in set(self.lay.trainable_keys)}
        for arena, st in ((self.M, exp_avg), (self.V, exp_avg_sq), (self.VMAX, max_exp_avg_sq)):
            full = dict(zeros)
            full.update({k: np.asarray(v, np.float32) for k, v in st.items() if k in full})
            arena.copy_(torch.from_numpy(self.lay.pack(full)))
        self.opt_state.zero_()
        self.opt_state[L.ST_STEP] = float(step)
        if rng is not None:
            self.RNG.copy_(torch.as_tensor(np.asarray(rng).astype(np.uint32).view(np.int32)))
        torch.cuda.synchronize(self.dev)

    def segment_grad(self, name):
        return self.g32[name]

    def param_view(self, key):
        """(parameter, gradient) device views of reference state-dict entry `key` inside the
        flat fp32 arenas (no copy: they alias the engine's live weights / gradients).  The
        q|k|v and k|v stacks are row blocks, so their parts are exact reference-shaped views;
        the ConvTranspose2d scaler is stored as the flipped conv weight, so its view has the
        kernel layout [768, 3, 3, Cin] (layout.py).  None if `key` is not trainable here."""
        specs = S.model_specs(self.vision, self.A, self.NB, self.dims)
        for sg in self.lay.segments.values():
            if key not in sg.parts:
                continue
            p32, g32 = self.p32[sg.name], self.g32[sg.name]
            if sg.kind == "convT":
                return p32, g32
            if sg.kind == "flat":
                return p32.view(specs[key]), g32.view(specs[key])
            row = 0
            for part in sg.parts:
                n = specs[part][0]
                if part == key:
                    return p32[row:row + n].view(specs[key]), g32[row:row + n].view(specs[key])
                row += n
        return None

    def refresh_shadow(self):
        """Re-derive the bf16 GEMM shadow from the fp32 masters (after writing weights through
        param_view / ParameterGroup views)."""
        self.P16.copy_(self.P32)
        self._run(self.quant_all)

    def layer4_features(self):
        """The frozen ResNet's layer4 map of the current batch as NCHW fp32 (the kernels keep
        it NHWC bf16): the `features` generate_answers returns (resnet_vqa_model.py:186-203)."""
        return self.F4[:self.rows].permute(0, 3, 1, 2).float()
