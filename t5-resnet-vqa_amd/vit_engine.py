"""`VitVQAEngine` -- one training step of BASELINE config 4, the reference's
`VitVQAModel` (model/vit_vqa_model.py:127-227) trained by the ViT trainer
(trainer/vit_vqa_trainer.py:450-464: zero_grad -> forward -> backward ->
clip_grad_norm_ -> AdamW(amsgrad) -> sched), as a static schedule of the C-ABI
kernels over flat fp32 arenas, replayed as one hipGraph.

Forward (:166-225):
  * frozen ViT-base under no_grad (:183-186): patch im2col + GEMM (+ bias, + position
    embeddings as a broadcast residual) into rows 1..196 of each image, the CLS +
    position row scattered into row 0; 12 pre-LN layers (LayerNorm eps 1e-12,
    q|k|v GEMM with bias, the long-sequence MFMA attention, output GEMM + residual,
    LayerNorm, GELU GEMM, GEMM + residual); final LayerNorm and tanh pooler on the
    CLS rows only (the pooler reads nothing else);
  * T5 encoder as in the ResNet path; its CLS rows (encoder_outputs[:, 0, :], :189)
    and the pooled ViT output are the fusing layer's concat (:192-195);
  * fusing_layer: Linear(1536, 768) + ReLU + Dropout(0.5), one GEMM (:198);
  * T5 decoder (:199-205) over the ONE fused token: causal self-attention with the
    decoder's unidirectional relative bias (bucket -1 = finfo.min), cross-attention
    whose softmax over a single key is 1 (context = dropout(1) * v: vqa_xattn1_fwd;
    the 12 layers' value projections of the fused token are one GEMM), ReLU FF;
  * answer token = the last position with decoder mask 1 (:208-212), classifier +
    log_softmax + NLL (the head kernel with a length-1 pooler, whose softmax is 1).
Backward: the reverse schedule; the cross-attention q / k projections and the cross
layer norm get exactly zero gradients (softmax over one key is constant), computed as
such (the norm backward runs with dy = 0); the shared embedding table gets the encoder
and decoder token rows in one deterministic scatter.
Dropout: the counter-hash masks of the ResNet path (p = 0.1 at the T5 sites, 0.5 at
the fusing layer); the oracle (oracle/vit_oracle.py) restates the same sites.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import lib as L
from . import ops
from . import synthetic as S
from . import vit_model as VM
from .engine import (BF16, F32, I64, IGNORE_INDEX, SITE_EMBED, SITE_FINAL, VQAEngine, batch_rows, load_rows,
                     no_gc_capture, t5_site)
from .layout import t5_bucket_map

D = S.D_MODEL
NL, H5, DKV, DFF = S.T5_LAYERS, S.T5_HEADS, S.T5_DKV, S.T5_DFF
SITE_DEC_EMBED, SITE_DEC_FINAL, SITE_FUSE = 3, 4, 5


def dec_site(layer, kind):
    """kind 0 self probs, 1 self branch, 2 cross probs, 3 cross branch, 4 FF inner, 5 FF branch."""
    return 256 + 8 * layer + kind


class VitVQAEngine:
    # the call helpers, tuner and dropout plumbing are the ResNet engine's
    _t = VQAEngine._t
    _gemm = VQAEngine._gemm
    _call = VQAEngine._call
    _attn = VQAEngine._attn
    _drop = VQAEngine._drop
    _dptr = VQAEngine._dptr
    drop_scale = VQAEngine.drop_scale
    _linear = VQAEngine._linear
    _dx = VQAEngine._dx
    _defer = VQAEngine._defer
    _flush = VQAEngine._flush
    _run = VQAEngine._run
    set_training = VQAEngine.set_training
    autotune = VQAEngine.autotune
    _apply_choice = VQAEngine._apply_choice
    _tune_scratch = VQAEngine._tune_scratch
    last_grad_norm = VQAEngine.last_grad_norm

    def __init__(self, state_dict, batch=64, seq_len=32, dec_len=VM.DEC_LEN, image_size=VM.VIT_IMAGE,
                 device="cuda:0", warmup=10, total=100, answer_spaces=170, max_norm=1.0, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.1, dropout=0.1, seed=0, group_lr=None):
        L.load()
        if not 1 <= answer_spaces <= 1024:
            raise ValueError(f"answer_spaces={answer_spaces}: the fused answer head supports 1..1024 answers")
        if not (1 <= seq_len <= 32 and 1 <= dec_len <= 32):
            raise ValueError("seq_len and dec_len must be in 1..32 (one 32-query MFMA attention tile)")
        if image_size % VM.VIT_PATCH:
            raise ValueError(f"image_size must be a multiple of {VM.VIT_PATCH}")
        self.dev = torch.device(device)
        self.B, self.L, self.Ld, self.H = batch, seq_len, dec_len, image_size
        self.T, self.TD = batch * seq_len, batch * dec_len
        self.rows = batch                 # real rows of the loaded batch (a short last batch is padded)
        self.NV = VM.vit_tokens(image_size)
        self.TV = batch * self.NV
        self.A = answer_spaces
        self.p_drop, self.seed = float(dropout), int(seed)
        self.warmup, self.total, self.max_norm = warmup, total, max_norm
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.grad_scale = 1.0
        self.group_lr = dict(group_lr or {})
        self.pipeline, self.res_calls, self.pair_bwd = False, [], False
        self.lay = VM.VitLayout(answer_spaces)
        sd = {k: np.asarray(v) for k, v in state_dict.items()}
        self._frozen = {k: v for k, v in sd.items() if k.startswith("vision_model.")}
        self._jobs = []
        with torch.cuda.device(self.dev):
            self._alloc_params(sd)
            self._alloc_vit(sd)
            self._alloc_activations()
            self.fwd_calls, self.bwd_calls, self.opt_calls = [], [], []
            self._plan_forward()
            self._plan_backward()
            self._plan_optimizer()
        self.graph = None
        self._scratch = None

    # ------------------------------------------------------------------ allocation
    def _alloc_params(self, sd):
        lay = self.lay
        self.P32 = torch.from_numpy(lay.pack(sd)).to(self.dev)
        self.P16 = self.P32.to(BF16)
        self.G32, self.M, self.V, self.VMAX = (self._t(lay.total, zero=True) for _ in range(4))
        self.p32, self.p16, self.g32 = {}, {}, {}
        for s in lay.segments.values():
            sl = slice(s.offset, s.offset + s.numel)
            self.p32[s.name] = self.P32[sl].view(s.shape)
            self.p16[s.name] = self.P16[sl].view(s.shape)
            self.g32[s.name] = self.G32[sl].view(s.shape)
        self.opt_state = self._t(L.ST_FLOATS, zero=True)
        self.RNG = torch.from_numpy(np.array([self.seed & 0xFFFFFFFF, 0, 1, 0], np.uint32).view(np.int32)).to(self.dev)
        self.bucket_e = torch.from_numpy(t5_bucket_map(self.L, self.L)).reshape(-1).to(self.dev)
        self.bucket_d = torch.from_numpy(VM.causal_bucket_map(self.Ld)).reshape(-1).to(self.dev)

    def _alloc_vit(self, sd):
        """Frozen ViT weights: bf16 GEMM operands, fp32 biases / norms (not in the arena)."""
        dev = self.dev
        f32 = lambda k: torch.from_numpy(np.ascontiguousarray(sd["vision_model." + k], np.float32)).to(dev)
        b16 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev).to(BF16)
        e = "embeddings."
        self.vw = {"patch_w": b16(sd["vision_model." + e + "patch_embeddings.projection.weight"].reshape(D, -1)),
                   "patch_b": f32(e + "patch_embeddings.projection.bias")}
        cls = np.asarray(sd["vision_model." + e + "cls_token"], np.float32).reshape(D)
        pos = np.asarray(sd["vision_model." + e + "position_embeddings"], np.float32).reshape(self.NV, D)
        self.vw["clspos"] = torch.from_numpy((cls + pos[0]).astype(np.float32)).to(dev)   # torch adds in fp32
        self.vw["pos"] = torch.from_numpy(np.ascontiguousarray(pos[1:])).to(dev)
        for i in range(VM.VIT_LAYERS):
            p = f"encoder.layer.{i}."
            a = p + "attention.attention."
            self.vw[f"{i}.qkv_w"] = b16(np.concatenate([sd["vision_model." + a + n + ".weight"]
                                                        for n in ("query", "key", "value")]))
            self.vw[f"{i}.qkv_b"] = torch.cat([f32(a + n + ".bias") for n in ("query", "key", "value")])
            self.vw[f"{i}.o_w"] = b16(sd["vision_model." + p + "attention.output.dense.weight"])
            self.vw[f"{i}.o_b"] = f32(p + "attention.output.dense.bias")
            self.vw[f"{i}.fc1_w"] = b16(sd["vision_model." + p + "intermediate.dense.weight"])
            self.vw[f"{i}.fc1_b"] = f32(p + "intermediate.dense.bias")
            self.vw[f"{i}.fc2_w"] = b16(sd["vision_model." + p + "output.dense.weight"])
            self.vw[f"{i}.fc2_b"] = f32(p + "output.dense.bias")
            for n, k in (("ln1", "layernorm_before"), ("ln2", "layernorm_after")):
                self.vw[f"{i}.{n}_g"], self.vw[f"{i}.{n}_b"] = f32(p + k + ".weight"), f32(p + k + ".bias")
        self.vw["lnf_g"], self.vw["lnf_b"] = f32("layernorm.weight"), f32("layernorm.bias")
        self.vw["pool_w"] = b16(sd["vision_model.pooler.dense.weight"])
        self.vw["pool_b"] = f32("pooler.dense.bias")

    def _alloc_activations(self):
        B, Lq, Ld, T, TD, TV = self.B, self.L, self.Ld, self.T, self.TD, self.TV
        t = self._t
        self.PIX = t((B, 3, self.H, self.H), zero=True)
        self.IDS_ALL = t(T + TD, I64, zero=True)                   # encoder then decoder token ids
        self.IDS_PREV = t(T + TD, I64, zero=True)
        self.IDS, self.DIDS = self.IDS_ALL[:T].view(B, Lq), self.IDS_ALL[T:].view(B, Ld)
        self.MASK, self.DMASK = t((B, Lq), I64, zero=True), t((B, Ld), I64, zero=True)
        self.TGT = t((B,), I64, zero=True)
        # ViT
        self.XP16 = t((B * (self.NV - 1), D), BF16)
        self.VH32, self.VLN16 = t((TV, D)), t((TV, D), BF16)
        self.VMU, self.VRS = t(TV), t(TV)
        self.VQKV16, self.VO16, self.VFF16 = t((TV, 3 * D), BF16), t((TV, D), BF16), t((TV, VM.VIT_FF), BF16)
        self.VCLS32, self.VCLSN16, self.VCMU, self.VCRS = t((B, D)), t((B, D), BF16), t(B), t(B)
        self.CAT16, self.FUSED16 = t((B, 2 * D), BF16), t((B, D), BF16)
        self.VALL16 = t((B, NL * D), BF16)
        # T5 encoder
        self.PB_e = t((H5, Lq, Lq))
        self.HS_e = [t((T, D)) for _ in range(NL + 1)]
        self.N0_e, self.O_e, self.N1_e = ([t((T, D), BF16) for _ in range(NL)] for _ in range(3))
        self.QKV_e = [t((T, 3 * D), BF16) for _ in range(NL)]
        self.PT_e = [t((B, H5, Lq, Lq)) for _ in range(NL)]
        self.HM_e = [t((T, D)) for _ in range(NL)]
        self.FF_e = [t((T, DFF), BF16) for _ in range(NL)]
        self.R0_e, self.R1_e = [t(T) for _ in range(NL)], [t(T) for _ in range(NL)]
        self.RF_e, self.TXT32, self.TXT16 = t(T), t((T, D)), t((T, D), BF16)
        # T5 decoder
        self.PB_d = t((H5, Ld, Ld))
        self.HS_d = [t((TD, D)) for _ in range(NL + 1)]
        self.N0_d, self.O_d, self.CTX_d, self.N2_d = ([t((TD, D), BF16) for _ in range(NL)] for _ in range(4))
        self.QKV_d = [t((TD, 3 * D), BF16) for _ in range(NL)]
        self.PT_d = [t((B, H5, Ld, Ld)) for _ in range(NL)]
        self.HM_d, self.HX_d = [t((TD, D)) for _ in range(NL)], [t((TD, D)) for _ in range(NL)]
        self.FF_d = [t((TD, DFF), BF16) for _ in range(NL)]
        self.R0_d, self.R2_d = [t(TD) for _ in range(NL)], [t(TD) for _ in range(NL)]
        self.RF_d, self.DEC32, self.DEC16 = t(TD), t((TD, D)), t((TD, D), BF16)
        # answer gather + head (the pooler of the head kernel over a length-1 sequence: identity)
        self.LASTIDX, self.ANS32 = t(B, I64, zero=True), t((B, D))
        self.DUMMY_PW, self.DUMMY_PB = t(D, zero=True), t(1, zero=True)
        self.DUMMY_GPW, self.DUMMY_GPB = t(D, zero=True), t(1, zero=True)
        self.ATT, self.POOLED = t((B, 1)), t((B, D))
        self.LOGP, self.NLL, self.LOSS = t((B, self.A)), t(B), t(1)
        # backward
        mx = max(T, TD)
        self.dH32_ALL = t((T + TD, D), zero=True)                  # embedding-row gradients, enc then dec
        self.dH32_e, self.dH32_d = self.dH32_ALL[:T], self.dH32_ALL[T:]
        self.dANS32, self.dDEC32, self.dTXT32 = t((B, D)), t((TD, D), zero=True), t((T, D), zero=True)
        self.dC32, self.dR32, self.dX32 = t((mx, D)), t((mx, D)), t((mx, D))
        self.ZERO32 = t((TD, D), zero=True)
        self.dH16 = [t((mx, D), BF16), t((mx, D), BF16)]
        self.dB16, self.dF16, self.dO16 = t((mx, D), BF16), t((mx, DFF), BF16), t((mx, D), BF16)
        self.dQKV16 = t((mx, 3 * D), BF16)
        self.dVALL16, self.dPRE16, self.dCLS32 = t((B, NL * D), BF16), t((B, D), BF16), t((B, D))
        self.dSB_e, self.dSB_d = t((NL, B, H5, Lq, Lq)), t((NL, B, H5, Ld, Ld))
        self.dPB_e, self.dPB_d = t((H5, Lq, Lq)), t((H5, Ld, Ld))
        lib = L.load()
        self.WS_EMB = t(3 * min(T + TD, 16384), torch.int32)
        self.WS_HEAD = t(lib.vqa_head_workspace_floats(B, 1, D, self.A))
        self.SQ_PARTS = 1024
        self.WS_SQ = t(self.SQ_PARTS, torch.float64)

    def _nws(self, rows):
        return self._t(L.load().vqa_norm_bwd_workspace_floats(rows, D))

    def _dw(self, lst, dy16, x16, wname, rows, bias_from=None):
        """dW[n, k] = dY[rows, n]^T X[rows, k] (+ bias = column sums of dY, deferred)."""
        g = self.g32[wname]
        n, k = g.shape
        self._gemm(lst, dy16, x16, n, k, rows, lda=dy16.shape[-1], ldb=x16.shape[-1], a_trans=True, b_trans=True,
                   c32=g, ldc32=k)
        if bias_from is not None:
            lib = L.load()
            ws = self._t(lib.vqa_colsum_workspace_floats(rows, n))
            self._call(lst, "vqa_colsum", bias_from, 1, rows, n, n, None, 0.0, ws)
            self._defer(ws, lib.vqa_colsum_parts(rows), n, n, self.g32[wname[:-1] + "b"])

    # ------------------------------------------------------------------ forward
    def _plan_forward(self):
        f = self.fwd_calls
        self._vit_attn_at, self.ATT_MAPS, self._probs_calls = [], None, None
        B, Lq, Ld, T, TD, TV, NV = self.B, self.L, self.Ld, self.T, self.TD, self.TV, self.NV
        vw = self.vw
        if self.p_drop > 0.0:
            self._call(f, "vqa_rng_advance", self.RNG)
        # ---- frozen ViT (ViTEmbeddings + 12 ViTLayer + layernorm + pooler)
        self._call(f, "vqa_vit_patchify", self.PIX, self.XP16, B, self.H, self.H, VM.VIT_PATCH)
        npch = NV - 1
        self._gemm(f, self.XP16, vw["patch_w"], npch, D, D, lda=D, ldb=D, c32=ops.addr(self.VH32, D), ldc32=D,
                   bias=vw["patch_b"], res32=vw["pos"], ldres=D, batch=B, stride_a=npch * D, stride_b=0,
                   stride_c32=NV * D, stride_res=0, keep=(self.VH32,))
        self._call(f, "vqa_scatter_rows", vw["clspos"], 0, None, NV, 0, self.VH32, D, B, D, 4)
        for i in range(VM.VIT_LAYERS):
            self._call(f, "vqa_layernorm_fwd", self.VH32, vw[f"{i}.ln1_g"], vw[f"{i}.ln1_b"], None, self.VLN16,
                       self.VMU, self.VRS, TV, D, VM.VIT_EPS)
            self._gemm(f, self.VLN16, vw[f"{i}.qkv_w"], TV, 3 * D, D, lda=D, ldb=D, c16=self.VQKV16, ldc16=3 * D,
                       bias=vw[f"{i}.qkv_b"])
            q = self.VQKV16
            self._attn(f, "vqa_attn_fwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, o=self.VO16, ldo=D, batch=B, heads=VM.VIT_HEADS, lq=NV, lk=NV, dh=VM.VIT_DH,
                       scale=VM.VIT_DH ** -0.5, keep=(q,))
            self._vit_attn_at.append(len(f))               # where forward_with_attentions reads layer i's P
            self._gemm(f, self.VO16, vw[f"{i}.o_w"], TV, D, D, lda=D, ldb=D, c32=self.VH32, ldc32=D,
                       bias=vw[f"{i}.o_b"], res32=self.VH32, ldres=D)
            self._call(f, "vqa_layernorm_fwd", self.VH32, vw[f"{i}.ln2_g"], vw[f"{i}.ln2_b"], None, self.VLN16,
                       self.VMU, self.VRS, TV, D, VM.VIT_EPS)
            self._gemm(f, self.VLN16, vw[f"{i}.fc1_w"], TV, VM.VIT_FF, D, lda=D, ldb=D, c16=self.VFF16,
                       ldc16=VM.VIT_FF, bias=vw[f"{i}.fc1_b"], relu=2)
            self._gemm(f, self.VFF16, vw[f"{i}.fc2_w"], TV, D, VM.VIT_FF, lda=VM.VIT_FF, ldb=VM.VIT_FF,
                       c32=self.VH32, ldc32=D, bias=vw[f"{i}.fc2_b"], res32=self.VH32, ldres=D)
        # the pooler reads only the CLS rows: final LayerNorm of those rows, then dense + tanh
        self._call(f, "vqa_gather_rows", self.VH32, D, None, NV, 0, self.VCLS32, D, B, D, 4)
        self._call(f, "vqa_layernorm_fwd", self.VCLS32, vw["lnf_g"], vw["lnf_b"], None, self.VCLSN16, self.VCMU,
                   self.VCRS, B, D, VM.VIT_EPS)
        self._gemm(f, self.VCLSN16, vw["pool_w"], B, D, D, lda=D, ldb=D, c16=self.CAT16, ldc16=2 * D,
                   bias=vw["pool_b"], relu=3)
        self.vit_calls = len(f)
        # ---- T5 encoder (the ResNet path's plan, config-4 arena names)
        self._t5_forward(f, "enc", self.IDS, self.MASK, T, Lq, self.HS_e, self.N0_e, self.QKV_e, self.PT_e, self.O_e,
                         self.HM_e, self.N1_e, self.FF_e, self.R0_e, self.R1_e, self.PB_e, self.bucket_e)
        kp = []
        self._call(f, "vqa_rmsnorm_fwd", self.HS_e[-1], self.p32["enc.final_ln"], self.TXT32, self.TXT16, self.RF_e,
                   T, D, 1e-6, self._dptr(SITE_FINAL, kp), extra=kp + [self.RNG])
        # encoder_outputs[:, 0, :] -> right half of the fusing layer's input
        self._call(f, "vqa_gather_rows", self.TXT16, D, None, Lq, 0, ops.addr(self.CAT16, D), 2 * D, B, D, 2,
                   extra=[self.CAT16])
        # fusing_layer: dropout(0.5)(relu(W [pooled | cls] + b))
        self._gemm(f, self.CAT16, self.p16["fuse_w"], B, D, 2 * D, lda=2 * D, ldb=2 * D, c16=self.FUSED16, ldc16=D,
                   bias=self.p32["fuse_b"], relu=True)
        if self.p_drop > 0.0:
            f[-1].desc.drop = L.Dropout(VM.FUSE_P, SITE_FUSE, self.RNG.data_ptr())
            f[-1].keep = f[-1].keep + (self.RNG,)
        # the 12 decoder layers' cross-attention values of the single fused token: one GEMM
        self._gemm(f, self.FUSED16, self.p16["dec.xv_w"], B, NL * D, D, lda=D, ldb=D, c16=self.VALL16,
                   ldc16=NL * D)
        # ---- T5 decoder
        kp = []
        self._call(f, "vqa_embedding_fwd", self.DIDS, self.p32["embed"], self.HS_d[0], TD, D, S.T5_VOCAB,
                   self._dptr(SITE_DEC_EMBED, kp), extra=kp + [self.RNG])
        self._call(f, "vqa_t5_relbias_fwd", self.p32["dec.relbias"], self.bucket_d, self.PB_d, H5, Ld, Ld)
        for i in range(NL):
            p = f"dec.{i}."
            self._call(f, "vqa_rmsnorm_fwd", self.HS_d[i], self.p32[p + "ln0"], None, self.N0_d[i], self.R0_d[i],
                       TD, D, 1e-6, None)
            self._linear(f, self.N0_d[i], p + "qkv_w", TD, out16=self.QKV_d[i], bias=False)
            q = self.QKV_d[i]
            self._attn(f, "vqa_attn_fwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, o=self.O_d[i], ldo=D, p=self.PT_d[i], bias=self.PB_d, key_mask=self.DMASK, batch=B,
                       heads=H5, lq=Ld, lk=Ld, dh=DKV, scale=1.0, drop=dec_site(i, 0))
            self._linear(f, self.O_d[i], p + "o_w", TD, out32=self.HM_d[i], bias=False, res32=self.HS_d[i],
                         drop=dec_site(i, 1))
            kp = []
            self._call(f, "vqa_xattn1_fwd", ops.addr(self.VALL16, i * D), NL * D, self.CTX_d[i], D, B, Ld, H5, DKV,
                       self._dptr(dec_site(i, 2), kp), extra=kp + [self.VALL16, self.RNG])
            self._linear(f, self.CTX_d[i], p + "xo_w", TD, out32=self.HX_d[i], bias=False, res32=self.HM_d[i],
                         drop=dec_site(i, 3))
            self._call(f, "vqa_rmsnorm_fwd", self.HX_d[i], self.p32[p + "ln2"], None, self.N2_d[i], self.R2_d[i],
                       TD, D, 1e-6, None)
            self._linear(f, self.N2_d[i], p + "wi", TD, out16=self.FF_d[i], bias=False, relu=True,
                         drop=dec_site(i, 4))
            self._linear(f, self.FF_d[i], p + "wo", TD, out32=self.HS_d[i + 1], bias=False, res32=self.HX_d[i],
                         drop=dec_site(i, 5))
        kp = []
        self._call(f, "vqa_rmsnorm_fwd", self.HS_d[-1], self.p32["dec.final_ln"], self.DEC32, self.DEC16, self.RF_d,
                   TD, D, 1e-6, self._dptr(SITE_DEC_FINAL, kp), extra=kp + [self.RNG])
        # the answer token (last position of the decoder mask), classifier, log_softmax, NLL
        self._call(f, "vqa_last_index", self.DMASK, B, Ld, self.LASTIDX)
        self._call(f, "vqa_gather_rows", self.DEC32, D, self.LASTIDX, 0, 0, self.ANS32, D, B, D, 4)
        self._call(f, "vqa_head_fwd", self.ANS32, self.DUMMY_PW, self.DUMMY_PB, self.p32["cls_w"], self.p32["cls_b"],
                   self.TGT, self.ATT, self.POOLED, self.LOGP, self.NLL, self.LOSS, B, 1, D, self.A)

    def _t5_forward(self, f, pre, ids, mask, T, Lq, HS, N0, QKV, PT, O, HM, N1, FF, R0, R1, PB, bucket):
        B = self.B
        kp = []
        self._call(f, "vqa_embedding_fwd", ids, self.p32["embed"], HS[0], T, D, S.T5_VOCAB, self._dptr(SITE_EMBED, kp),
                   extra=kp + [self.RNG])
        self._call(f, "vqa_t5_relbias_fwd", self.p32[pre + ".relbias"], bucket, PB, H5, Lq, Lq)
        for i in range(NL):
            p = f"{pre}.{i}."
            self._call(f, "vqa_rmsnorm_fwd", HS[i], self.p32[p + "ln0"], None, N0[i], R0[i], T, D, 1e-6, None)
            self._linear(f, N0[i], p + "qkv_w", T, out16=QKV[i], bias=False)
            q = QKV[i]
            self._attn(f, "vqa_attn_fwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, o=O[i], ldo=D, p=PT[i], bias=PB, key_mask=mask, batch=B, heads=H5, lq=Lq, lk=Lq,
                       dh=DKV, scale=1.0, drop=t5_site(i, 0))
            self._linear(f, O[i], p + "o_w", T, out32=HM[i], bias=False, res32=HS[i], drop=t5_site(i, 1))
            self._call(f, "vqa_rmsnorm_fwd", HM[i], self.p32[p + "ln1"], None, N1[i], R1[i], T, D, 1e-6, None)
            self._linear(f, N1[i], p + "wi", T, out16=FF[i], bias=False, relu=True, drop=t5_site(i, 2))
            self._linear(f, FF[i], p + "wo", T, out32=HS[i + 1], bias=False, res32=HM[i], drop=t5_site(i, 3))

    # ------------------------------------------------------------------ backward
    def _plan_backward(self):
        b = self.bwd_calls
        B, Lq, Ld, T, TD = self.B, self.L, self.Ld, self.T, self.TD
        ks = self.drop_scale if self.p_drop > 0.0 else 1.0
        z = self.g32["embed"]
        self._call(b, "vqa_embedding_zero_rows", self.IDS_PREV, self.IDS_ALL, T + TD, z, D, S.T5_VOCAB)
        self._call(b, "vqa_head_bwd", self.ANS32, self.ATT, self.POOLED, self.LOGP, self.TGT, self.DUMMY_PW,
                   self.p32["cls_w"], self.dANS32, None, self.DUMMY_GPW, self.DUMMY_GPB, self.g32["cls_w"],
                   self.g32["cls_b"], self.WS_HEAD, B, 1, D, self.A, None, None, None, 1.0)
        # the answer rows move with the batch's decoder masks: clear last step's rows first
        self._call(b, "vqa_zero", self.dDEC32, TD * D * 4)
        self._call(b, "vqa_scatter_rows", self.dANS32, D, self.LASTIDX, 0, 0, self.dDEC32, D, B, D, 4)
        # ---- decoder (reverse): dH32 = gradient of the residual stream, dH16 the FF-branch gradient
        dH32, dR32 = self.dH32_d, self.dR32
        kp, ws = [], self._nws(TD)
        self._call(b, "vqa_rmsnorm_bwd", self.dDEC32, self.HS_d[-1], self.RF_d, self.p32["dec.final_ln"], None,
                   dH32, self.dH16[0], None, 0.0, ws, TD, D, self._dptr(SITE_DEC_FINAL, kp), None,
                   self._dptr(dec_site(NL - 1, 5), kp), extra=kp + [self.RNG])
        self._defer(ws, L.load().vqa_norm_bwd_parts(TD), D, D, self.g32["dec.final_ln"])
        cur = 0
        for i in reversed(range(NL)):
            p = f"dec.{i}."
            dH16 = self.dH16[cur]
            # FF sub-layer: h_out = hx + drop(wo(drop(relu(wi(rms(hx))))))
            self._dx(b, dH16[:TD], p + "wo", TD, out16=self.dF16[:TD], mask16=self.FF_d[i], alpha=ks)
            self._dw(b, dH16[:TD], self.FF_d[i], p + "wo", TD)
            self._dx(b, self.dF16[:TD], p + "wi", TD, out32=self.dC32[:TD])
            self._dw(b, self.dF16[:TD], self.N2_d[i], p + "wi", TD)
            kp, ws = [], self._nws(TD)
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HX_d[i], self.R2_d[i], self.p32[p + "ln2"], dH32,
                       self.dX32, self.dB16, None, 0.0, ws, TD, D, None, None, self._dptr(dec_site(i, 3), kp),
                       extra=kp + [self.RNG])
            self._defer(ws, L.load().vqa_norm_bwd_parts(TD), D, D, self.g32[p + "ln2"])
            # cross sub-layer: hx = hm + drop(xo(ctx)), ctx = drop(1) * v  (q, k, the cross norm: zero grads)
            self._dx(b, self.dB16[:TD], p + "xo_w", TD, out16=self.dO16[:TD])
            self._dw(b, self.dB16[:TD], self.CTX_d[i], p + "xo_w", TD)
            kp = []
            self._call(b, "vqa_xattn1_bwd", self.dO16, D, None, ops.addr(self.dVALL16, i * D), NL * D, B, Ld, H5, DKV,
                       self._dptr(dec_site(i, 2), kp), extra=kp + [self.dVALL16, self.RNG])
            kp, ws = [], self._nws(TD)
            self._call(b, "vqa_rmsnorm_bwd", self.ZERO32, self.HM_d[i], self.R0_d[i], self.p32[p + "ln1"], self.dX32,
                       dR32, self.dB16, None, 0.0, ws, TD, D, None, None, self._dptr(dec_site(i, 1), kp),
                       extra=kp + [self.RNG])
            self._defer(ws, L.load().vqa_norm_bwd_parts(TD), D, D, self.g32[p + "ln1"])
            # self-attention sub-layer
            self._dx(b, self.dB16[:TD], p + "o_w", TD, out16=self.dO16[:TD])
            self._dw(b, self.dB16[:TD], self.O_d[i], p + "o_w", TD)
            q, dq = self.QKV_d[i], self.dQKV16
            self._attn(b, "vqa_attn_bwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, p=self.PT_d[i], bias=self.PB_d, key_mask=self.DMASK, batch=B, heads=H5, lq=Ld,
                       lk=Ld, dh=DKV, scale=1.0, dout=self.dO16, lddo=D, dq=dq, lddq=3 * D, dk=ops.addr(dq, D),
                       lddk=3 * D, dv=ops.addr(dq, 2 * D), lddv=3 * D, dbias=self.dSB_d[i], drop=dec_site(i, 0),
                       keep=(dq,))
            self._dx(b, dq[:TD], p + "qkv_w", TD, out32=self.dC32[:TD])
            self._dw(b, dq[:TD], self.N0_d[i], p + "qkv_w", TD)
            kp = []
            nxt = self.dH16[1 - cur]
            d32 = self._dptr(SITE_DEC_EMBED, kp) if i == 0 else None
            d16 = self._dptr(dec_site(i - 1, 5), kp) if i > 0 else None
            ws = self._nws(TD)
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HS_d[i], self.R0_d[i], self.p32[p + "ln0"], dR32, dH32,
                       nxt if i > 0 else None, None, 0.0, ws, TD, D, None, d32, d16, extra=kp + [self.RNG])
            self._defer(ws, L.load().vqa_norm_bwd_parts(TD), D, D, self.g32[p + "ln0"])
            cur = 1 - cur
        self._call(b, "vqa_batch_sum", self.dSB_d, NL * B, H5 * Ld * Ld, self.dPB_d, 0.0)
        self._call(b, "vqa_t5_relbias_bwd", self.dPB_d, self.bucket_d, self.g32["dec.relbias"], H5, Ld, Ld,
                   S.T5_BUCKETS)
        # ---- the fused token: all layers' value projections, then the fusing layer
        ksf = (1.0 / (1.0 - VM.FUSE_P)) if self.p_drop > 0.0 else 1.0
        self._gemm(b, self.dVALL16, self.p16["dec.xv_w"], B, D, NL * D, lda=NL * D, ldb=D, b_trans=True,
                   c16=self.dPRE16, ldc16=D, mask16=self.FUSED16, ldmask=D, alpha=ksf)
        self._gemm(b, self.dVALL16, self.FUSED16, NL * D, D, B, lda=NL * D, ldb=D, a_trans=True, b_trans=True,
                   c32=self.g32["dec.xv_w"], ldc32=D)
        self._gemm(b, self.dPRE16, ops.addr(self.p16["fuse_w"], D), B, D, D, lda=D, ldb=2 * D, b_trans=True,
                   c32=self.dCLS32, ldc32=D, keep=(self.P16,))
        self._dw(b, self.dPRE16, self.CAT16, "fuse_w", B, bias_from=self.dPRE16)
        # ---- encoder: the CLS rows' gradient, final norm, layers
        self._call(b, "vqa_scatter_rows", self.dCLS32, D, None, Lq, 0, self.dTXT32, D, B, D, 4)
        self._t5_backward(b, ks)
        self._flush(b)
        self._call(b, "vqa_embedding_bwd", self.IDS_ALL, self.dH32_ALL, self.g32["embed"], T + TD, D, S.T5_VOCAB,
                   self.WS_EMB)

    def _t5_backward(self, b, ks):
        B, Lq, T = self.B, self.L, self.T
        dH32, dR32 = self.dH32_e, self.dR32
        kp, ws = [], self._nws(T)
        self._call(b, "vqa_rmsnorm_bwd", self.dTXT32, self.HS_e[-1], self.RF_e, self.p32["enc.final_ln"], None,
                   dH32, self.dH16[0], None, 0.0, ws, T, D, self._dptr(SITE_FINAL, kp), None,
                   self._dptr(t5_site(NL - 1, 3), kp), extra=kp + [self.RNG])
        self._defer(ws, L.load().vqa_norm_bwd_parts(T), D, D, self.g32["enc.final_ln"])
        cur = 0
        for i in reversed(range(NL)):
            p = f"enc.{i}."
            dH16 = self.dH16[cur]
            self._dx(b, dH16[:T], p + "wo", T, out16=self.dF16[:T], mask16=self.FF_e[i], alpha=ks)
            self._dw(b, dH16[:T], self.FF_e[i], p + "wo", T)
            self._dx(b, self.dF16[:T], p + "wi", T, out32=self.dC32[:T])
            self._dw(b, self.dF16[:T], self.N1_e[i], p + "wi", T)
            kp, ws = [], self._nws(T)
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HM_e[i], self.R1_e[i], self.p32[p + "ln1"], dH32, dR32,
                       self.dB16, None, 0.0, ws, T, D, None, None, self._dptr(t5_site(i, 1), kp),
                       extra=kp + [self.RNG])
            self._defer(ws, L.load().vqa_norm_bwd_parts(T), D, D, self.g32[p + "ln1"])
            self._dx(b, self.dB16[:T], p + "o_w", T, out16=self.dO16[:T])
            self._dw(b, self.dB16[:T], self.O_e[i], p + "o_w", T)
            q, dq = self.QKV_e[i], self.dQKV16
            self._attn(b, "vqa_attn_bwd", q=q, ldq=3 * D, k=ops.addr(q, D), ldk=3 * D, v=ops.addr(q, 2 * D),
                       ldv=3 * D, p=self.PT_e[i], bias=self.PB_e, key_mask=self.MASK, batch=B, heads=H5, lq=Lq,
                       lk=Lq, dh=DKV, scale=1.0, dout=self.dO16, lddo=D, dq=dq, lddq=3 * D, dk=ops.addr(dq, D),
                       lddk=3 * D, dv=ops.addr(dq, 2 * D), lddv=3 * D, dbias=self.dSB_e[i], drop=t5_site(i, 0),
                       keep=(dq,))
            self._dx(b, dq[:T], p + "qkv_w", T, out32=self.dC32[:T])
            self._dw(b, dq[:T], self.N0_e[i], p + "qkv_w", T)
            kp = []
            nxt = self.dH16[1 - cur]
            d32 = self._dptr(SITE_EMBED, kp) if i == 0 else None
            d16 = self._dptr(t5_site(i - 1, 3), kp) if i > 0 else None
            ws = self._nws(T)
            self._call(b, "vqa_rmsnorm_bwd", self.dC32, self.HS_e[i], self.R0_e[i], self.p32[p + "ln0"], dR32, dH32,
                       nxt if i > 0 else None, None, 0.0, ws, T, D, None, d32, d16, extra=kp + [self.RNG])
            self._defer(ws, L.load().vqa_norm_bwd_parts(T), D, D, self.g32[p + "ln0"])
            cur = 1 - cur
        self._call(b, "vqa_batch_sum", self.dSB_e, NL * B, H5 * Lq * Lq, self.dPB_e, 0.0)
        self._call(b, "vqa_t5_relbias_bwd", self.dPB_e, self.bucket_e, self.g32["enc.relbias"], H5, Lq, Lq,
                   S.T5_BUCKETS)

    # ------------------------------------------------------------------ optimizer
    def _plan_optimizer(self):
        o = self.opt_calls
        n = self.lay.total
        self._call(o, "vqa_grad_sqnorm", self.G32, n, self.WS_SQ, self.SQ_PARTS)
        self._call(o, "vqa_optim_finalize", self.WS_SQ, self.SQ_PARTS, float(self.grad_scale), float(self.max_norm),
                   int(self.warmup), int(self.total), float(self.betas[0]), float(self.betas[1]), self.opt_state)
        d = L.AdamWDesc()
        d.param, d.grad = self.P32.data_ptr(), self.G32.data_ptr()
        d.exp_avg, d.exp_avg_sq, d.max_exp_avg_sq = self.M.data_ptr(), self.V.data_ptr(), self.VMAX.data_ptr()
        d.param16 = self.P16.data_ptr()
        d.n = n
        ends, lrs = self.lay.group_of_element(self.group_lr)
        d.ngroups = len(ends)
        for i, (e, lr) in enumerate(zip(ends, lrs)):
            d.group_end[i], d.group_lr[i] = e, lr
        d.beta1, d.beta2, d.eps, d.weight_decay = self.betas[0], self.betas[1], self.eps, self.wd
        d.grad_scale = self.grad_scale
        d.state = self.opt_state.data_ptr()
        keep = (self.P32, self.G32, self.M, self.V, self.VMAX, self.P16, self.opt_state)
        # AdamW at the end of the step (a no-op unless the finalize flagged a pending update).
        # Deferring it into the next step beside the frozen ViT, which reads no trained
        # parameter, measured slower (15.1-15.4 vs 14.2 ms per step: HBM / CU contention)
        o.append(ops.Call("vqa_adamw_amsgrad", ctypes.byref(d), desc=d, keep=keep))
        self._call(o, "vqa_zero", ops.addr(self.opt_state, L.ST_PENDING), 16, extra=[self.opt_state])

    def configure_optimizer(self, group_lr=None, warmup=None, total=None, max_norm=None, weight_decay=None,
                            betas=None, eps=None):
        if group_lr:
            self.group_lr.update(group_lr)
        for name, v in (("warmup", warmup), ("total", total)):
            if v is not None:
                setattr(self, name, int(v))
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

    # ------------------------------------------------------------------ execution
    def load_batch(self, batch):
        """The ViT collate's batch dict (pixel_values, question / decoder ids and masks,
        annotation_ids), numpy or torch, host or device."""
        n = self.rows = batch_rows(batch, "question_input_ids", self.B)
        load_rows(self.PIX, batch["pixel_values"], n)
        load_rows(self.IDS, batch["question_input_ids"], n)
        load_rows(self.MASK, batch["question_attention_masks"], n)
        load_rows(self.DIDS, batch["decoder_question_input_ids"], n)
        load_rows(self.DMASK, batch["decoder_question_attention_masks"], n)
        load_rows(self.TGT, batch.get("annotation_ids"), n, fill=IGNORE_INDEX)

    def forward(self):
        self._run(self.fwd_calls)

    def forward_with_attentions(self):
        """forward() that also writes the frozen ViT's attention probabilities, HF
        ViTModel(output_attentions=True) (vit_vqa_model.py:238-240): a tuple of 12
        [B, 12, NV, NV] fp32 tensors (vqa_attn_probs after each layer's q|k|v projection; the
        buffer is allocated on the first call).  Eval readout for generate_answers."""
        B, NV = self.B, self.NV
        if self.ATT_MAPS is None:
            self.ATT_MAPS = torch.empty((VM.VIT_LAYERS, B, VM.VIT_HEADS, NV, NV), dtype=F32, device=self.dev)
            q = self.VQKV16
            self._probs_calls = []
            for i in range(VM.VIT_LAYERS):
                d = L.AttnDesc()
                d.q, d.ldq, d.k, d.ldk = ops.addr(q), 3 * D, ops.addr(q, D), 3 * D
                d.p = ops.addr(self.ATT_MAPS[i])
                d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, VM.VIT_HEADS, NV, NV, VM.VIT_DH, VM.VIT_DH ** -0.5
                self._probs_calls.append(ops.Call("vqa_attn_probs", ctypes.byref(d), desc=d, keep=(q, self.ATT_MAPS)))
        s = L.stream_handle()
        at = {k: i for i, k in enumerate(self._vit_attn_at)}
        for idx, c in enumerate(self.fwd_calls):
            c(s)
            if idx + 1 in at:
                self._probs_calls[at[idx + 1]](s)
        return tuple(self.ATT_MAPS[i] for i in range(VM.VIT_LAYERS))

    def backward(self):
        self._run(self.bwd_calls)

    def optimizer_step(self):
        self._run(self.opt_calls)

    def train_step(self):
        if self.graph is not None:
            self.graph.replay()
            return
        self.forward()
        self.backward()
        self.optimizer_step()

    def capture(self, warm=True):
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        saved, saved_rng = self.opt_state.clone(), self.RNG.clone()
        with torch.cuda.stream(s):
            if warm:
                self._run(self.fwd_calls)
                self.backward()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with no_gc_capture():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._run(self.fwd_calls)
                self.backward()
                self.optimizer_step()
        self.opt_state.copy_(saved)
        self.RNG.copy_(saved_rng)
        self.graph = g

    # ------------------------------------------------------------------ readouts
    def forward_backward(self, batch):
        self.load_batch(batch)
        self.forward()
        self.backward()
        torch.cuda.synchronize(self.dev)
        return self.LOGP[:self.rows].cpu().numpy(), float(self.LOSS.item())

    def flush_optimizer(self):
        """Nothing is deferred here: the update runs at the end of the step."""

    def grad_norm(self):
        return float(self.G32.double().norm())

    def group_grad_norms(self):
        return {g: float(self.G32[a:e].double().norm()) for g, (a, e) in self.lay.groups.items()}

    def state_dict(self):
        sd = dict(self._frozen)
        sd.update(self.lay.unpack(self.P32.cpu().numpy()))
        return {k: sd[k] for k in VM.model_specs(self.A, self.H)}

    def param_view(self, key):
        """(parameter, gradient) views of reference entry `key` in the flat arenas (the tied
        embedding keys all alias the `embed` segment); None for frozen / unknown keys."""
        specs = VM.model_specs(self.A, self.H)
        if key in VM.TIED:
            key = "lang_model.shared.weight"
        for sg in self.lay.segments.values():
            if key not in sg.parts:
                continue
            p32, g32 = self.p32[sg.name], self.g32[sg.name]
            row = 0
            for part in sg.parts:
                n = specs[part][0]
                if part == key:
                    return p32[row:row + n].view(specs[key]), g32[row:row + n].view(specs[key])
                row += n
        return None

    def refresh_shadow(self):
        self.P16.copy_(self.P32)

    def optimizer_state(self):
        """AdamW(amsgrad) state in reference layout, as VQAEngine.optimizer_state: ({key: exp_avg},
        {key: exp_avg_sq}, {key: max_exp_avg_sq}, step, dropout RNG) over the trainable keys."""
        torch.cuda.synchronize(self.dev)
        unpack = lambda t: {k: v for k, v in self.lay.unpack(t.cpu().numpy()).items() if k not in VM.TIED}  # noqa: E731
        return (unpack(self.M), unpack(self.V), unpack(self.VMAX), float(self.opt_state[L.ST_STEP].item()),
                self.RNG.cpu().numpy().copy())

    def load_optimizer_state(self, exp_avg, exp_avg_sq, max_exp_avg_sq, step, rng=None):
        """Restore what optimizer_state() returned (keys missing from the dicts: zero state)."""
        specs = VM.model_specs(self.A, self.H)
        train = [k for s_ in self.lay.segments.values() for k in s_.parts]
        zeros = {k: np.zeros(specs[k], np.float32) for k in train}
        for arena, st in ((self.M, exp_avg), (self.V, exp_avg_sq), (self.VMAX, max_exp_avg_sq)):
            full = dict(zeros)
            full.update({k: np.asarray(v, np.float32) for k, v in st.items() if k in full})
            arena.copy_(torch.from_numpy(self.lay.pack(full)))
        self.opt_state.zero_()
        self.opt_state[L.ST_STEP] = float(step)
        if rng is not None:
            self.RNG.copy_(torch.as_tensor(np.asarray(rng).astype(np.uint32).view(np.int32)))
        torch.cuda.synchronize(self.dev)

    def vit_pooled(self):
        """pooler_output of the frozen ViT for the current batch ([rows, 768], from its bf16 copy)."""
        return self.CAT16[:self.rows, :D].float()
