"""Per-kernel numerics vs a plain PyTorch fp32 reference of the same op (GPU)."""
import ctypes
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def k(pkg):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    pkg.lib.load()
    return pkg


def run(pkg, name, *args):
    pkg.ops.Call(name, *[pkg.ops.addr(a) if isinstance(a, torch.Tensor) else a for a in args])(
        pkg.lib.stream_handle())


def rnd(shape, seed, scale=1.0, dtype=torch.float32):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(shape, device="cuda", generator=g) * scale).to(dtype)


@pytest.mark.parametrize("rows", [2048, 37])
def test_rmsnorm_fwd_bwd(k, rows):
    D = 768
    x, w = rnd((rows, D), 1), 1 + 0.1 * rnd(D, 2)
    dy, dres = rnd((rows, D), 3), rnd((rows, D), 4)
    y32, y16, rstd = torch.empty_like(x), torch.empty(rows, D, device="cuda", dtype=torch.bfloat16), \
        torch.empty(rows, device="cuda")
    run(k, "vqa_rmsnorm_fwd", x, w, y32, y16, rstd, rows, D, 1e-6, None)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    ref = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6))
    ref.backward(dy)
    torch.testing.assert_close(y32, ref.detach(), rtol=1e-5, atol=1e-5)
    dx32, dx16, dw = torch.empty_like(x), torch.empty_like(y16), torch.empty(D, device="cuda")
    ws = torch.empty(k.lib.load().vqa_norm_bwd_workspace_floats(rows, D), device="cuda")
    run(k, "vqa_rmsnorm_bwd", dy, x, rstd, w, dres, dx32, dx16, dw, 0.0, ws, rows, D, None, None, None)
    torch.cuda.synchronize()
    torch.testing.assert_close(dx32, xr.grad + dres, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw, wr.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("rows", [2048, 50])
def test_layernorm_fwd_bwd(k, rows):
    D = 768
    x, g, b = rnd((rows, D), 5, 3.0) + 0.5, 1 + 0.1 * rnd(D, 6), 0.1 * rnd(D, 7)
    dy = rnd((rows, D), 8)
    y32, y16 = torch.empty_like(x), torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
    mu, rs = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    run(k, "vqa_layernorm_fwd", x, g, b, y32, y16, mu, rs, rows, D, 1e-5)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, g, b))
    ref = F.layer_norm(xr, (D,), gr, br, 1e-5)
    ref.backward(dy)
    torch.testing.assert_close(y32, ref.detach(), rtol=1e-5, atol=1e-5)
    dx, dg, db = torch.empty_like(x), torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    ws = torch.empty(k.lib.load().vqa_norm_bwd_workspace_floats(rows, D), device="cuda")
    run(k, "vqa_layernorm_bwd", dy, x, mu, rs, g, None, dx, None, dg, db, ws, rows, D, None, None)
    torch.cuda.synchronize()
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    # dres accumulates into dx32 only; the bf16 branch output and dsum are the LN gradient alone
    dres, dx16, dsum = rnd((rows, D), 9), torch.empty(rows, D, device="cuda", dtype=torch.bfloat16), \
        torch.empty(D, device="cuda")
    run(k, "vqa_layernorm_bwd", dy, x, mu, rs, g, dres, dx, dx16, dg, db, ws, rows, D, None, dsum)
    torch.cuda.synchronize()
    torch.testing.assert_close(dx, xr.grad + dres, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dx16.float(), xr.grad.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dsum, xr.grad.sum(0), rtol=1e-4, atol=1e-3)


def attn_ref(q, kk, v, scale, bias, mask, mult=None):
    s = q @ kk.transpose(-1, -2) * scale
    if bias is not None:
        s = s + bias
    if mask is not None:
        s = s + (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    p = torch.softmax(s, -1)
    return (p if mult is None else p * mult) @ v


@pytest.mark.parametrize("B,H,Lq,Lk,dh,t5,pd", [(4, 8, 32, 49, 96, False, 0.0), (4, 8, 32, 32, 96, False, 0.0),
                                                 (3, 12, 32, 32, 64, True, 0.0), (2, 8, 16, 64, 96, False, 0.0),
                                                 (2, 12, 16, 16, 64, True, 0.0), (4, 8, 32, 49, 96, False, 0.1),
                                                 (3, 12, 32, 32, 64, True, 0.1),
                                                 (2, 8, 48, 40, 96, False, 0.0),      # lq > 32: VALU kernel
                                                 (2, 12, 40, 40, 64, True, 0.1),
                                                 # more vision keys (SGA block 0 at 384^2: 12 x 12) and
                                                 # head dim 128 (d 1024 / 8 heads): one wave per block
                                                 (2, 8, 32, 144, 96, False, 0.1), (3, 8, 32, 100, 96, False, 0.0),
                                                 (2, 8, 16, 160, 128, False, 0.1), (2, 8, 32, 49, 128, False, 0.0),
                                                 (2, 16, 32, 96, 64, False, 0.0)])
def test_attention_fwd_bwd(k, B, H, Lq, Lk, dh, t5, pd):
    D = H * dh
    q16 = rnd((B * Lq, 3 * D), 10, dtype=torch.bfloat16)                   # fused qkv-like layout
    kv16 = rnd((B * Lk, 2 * D), 11, dtype=torch.bfloat16)
    do16 = rnd((B * Lq, D), 12, dtype=torch.bfloat16)
    bias = rnd((H, Lq, Lk), 13) if t5 else None
    mask = None
    if t5:
        lens = torch.tensor([Lk - 3 * i for i in range(B)], device="cuda")
        mask = (torch.arange(Lk, device="cuda")[None, :] < lens[:, None]).long()
    scale = 1.0 if t5 else 1.0 / math.sqrt(dh)
    L = k.lib
    o = torch.empty(B * Lq, D, device="cuda", dtype=torch.bfloat16)
    p = torch.empty(B, H, Lq, Lk, device="cuda")
    d = L.AttnDesc()
    A = k.ops.addr
    d.q, d.ldq, d.k, d.ldk, d.v, d.ldv = A(q16), 3 * D, A(kv16), 2 * D, A(kv16, D), 2 * D
    d.o, d.ldo, d.p = A(o), D, A(p)
    d.bias, d.key_mask = A(bias), A(mask)
    d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, H, Lq, Lk, dh, scale
    mult = None
    if pd > 0:
        from oracle import vqa_oracle as orc
        rng = torch.tensor([11, 4, 1], dtype=torch.int32, device="cuda")
        d.drop = L.Dropout(pd, 77, rng.data_ptr())
        mult = torch.from_numpy(orc.dropout_multiplier(pd, 11, 4, 77, B * H * Lq * Lk)).cuda().view(B, H, Lq, Lk)
    L.check(L.load().vqa_attn_fwd(ctypes.byref(d), L.stream_handle()), "fwd")
    qf = q16[:, :D].float().view(B, Lq, H, dh).transpose(1, 2).requires_grad_(True)
    kf = kv16[:, :D].float().view(B, Lk, H, dh).transpose(1, 2).requires_grad_(True)
    vf = kv16[:, D:].float().view(B, Lk, H, dh).transpose(1, 2).requires_grad_(True)
    bf = bias.clone().requires_grad_(True) if t5 else None
    ref = attn_ref(qf, kf, vf, scale, bf, mask, mult)
    ref_o = ref.transpose(1, 2).reshape(B * Lq, D)
    torch.testing.assert_close(o.float(), ref_o.detach(), rtol=1e-2, atol=1e-2)
    ref_o.backward(do16.float())
    dq = torch.empty(B * Lq, D, device="cuda", dtype=torch.bfloat16)
    dkv = torch.empty(B * Lk, 2 * D, device="cuda", dtype=torch.bfloat16)
    dbias = torch.zeros(B, H, Lq, Lk, device="cuda") if t5 else None     # per-sample dS
    d.dout, d.lddo, d.dq, d.lddq = A(do16), D, A(dq), D
    d.dk, d.lddk, d.dv, d.lddv, d.dbias = A(dkv), 2 * D, A(dkv, D), 2 * D, A(dbias)
    L.check(L.load().vqa_attn_bwd(ctypes.byref(d), L.stream_handle()), "bwd")
    torch.cuda.synchronize()

    def chk(got, ref_t):
        ref_t = ref_t.transpose(1, 2).reshape(got.shape)
        err = (got.float() - ref_t).abs().max().item()
        assert err <= 1e-2 * ref_t.abs().max().item() + 1e-3, err
    chk(dq, qf.grad)
    chk(dkv[:, :D], kf.grad)
    chk(dkv[:, D:], vf.grad)
    if t5:
        red = torch.full((H, Lq, Lk), 3.0, device="cuda")
        run(k, "vqa_batch_sum", dbias, B, H * Lq * Lk, red, 1.0)
        torch.cuda.synchronize()
        torch.testing.assert_close(red - 3.0, bf.grad, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("G,Lk,dh", [(3, 32, 96), (2, 49, 96), (4, 40, 64)])
def test_grouped_attention_equals_separate_launches(k, G, Lk, dh):
    """vqa_attn_desc.groups: G attentions in one forward and one backward launch give the bits
    of G separate launches (q|k|v of group g at column g*3D of one row, outputs / P / dO at
    per-group strides, dropout site + g*stride)."""
    B, H, Lq = 3, 8, 32
    D = H * dh
    L = k.lib
    A = k.ops.addr
    qkv = rnd((B * Lq, G * 3 * D), 20, dtype=torch.bfloat16)
    kv = qkv if Lk == Lq else rnd((B * Lk, G * 3 * D), 21, dtype=torch.bfloat16)
    do = rnd((G, B * Lq, D), 22, dtype=torch.bfloat16)
    rng = torch.tensor([5, 2, 1], dtype=torch.int32, device="cuda")
    outs = []
    for grouped in (False, True):
        o = torch.zeros(G, B * Lq, D, device="cuda", dtype=torch.bfloat16)
        p = torch.zeros(G, B, H, Lq, Lk, device="cuda")
        dq = torch.zeros(B * Lq, G * 3 * D, device="cuda", dtype=torch.bfloat16)
        dkv = dq if Lk == Lq else torch.zeros(B * Lk, G * 3 * D, device="cuda", dtype=torch.bfloat16)
        for g in range(1 if grouped else G):
            d = L.AttnDesc()
            c = g * 3 * D
            d.q, d.ldq, d.k, d.ldk, d.v, d.ldv = A(qkv, c), G * 3 * D, A(kv, c + D), G * 3 * D, A(kv, c + 2 * D), G * 3 * D
            d.o, d.ldo, d.p = A(o[g]), D, A(p[g])
            d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, H, Lq, Lk, dh, 1.0 / math.sqrt(dh)
            d.drop = L.Dropout(0.1, 40 + 8 * g, rng.data_ptr())
            if grouped:
                d.groups, d.gstride_qkv, d.gstride_o, d.gstride_p, d.gstride_dout = G, 3 * D, B * Lq * D, p[0].numel(), \
                    B * Lq * D
                d.gdrop_site_stride = 8
            assert L.load().vqa_attn_path(ctypes.byref(d), 0) == L.ATTN_MFMA
            L.check(L.load().vqa_attn_fwd(ctypes.byref(d), L.stream_handle()), "fwd")
            d.dout, d.lddo = A(do[g]), D
            d.dq, d.lddq, d.dk, d.lddk, d.dv, d.lddv = A(dq, c), G * 3 * D, A(dkv, c + D), G * 3 * D, \
                A(dkv, c + 2 * D), G * 3 * D
            L.check(L.load().vqa_attn_bwd(ctypes.byref(d), L.stream_handle()), "bwd")
        torch.cuda.synchronize()
        outs.append((o, p, dq, dkv))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert float(outs[1][1].abs().sum()) > 0


@pytest.mark.parametrize("Lq", [20, 40])
def test_causal_bias_with_key_mask_one_finfo_min(k, Lq):
    """The T5 decoder's causal pairs (bias = finfo.min, vqa_t5_relbias_fwd bucket < 0) under a
    key-padding mask: HF adds ONE combined extended mask (rel-bias + finfo.min where causal OR
    padded), so a fully masked query row is a uniform softmax over its keys, not -inf / one-hot
    (TF modeling_t5.py: position_bias + mask; vit_vqa_model.py:199-205).  Lq 40: VALU kernel."""
    B, H, dh = 3, 12, 64
    D, Lk = H * dh, Lq
    fmin = torch.finfo(torch.float32).min
    q16 = rnd((B * Lq, D), 40, dtype=torch.bfloat16)
    kv16 = rnd((B * Lk, 2 * D), 41, dtype=torch.bfloat16)
    rel = rnd((H, Lq, Lk), 42)
    causal = torch.triu(torch.ones(Lq, Lk, device="cuda", dtype=torch.bool), 1)
    bias = torch.where(causal, torch.full_like(rel, fmin), rel)
    mask = torch.ones(B, Lk, device="cuda", dtype=torch.long)
    mask[0] = 0                                                   # an empty decoder question
    mask[1, 5:] = 0
    L = k.lib
    o = torch.empty(B * Lq, D, device="cuda", dtype=torch.bfloat16)
    p = torch.empty(B, H, Lq, Lk, device="cuda")
    d = L.AttnDesc()
    A = k.ops.addr
    d.q, d.ldq, d.k, d.ldk, d.v, d.ldv = A(q16), D, A(kv16), 2 * D, A(kv16, D), 2 * D
    d.o, d.ldo, d.p, d.bias, d.key_mask = A(o), D, A(p), A(bias), A(mask)
    d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, H, Lq, Lk, dh, 1.0
    L.check(L.load().vqa_attn_fwd(ctypes.byref(d), L.stream_handle()), "fwd")
    torch.cuda.synchronize()
    qf = q16.float().view(B, Lq, H, dh).transpose(1, 2)
    kf = kv16[:, :D].float().view(B, Lk, H, dh).transpose(1, 2)
    vf = kv16[:, D:].float().view(B, Lk, H, dh).transpose(1, 2)
    ext = (causal[None, None] | (mask[:, None, None, :] == 0)).float() * fmin
    pr = torch.softmax(qf @ kf.transpose(-1, -2) + rel + ext, -1)
    ref = (pr @ vf).transpose(1, 2).reshape(B * Lq, D)
    assert torch.isfinite(p).all()
    torch.testing.assert_close(p, pr, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(o.float(), ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(p[0], torch.full_like(p[0], 1.0 / Lk))   # fully masked: uniform


@pytest.mark.parametrize("B,L,A,D,ign", [(8, 32, 170, 768, 0), (64, 32, 170, 768, 0), (37, 49, 13, 768, 0),
                                         (5, 16, 192, 768, 0), (64, 32, 170, 1024, 0), (19, 49, 37, 1024, 0),
                                         (6, 16, 192, 836, 0), (3, 7, 5, 20, 0), (16, 32, 193, 768, 0),
                                         (21, 32, 700, 768, 0), (5, 16, 1024, 1024, 0),
                                         (64, 32, 170, 768, 27), (300, 16, 170, 768, 33), (9, 16, 700, 768, 8)])
def test_head_fwd_bwd(k, B, L, A, D, ign):
    """D = 1024 is T5-large's width (BASELINE config 5); 836 / 20 exercise the masked
    column tail of the 256- and 192-column pooler layouts; A > 192 the chunked answer
    loop of the dpooled kernel (193: a one-answer second chunk).  ign > 0: that many rows
    (the last, as the engines pad a short final batch) carry target -100, NLLLoss's
    ignore_index: nll 0, the mean over the other rows, no gradient from them (300 rows:
    the divisor's count runs over two 256-row passes)."""
    x = rnd((B, L, D), 20)
    wp, bp = 0.03 * rnd(D, 21), 0.1 * rnd(1, 22)
    wc, bc = 0.03 * rnd((A, D), 23), 0.1 * rnd(A, 24)
    tgt = torch.randint(0, A, (B,), device="cuda")
    if ign:
        tgt[B - ign:] = -100
    att, pooled, logp = torch.empty(B, L, device="cuda"), torch.empty(B, D, device="cuda"), \
        torch.empty(B, A, device="cuda")
    nll, loss = torch.empty(B, device="cuda"), torch.empty(1, device="cuda")
    run(k, "vqa_head_fwd", x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A)
    xr, wpr, bpr, wcr, bcr = (t.clone().requires_grad_(True) for t in (x, wp, bp, wc, bc))
    a = torch.softmax(xr @ wpr[:, None] + bpr, dim=1)
    pr = torch.bmm(a.transpose(1, 2), xr).squeeze(1)
    lp = F.log_softmax(pr @ wcr.T + bcr, -1)
    ls = F.nll_loss(lp, tgt)
    ls.backward()
    torch.testing.assert_close(logp, lp.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss[0], ls.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(nll, F.nll_loss(lp, tgt, reduction="none").detach(), rtol=1e-5, atol=1e-6)
    dx = torch.empty_like(x)
    dwp, dbp, dwc, dbc = torch.empty_like(wp), torch.empty(1, device="cuda"), torch.empty_like(wc), \
        torch.empty_like(bc)
    ws = torch.empty(k.lib.load().vqa_head_workspace_floats(B, L, D, A), device="cuda")
    run(k, "vqa_head_bwd", x, att, pooled, logp, tgt, wp, wc, dx, None, dwp, dbp, dwc, dbc, ws, B, L, D, A,
        None, None, None, 1.0)
    torch.cuda.synchronize()
    for got, ref in ((dx, xr.grad), (dwp, wpr.grad), (dbp, bpr.grad), (dwc, wcr.grad), (dbc, bcr.grad)):
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("B,ign,others,world", [(8, 0, 8, 2), (8, 3, 1, 2), (8, 8, 5, 2), (64, 10, 150, 3),
                                               (300, 40, 0, 1)])
def test_head_bwd_global_rows(k, B, ign, others, world):
    """Data-parallel divisor (ABI 18): vqa_count_targets counts this rank's valid rows; with
    row_total = that count + `others` (the other ranks' rows) and row_scale = world, dlogits are
    (softmax - onehot) * world / total and the loss is sum(nll) * world / total -- summed over
    the ranks and scaled by 1/world, the global batch's mean.  ign = B: a rank with no valid row
    (zero gradient, loss 0)."""
    L, A, D = 16, 170, 768
    x = rnd((B, L, D), 30)
    wp, bp = 0.03 * rnd(D, 31), 0.1 * rnd(1, 32)
    wc, bc = 0.03 * rnd((A, D), 33), 0.1 * rnd(A, 34)
    tgt = torch.randint(0, A, (B,), device="cuda")
    if ign:
        tgt[B - ign:] = -100
    cnt = torch.full((1,), -1.0, device="cuda")
    run(k, "vqa_count_targets", tgt, B, cnt)
    torch.cuda.synchronize()
    assert cnt.item() == float(B - ign)
    total = cnt + others
    att, pooled, logp = torch.empty(B, L, device="cuda"), torch.empty(B, D, device="cuda"), \
        torch.empty(B, A, device="cuda")
    nll, loss = torch.empty(B, device="cuda"), torch.empty(1, device="cuda")
    run(k, "vqa_head_fwd", x, wp, bp, wc, bc, tgt, att, pooled, logp, nll, loss, B, L, D, A)
    xr, wpr, bpr, wcr, bcr = (t.clone().requires_grad_(True) for t in (x, wp, bp, wc, bc))
    a = torch.softmax(xr @ wpr[:, None] + bpr, dim=1)
    pr = torch.bmm(a.transpose(1, 2), xr).squeeze(1)
    lp = F.log_softmax(pr @ wcr.T + bcr, -1)
    ls = F.nll_loss(lp, tgt, reduction="sum") * world / total.item()
    ls.backward()
    dx = torch.empty_like(x)
    dwp, dbp, dwc, dbc = torch.empty_like(wp), torch.empty(1, device="cuda"), torch.empty_like(wc), \
        torch.empty_like(bc)
    ws = torch.empty(k.lib.load().vqa_head_workspace_floats(B, L, D, A), device="cuda")
    run(k, "vqa_head_bwd", x, att, pooled, logp, tgt, wp, wc, dx, None, dwp, dbp, dwc, dbc, ws, B, L, D, A,
        nll, loss, total, float(world))
    torch.cuda.synchronize()
    torch.testing.assert_close(loss[0], ls.detach(), rtol=1e-5, atol=1e-6)
    for got, ref in ((dx, xr.grad), (dwp, wpr.grad), (dbp, bpr.grad), (dwc, wcr.grad), (dbc, bcr.grad)):
        if ign == B:
            assert not got.any()
        else:
            torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("T,pad", [(300, 0), (2048, 900), (1, 0), (8192, 5000), (16384, 7000), (40000, 16000)])
def test_embedding_relbias_colsum_cast(k, T, pad):
    D, Vv = 768, 1000
    ids = torch.randint(0, Vv, (T,), device="cuda")
    ids[:min(50, T)] = 7                                       # heavy duplicates
    if pad:                                                    # a long pad-id run scattered over the batch
        ids[torch.randperm(T, device="cuda")[:pad]] = 0
    table = rnd((Vv, D), 30)
    out = torch.empty(T, D, device="cuda")
    run(k, "vqa_embedding_fwd", ids, table, out, T, D, Vv, None)
    torch.testing.assert_close(out, table[ids])
    dh = rnd((T, D), 31)
    dt = torch.zeros(Vv, D, device="cuda")
    ws = torch.empty(3 * T, device="cuda", dtype=torch.int32)
    run(k, "vqa_embedding_bwd", ids, dh, dt, T, D, Vv, ws)
    ref = torch.zeros(Vv, D, device="cuda", dtype=torch.float64).index_add_(0, ids, dh.double()).float()
    # a row summed over n tokens in fp32 (fixed token order) carries ~sqrt(n) ulps of its partial sums
    nmax = int(torch.bincount(ids, minlength=Vv).max())
    torch.testing.assert_close(dt, ref, rtol=1e-5, atol=1e-4 * max(1.0, (nmax / 2000) ** 0.5))
    dt2 = torch.zeros(Vv, D, device="cuda")
    run(k, "vqa_embedding_bwd", ids, dh, dt2, T, D, Vv, ws)
    assert torch.equal(dt, dt2), "embedding backward must be deterministic"
    Lq = 32
    bucket = torch.from_numpy(k.layout.t5_bucket_map(Lq, Lq)).reshape(-1).cuda()
    tab = rnd((32, 12), 32)
    pb = torch.empty(12, Lq, Lq, device="cuda")
    run(k, "vqa_t5_relbias_fwd", tab, bucket, pb, 12, Lq, Lq)
    torch.testing.assert_close(pb, tab[bucket.long()].T.reshape(12, Lq, Lq))
    dpb = rnd((12, Lq, Lq), 33)
    dtab = torch.zeros(32, 12, device="cuda")
    run(k, "vqa_t5_relbias_bwd", dpb, bucket, dtab, 12, Lq, Lq, 32)
    ref = torch.zeros(32, 12, device="cuda").index_add_(0, bucket.long(), dpb.reshape(12, -1).T)
    torch.testing.assert_close(dtab, ref, rtol=1e-5, atol=1e-5)
    for bf in (0, 1):
        x = rnd((3136, 2304), 34, dtype=torch.bfloat16 if bf else torch.float32)
        o = torch.full((2304,), 2.0, device="cuda")
        ws = torch.empty(k.lib.load().vqa_colsum_workspace_floats(3136, 2304), device="cuda")
        run(k, "vqa_colsum", x, bf, 3136, 2304, 2304, o, 1.0, ws)
        torch.testing.assert_close(o, x.float().sum(0) + 2.0, rtol=1e-4, atol=1e-3)
    x = rnd(1003, 35)
    y = torch.empty(1003, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_cast_f32_bf16", x, y, 1003)
    assert torch.equal(y, x.to(torch.bfloat16))


def test_image_and_maxpool(k):
    img = torch.rand(2, 3, 20, 20, device="cuda")
    out = torch.empty(2, 20, 20, 8, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_image_to_nhwc8", img, out, 2, 20, 20)
    ref = torch.zeros(2, 20, 20, 8, device="cuda")
    ref[..., :3] = img.permute(0, 2, 3, 1)
    assert torch.equal(out, ref.to(torch.bfloat16))
    # space-to-depth stem image: exact layout, and the 4x4/1 conv over it equals the 7x7/2 conv
    for hw in (20, 224):
        img = torch.rand(2, 3, hw, hw, device="cuda")
        hz = hw // 2 + 1
        z = torch.empty(2, hz, hz, 16, device="cuda", dtype=torch.bfloat16)
        run(k, "vqa_image_to_s2d16", img, z, 2, hw, hw)
        xp = F.pad(img, (1, 1, 1, 1))                      # x index 2v+q-1 -> padded 2v+q
        ref = torch.zeros(2, hz, hz, 16, device="cuda")
        for p in range(2):
            for q in range(2):
                ref[..., (2 * p + q) * 3:(2 * p + q) * 3 + 3] = xp[:, :, p:p + 2 * hz:2, q:q + 2 * hz:2].permute(0, 2, 3, 1)
        assert torch.equal(z, ref.to(torch.bfloat16))
        w = torch.randn(64, 3, 7, 7)
        w2 = torch.from_numpy(k.engine.stem_s2d_weight(w.permute(0, 2, 3, 1).numpy()))   # [64, 4, 4, 16]
        y_ref = F.conv2d(img.to(torch.bfloat16).float().cpu().double(), w.double(), stride=2, padding=3)
        y_s2d = F.conv2d(z.float().cpu().permute(0, 3, 1, 2).double(), w2.permute(0, 3, 1, 2).double(), padding=1)
        torch.testing.assert_close(y_s2d, y_ref, rtol=1e-9, atol=1e-9)
    x = rnd((2, 21, 21, 64), 36, dtype=torch.bfloat16)
    y = torch.empty(2, 11, 11, 64, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_maxpool3x3s2_nhwc", x, y, 2, 21, 21, 64, 11, 11)
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y.float(), ref)


@pytest.mark.parametrize("n,h,c,s", [(2, 7, 64, 1), (3, 13, 256, 2), (2, 56, 64, 1), (1, 28, 512, 2)])
def test_subsample_into_concatenated_rows(k, n, h, c, s):
    """vqa_subsample_nhwc: x[:, ::s, ::s, :] written beside other columns (row stride ldy), the
    second half of the fused conv3 + downsample GEMM's A operand -- exact, and the columns left
    of it untouched."""
    x = rnd((n, h, h, c), 37, dtype=torch.bfloat16)
    oh = (h - 1) // s + 1
    left = 64
    y = torch.full((n * oh * oh, left + c), 7.0, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_subsample_nhwc", x, n, h, h, c, s, k.ops.addr(y, left), left + c)
    assert torch.equal(y[:, left:], x[:, ::s, ::s, :].reshape(-1, c))
    assert torch.equal(y[:, :left], torch.full_like(y[:, :left], 7.0))


@pytest.mark.parametrize("n,h,w,c", [(3, 7, 7, 768), (2, 5, 9, 24)])
def test_tap_shift_and_tap_batched_conv_transpose_dw(k, n, h, w, c):
    """vqa_tap_shift's 3x3 shifted copies (exact), and the scaler weight gradient as the
    engine plans it -- one GEMM batched over the taps -- against the implicit-im2col GEMM and
    torch's ConvTranspose2d weight gradient."""
    ops = k.ops
    x = rnd((n, h, w, c), 41, dtype=torch.bfloat16)
    out = torch.empty(9, n * h * w, c, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_tap_shift", x, out, n, h, w, c, 3, 3, 1)
    xp = F.pad(x, (0, 0, 1, 1, 1, 1))
    ref = torch.stack([xp[:, 2 - ky:2 - ky + h, 2 - kx:2 - kx + w].reshape(-1, c) for ky in range(3) for kx in range(3)])
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # dW [c, 9*cin] of a 3x3/1/1 ConvTranspose2d cin -> c (the flipped-conv weight layout)
    cin, K = 64, n * h * w
    f4 = rnd((K, cin), 42, dtype=torch.bfloat16)
    g32 = torch.zeros(c, 9 * cin, device="cuda")
    d = ops.gemm_desc(out, f4, c, cin, K, lda=c, ldb=cin, a_trans=True, b_trans=True, c32=g32, ldc32=9 * cin,
                      batch=9, stride_a=K * c, stride_b=0, stride_c32=cin)
    ops.gemm_call(d, [out, f4, g32])(k.lib.stream_handle())
    gi = torch.zeros(c, 9 * cin, device="cuda")
    geo = ops.conv_geom(n, h, w, cin, h, w, 3, 3, 1, 1)
    d2 = ops.gemm_desc(x.view(K, c), f4, c, 9 * cin, K, lda=c, ldb=9 * cin, a_trans=True, b_trans=True, c32=gi,
                       ldc32=9 * cin, gb=geo)
    ops.gemm_call(d2, [x, f4, gi])(k.lib.stream_handle())
    torch.cuda.synchronize()
    # torch: y = conv_transpose2d(f, W) with W [cin, c, 3, 3]; dW = autograd of <y, dy>, dy = x
    fm = f4.float().view(n, h, w, cin).permute(0, 3, 1, 2).double().cpu()
    dy = x.float().permute(0, 3, 1, 2).double().cpu()
    wt = torch.zeros(cin, c, 3, 3, dtype=torch.float64, requires_grad=True)
    (F.conv_transpose2d(fm, wt, padding=1) * dy).sum().backward()
    # flipped-conv layout: column (ky*3 + kx)*cin + ci holds W[ci, o, 2-ky, 2-kx]
    want = wt.grad.flip(2, 3).permute(1, 2, 3, 0).reshape(c, 9 * cin)
    scale = float(want.abs().max())
    assert float((g32.double().cpu() - want).abs().max()) <= 1e-5 * scale
    assert float((gi.double().cpu() - want).abs().max()) <= 1e-5 * scale


def test_adamw_amsgrad_matches_torch(k):
    n = 4096 + 64
    torch.manual_seed(0)
    p0 = torch.randn(n, device="cuda")
    grads = [torch.randn(n, device="cuda") * 3 for _ in range(4)]
    ends, lrs = [1024, 2048, n], [1e-3, 5e-4, 5e-3]
    ref_params = [p0[0:1024].clone(), p0[1024:2048].clone(), p0[2048:].clone()]
    for t in ref_params:
        t.requires_grad_(True)
    opt = torch.optim.AdamW([{"params": [t], "lr": lr} for t, lr in zip(ref_params, lrs)], weight_decay=0.1,
                            amsgrad=True, foreach=False)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: s / 2 if s < 2 else max(0.0, (10 - s) / 8))
    p, m, v, vm = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), \
        torch.zeros(n, device="cuda")
    p16 = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    st = torch.zeros(16, device="cuda")
    ws = torch.empty(64, device="cuda", dtype=torch.float64)
    L = k.lib
    d = L.AdamWDesc()
    A = k.ops.addr
    d.param, d.grad, d.exp_avg, d.exp_avg_sq, d.max_exp_avg_sq, d.param16 = A(p), 0, A(m), A(v), A(vm), A(p16)
    d.n, d.ngroups = n, 3
    for i in range(3):
        d.group_end[i], d.group_lr[i] = ends[i], lrs[i]
    d.beta1, d.beta2, d.eps, d.weight_decay, d.grad_scale, d.state = 0.9, 0.999, 1e-8, 0.1, 1.0, A(st)
    for g in grads:
        gg = g.clone()
        d.grad = A(gg)
        run(k, "vqa_grad_sqnorm", gg, n, ws, 64)
        run(k, "vqa_optim_finalize", ws, 64, 1.0, 1.0, 2, 10, 0.9, 0.999, st)
        L.check(L.load().vqa_adamw_amsgrad(ctypes.byref(d), L.stream_handle()), "adamw")
        for t, a, b in zip(ref_params, [0, 1024, 2048], ends):
            t.grad = g[a:b].clone()
        norm = torch.nn.utils.clip_grad_norm_(ref_params, 1.0)
        opt.step()
        sched.step()
        torch.cuda.synchronize()
        assert abs(st[1].item() - norm.item()) <= 1e-5 * norm.item()
        torch.testing.assert_close(p, torch.cat([t.detach() for t in ref_params]), rtol=1e-6, atol=1e-7)
    assert torch.equal(p16, p.to(torch.bfloat16))


def test_dropout_mask_matches_oracle_hash(k):
    """vqa_dropout_mask == the oracle's restatement of the counter hash, bit for bit."""
    from oracle import vqa_oracle as orc
    L = k.lib
    for seed, ctr, site, p, n in [(0, 1, 1, 0.1, 100003), (123456789, 77, 150, 0.1, 4096),
                                  (0xFFFFFFFF, 2**31 + 5, 16, 0.5, 5000), (3, 3, 3, 0.0, 64)]:
        rng = torch.from_numpy(np.array([seed, ctr, 1], np.uint32).view(np.int32)).cuda()
        d = L.Dropout(p, site, rng.data_ptr())
        out = torch.empty(n, device="cuda")
        L.check(L.load().vqa_dropout_mask(ctypes.byref(d), ctypes.c_void_p(out.data_ptr()), n, L.stream_handle()),
                "mask")
        torch.cuda.synchronize()
        ref = orc.dropout_multiplier(p, seed, ctr, site, n) if p > 0 else np.ones(n, np.float32)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    # law: keep rate 1-p, scale 1/(1-p); advancing the counter changes the mask
    rng = torch.tensor([0, 0, 1], dtype=torch.int32, device="cuda")
    d = L.Dropout(0.1, 5, rng.data_ptr())
    m0, m1 = torch.empty(1 << 20, device="cuda"), torch.empty(1 << 20, device="cuda")
    L.load().vqa_dropout_mask(ctypes.byref(d), ctypes.c_void_p(m0.data_ptr()), 1 << 20, L.stream_handle())
    run(k, "vqa_rng_advance", rng)
    L.load().vqa_dropout_mask(ctypes.byref(d), ctypes.c_void_p(m1.data_ptr()), 1 << 20, L.stream_handle())
    torch.cuda.synchronize()
    assert int(rng[1]) == 1
    keep0 = (m0 > 0).float().mean().item()
    assert abs(keep0 - 0.9) < 2e-3, keep0
    assert torch.all((m0 == 0) | (m0 == np.float32(1) / (np.float32(1) - np.float32(0.1))))
    both = ((m0 > 0) & (m1 > 0)).float().mean().item()
    assert abs(both - 0.81) < 3e-3, both                                # independent draws


def test_norm_and_embedding_dropout_hooks(k):
    from oracle import vqa_oracle as orc
    L = k.lib
    rows, D = 256, 768
    rng = torch.tensor([9, 2, 1], dtype=torch.int32, device="cuda")
    mk = lambda site: L.Dropout(0.1, site, rng.data_ptr())
    mult = lambda site: torch.from_numpy(orc.dropout_multiplier(0.1, 9, 2, site, rows * D)).cuda().view(rows, D)
    dA, dB, dC = mk(40), mk(41), mk(42)
    pa = lambda d: ctypes.addressof(d)
    x, w = rnd((rows, D), 1), 1 + 0.1 * rnd(D, 2)
    dy, dres = rnd((rows, D), 3), rnd((rows, D), 4)
    y32, rstd = torch.empty_like(x), torch.empty(rows, device="cuda")
    run(k, "vqa_rmsnorm_fwd", x, w, y32, None, rstd, rows, D, 1e-6, pa(dA))
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6)) * mult(40)
    ref.backward(dy)
    torch.testing.assert_close(y32, ref.detach(), rtol=1e-5, atol=1e-5)
    # backward of that dropout (drop_dy) + residual; masks on the two outputs
    dx32, dx16, dw = torch.empty_like(x), torch.empty(rows, D, device="cuda", dtype=torch.bfloat16), \
        torch.empty(D, device="cuda")
    ws = torch.empty(L.load().vqa_norm_bwd_workspace_floats(rows, D), device="cuda")
    run(k, "vqa_rmsnorm_bwd", dy, x, rstd, w, dres, dx32, dx16, dw, 0.0, ws, rows, D, pa(dA), pa(dB), pa(dC))
    torch.cuda.synchronize()
    full = xr.grad + dres
    torch.testing.assert_close(dx32, full * mult(41), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dx16.float(), (full * mult(42)).to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dw, wr.grad, rtol=1e-4, atol=1e-3)
    # LayerNorm backward: branch gradient masked in bf16 + its fp32 column sums (fused bias grad)
    g, b = 1 + 0.1 * rnd(D, 6), 0.1 * rnd(D, 7)
    mu, rs = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    y = torch.empty_like(x)
    run(k, "vqa_layernorm_fwd", x, g, b, y, None, mu, rs, rows, D, 1e-5)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, g, b))
    F.layer_norm(xr, (D,), gr, br, 1e-5).backward(dy)
    dx, dg, db, dsum = (torch.empty_like(x), torch.empty(D, device="cuda"), torch.empty(D, device="cuda"),
                        torch.empty(D, device="cuda"))
    run(k, "vqa_layernorm_bwd", dy, x, mu, rs, g, None, dx, dx16, dg, db, ws, rows, D, pa(dB), dsum)
    torch.cuda.synchronize()
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dx16.float(), (xr.grad * mult(41)).to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dsum, (xr.grad * mult(41)).sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    # embedding dropout
    T, Vv = rows, 1000
    ids = torch.randint(0, Vv, (T,), device="cuda")
    table = rnd((Vv, D), 30)
    out = torch.empty(T, D, device="cuda")
    run(k, "vqa_embedding_fwd", ids, table, out, T, D, Vv, pa(dC))
    torch.cuda.synchronize()
    torch.testing.assert_close(out, table[ids] * mult(42))


@pytest.mark.parametrize("n,oh", [(2, 112), (3, 32), (1, 192)])
def test_stem_patch_conv_equals_the_implicit_gemm(k, n, oh):
    """vqa_stem_s2d_conv (LDS-patch stem) against the implicit-im2col vqa_gemm the engine used
    before r05 (4x4 / stride 1 / pad 1 over the space-to-depth image, bias, ReLU): bit for bit."""
    ops = k.ops
    hz = oh + 1
    z = rnd((n, hz, hz, 16), 51, dtype=torch.bfloat16)
    w = rnd((64, 4, 4, 16), 52, scale=0.1, dtype=torch.bfloat16)
    b = rnd(64, 53)
    y_ref = torch.empty(n, oh, oh, 64, device="cuda", dtype=torch.bfloat16)
    g = ops.conv_geom(n, hz, hz, 16, oh, oh, 4, 4, 1, 1)
    ops.run(ops.gemm_desc(z, w, n * oh * oh, 64, 256, lda=256, ldb=256, ga=g, c16=y_ref, ldc16=64, bias=b, relu=True))
    y = torch.full_like(y_ref, 3.0)
    run(k, "vqa_stem_s2d_conv", z, w, b, y, n, hz, oh)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)


@pytest.mark.parametrize("n,oh", [(2, 112), (3, 32), (1, 192), (2, 16)])
def test_stem_pool_equals_stem_then_maxpool(k, n, oh):
    """vqa_stem_pool_s2d (stem + 3x3/2 maxpool fused, only the pooled map written) against the
    implicit-GEMM stem followed by vqa_maxpool3x3s2_nhwc: bit for bit, borders included."""
    ops = k.ops
    hz, ph = oh + 1, oh // 2
    z = rnd((n, hz, hz, 16), 54, dtype=torch.bfloat16)
    w = rnd((64, 4, 4, 16), 55, scale=0.1, dtype=torch.bfloat16)
    b = rnd(64, 56)
    s = torch.empty(n, oh, oh, 64, device="cuda", dtype=torch.bfloat16)
    g = ops.conv_geom(n, hz, hz, 16, oh, oh, 4, 4, 1, 1)
    ops.run(ops.gemm_desc(z, w, n * oh * oh, 64, 256, lda=256, ldb=256, ga=g, c16=s, ldc16=64, bias=b, relu=True))
    ref = torch.empty(n, ph, ph, 64, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_maxpool3x3s2_nhwc", s, ref, n, oh, oh, 64, ph, ph)
    y = torch.full_like(ref, 5.0)
    run(k, "vqa_stem_pool_s2d", z, w, b, y, n, hz, oh)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("n,h", [(2, 224), (3, 64), (1, 32), (1, 384)])
def test_stem_pool_from_the_image_equals_s2d_then_stem_pool(k, n, h):
    """vqa_stem_pool_img (space-to-depth staged from the fp32 image inside the stem kernel) against
    vqa_image_to_s2d16 followed by vqa_stem_pool_s2d: bit for bit.  The weights are random in the
    s2d channels 12..15 too, so the kernel's zeroed channels are checked."""
    hz, oh = h // 2 + 1, h // 2
    img = rnd((n, 3, h, h), 57)
    w = rnd((64, 4, 4, 16), 58, scale=0.1, dtype=torch.bfloat16)
    b = rnd(64, 59)
    z = torch.empty(n, hz, hz, 16, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_image_to_s2d16", img, z, n, h, h)
    ref = torch.empty(n, h // 4, h // 4, 64, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_stem_pool_s2d", z, w, b, ref, n, hz, oh)
    y = torch.full_like(ref, 7.0)
    run(k, "vqa_stem_pool_img", img, w, b, y, n, h)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("n", [16, 64])
def test_stem_pool_benched_shape_many_tiles_per_workgroup(k, n):
    """The benched stem shape (224², B = 64: 6,272 tiles over the persistent grid, ~12 per
    workgroup, so the register prefetch of the next tile's patch runs many times per workgroup;
    ADVICE r05): vqa_stem_pool_img and vqa_stem_pool_s2d against vqa_image_to_s2d16 + the
    implicit-GEMM stem + vqa_maxpool3x3s2_nhwc, bit for bit."""
    ops = k.ops
    h = 224
    hz, oh, ph = h // 2 + 1, h // 2, h // 4
    img = rnd((n, 3, h, h), 60)
    w = rnd((64, 4, 4, 16), 61, scale=0.1, dtype=torch.bfloat16)
    b = rnd(64, 62)
    z = torch.empty(n, hz, hz, 16, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_image_to_s2d16", img, z, n, h, h)
    s = torch.empty(n, oh, oh, 64, device="cuda", dtype=torch.bfloat16)
    g = ops.conv_geom(n, hz, hz, 16, oh, oh, 4, 4, 1, 1)
    ops.run(ops.gemm_desc(z, w, n * oh * oh, 64, 256, lda=256, ldb=256, ga=g, c16=s, ldc16=64, bias=b, relu=True))
    ref = torch.empty(n, ph, ph, 64, device="cuda", dtype=torch.bfloat16)
    run(k, "vqa_maxpool3x3s2_nhwc", s, ref, n, oh, oh, 64, ph, ph)
    y1 = torch.full_like(ref, 5.0)
    run(k, "vqa_stem_pool_s2d", z, w, b, y1, n, hz, oh)
    y2 = torch.full_like(ref, 7.0)
    run(k, "vqa_stem_pool_img", img, w, b, y2, n, h)
    torch.cuda.synchronize()
    assert torch.equal(y1, ref)
    assert torch.equal(y2, ref)


def test_adamw_rows_split_equals_dense(k):
    """vqa_embed_mark + vqa_adamw_rows (ABI 18): the embedding table's update split by rows -- the
    rows no token touched (zero gradient) before vqa_optim_finalize with the schedule it is about
    to set, the marked rows after it -- equals vqa_adamw_amsgrad over the whole table bit for bit
    (p, m, v, vmax and the bf16 shadow), two LR groups, duplicated ids, a warm-up-phase step."""
    L = k.lib
    V, D, T = 1000, 64, 300
    gen = torch.Generator(device="cuda").manual_seed(90)
    ids = torch.randint(0, V, (T,), device="cuda", generator=gen)
    g = torch.zeros(V, D, device="cuda")
    g[ids] = rnd((T, D), 91)                                  # touched rows only (duplicates overwrite)
    base = {"p": rnd((V, D), 92), "m": 0.01 * rnd((V, D), 93), "v": 0.001 * rnd((V, D), 94).abs()}
    base["vm"] = base["v"] + 0.0005 * rnd((V, D), 95).abs()
    ws = torch.tensor([3.25, 1.5], dtype=torch.float64, device="cuda")
    warm, total = 10, 100

    def state(step):
        st = torch.zeros(L.ST_FLOATS, device="cuda")
        st[0] = step
        return st

    def desc(t, st):
        d = L.AdamWDesc()
        d.param, d.grad, d.exp_avg = t["p"].data_ptr(), g.data_ptr(), t["m"].data_ptr()
        d.exp_avg_sq, d.max_exp_avg_sq, d.param16 = t["v"].data_ptr(), t["vm"].data_ptr(), t["p16"].data_ptr()
        d.n = V * D
        d.ngroups = 2
        d.group_end[0], d.group_end[1] = 300 * D, V * D
        d.group_lr[0], d.group_lr[1] = 5e-3, 1e-4
        d.beta1, d.beta2, d.eps, d.weight_decay, d.grad_scale = 0.9, 0.999, 1e-8, 0.1, 1.0
        d.state = st.data_ptr()
        return d
    for step in (3.0, 40.0):                                   # warm-up and decay phases of the schedule
        res = []
        for split in (False, True):
            t = {kk: vv.clone() for kk, vv in base.items()}
            t["p16"] = torch.empty(V, D, device="cuda", dtype=torch.bfloat16)
            st = state(step)
            d = desc(t, st)
            s = L.stream_handle()
            fin = lambda: L.check(L.load().vqa_optim_finalize(ctypes.c_void_p(ws.data_ptr()), 2, ctypes.c_float(1.0),  # noqa: E731
                                                              ctypes.c_float(1.0), warm, total, ctypes.c_float(0.9),
                                                              ctypes.c_float(0.999), ctypes.c_void_p(st.data_ptr()), s),
                                  "finalize")
            if split:
                mark = torch.full((V,), -1, dtype=torch.int32, device="cuda")
                run(k, "vqa_embed_mark", ids, T, V, mark, st)
                L.check(L.load().vqa_adamw_rows(ctypes.byref(d), mark.data_ptr(), V, D, 0, warm, total, s), "rows0")
                fin()
                L.check(L.load().vqa_adamw_rows(ctypes.byref(d), mark.data_ptr(), V, D, 1, warm, total, s), "rows1")
            else:
                fin()
                L.check(L.load().vqa_adamw_amsgrad(ctypes.byref(d), s), "dense")
            torch.cuda.synchronize()
            res.append(t)
        for kk in ("p", "m", "v", "vm", "p16"):
            assert torch.equal(res[0][kk], res[1][kk]), (step, kk)
        assert not torch.equal(res[0]["p"], base["p"])          # the update did something
