"""BASELINE config 4 (VitVQAModel, ViT-base + T5 encoder-decoder) on the GPU: the new
kernels against torch fp32 references, and the engine's train step against the
reference's own fixture (eval mode, tests/golden/make_golden_vit.py) and the CPU
oracle (train mode, hash dropout).  Measured errors go to the parity report."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vit_model_b4_l16.npz")
GROUPS = ("lang_model", "fusing_layer", "classification_layer")


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _bf(x):
    return x.to(torch.bfloat16)


def test_long_attention_matches_torch(cuda, pkg, parity_report):
    """vqa_attn_fwd at ViT's 197 tokens (online-softmax MFMA kernel) and a ragged length."""
    L_, ops = pkg.lib, pkg.ops
    errs = {}
    for B, Lt, dh in ((2, 197, 64), (3, 70, 64), (1, 33, 96)):
        H = 12 if dh == 64 else 8
        g = torch.Generator().manual_seed(Lt)
        qkv = torch.randn(B * Lt, 3 * H * dh, generator=g).cuda()
        q16 = _bf(qkv)
        o = torch.zeros(B * Lt, H * dh, dtype=torch.bfloat16, device="cuda")
        d = L_.AttnDesc()
        D = H * dh
        d.q, d.ldq, d.k, d.ldk, d.v, d.ldv = q16.data_ptr(), 3 * D, q16.data_ptr() + 2 * D, 3 * D, \
            q16.data_ptr() + 4 * D, 3 * D
        d.o, d.ldo = o.data_ptr(), D
        d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, H, Lt, Lt, dh, dh ** -0.5
        L_.check(L_.load().vqa_attn_fwd(__import__("ctypes").byref(d), L_.stream_handle()), "vqa_attn_fwd")
        torch.cuda.synchronize()
        x = q16.float().view(B, Lt, 3, H, dh)
        qq, kk, vv = (x[:, :, j].transpose(1, 2) for j in range(3))
        ref = (torch.softmax(qq @ kk.transpose(2, 3) * dh ** -0.5, -1) @ vv).transpose(1, 2).reshape(B * Lt, D)
        err = float((o.float() - ref).abs().max() / ref.abs().max())
        errs[f"{B}x{Lt}x{dh}"] = err
        assert err <= 1e-2, (B, Lt, dh, err)
    parity_report["vit_long_attention_rel"] = errs


def test_attention_probs_match_torch(cuda, pkg, parity_report):
    """vqa_attn_probs (HF output_attentions) against torch fp32 softmax over the same bf16 q / k,
    at ViT's 197 tokens and with a T5-style rel-bias + key mask; every row sums to 1."""
    import ctypes
    L_ = pkg.lib
    errs = {}
    for B, Lq, Lk, H, dh, masked in ((2, 197, 197, 12, 64, False), (3, 32, 40, 8, 96, True)):
        g = torch.Generator().manual_seed(Lq + Lk)
        D = H * dh
        qk = _bf(torch.randn(B * max(Lq, Lk), 2 * D, generator=g)).cuda()
        bias = (torch.randn(H, Lq, Lk, generator=g) * 2).cuda() if masked else None
        mask = torch.ones(B, Lk, dtype=torch.int64, device="cuda")
        if masked:
            mask[:, Lk - 7:] = 0
        p = torch.empty(B, H, Lq, Lk, device="cuda")
        d = L_.AttnDesc()
        d.q, d.ldq, d.k, d.ldk = qk.data_ptr(), 2 * D, qk.data_ptr() + 2 * D, 2 * D
        d.p, d.bias, d.key_mask = p.data_ptr(), bias.data_ptr() if masked else None, mask.data_ptr() if masked else None
        d.batch, d.heads, d.lq, d.lk, d.dh, d.scale = B, H, Lq, Lk, dh, dh ** -0.5
        L_.check(L_.load().vqa_attn_probs(ctypes.byref(d), L_.stream_handle()), "vqa_attn_probs")
        torch.cuda.synchronize()
        x = qk.float()
        q = x[:B * Lq, :D].view(B, Lq, H, dh).transpose(1, 2)
        k = x[:B * Lk, D:].view(B, Lk, H, dh).transpose(1, 2)
        s = q @ k.transpose(2, 3) * dh ** -0.5
        if masked:
            s = s + bias + (1 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
        ref = torch.softmax(s, -1)
        err = float((p - ref).abs().max())
        errs[f"{B}x{Lq}x{Lk}x{dh}"] = err
        assert err <= 2e-6, err
        assert float((p.sum(-1) - 1).abs().max()) <= 1e-5
    parity_report["attention_probs_max_abs"] = errs


def test_vit_attention_maps_match_oracle(cuda, pkg, parity_report):
    """generate_answers' attention_tensors (12 ViT layers) against the fp32 oracle's softmax
    probabilities of the same pixels and weights (the engine's q / k are bf16 GEMM outputs)."""
    from oracle import vit_oracle as vo
    vm = pkg.vit_model
    B, L, Ld = 2, 16, 12
    sd = vm.make_state_dict(seed=0)
    model = pkg.model.VitVQAModel(batch_size=B, seq_len=L, dec_len=Ld, state_dict=sd, dropout=0.0)
    model.eval()
    nb = vm.make_batch(B, L, dec_len=Ld, seed=3)
    dev = {k: (None if v is None else torch.as_tensor(v).cuda()) for k, v in nb.items()}
    _, _, att = model.generate_answers(**dev)
    ref = []
    tsd = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items() if k.startswith("vision_model.")}
    with torch.no_grad():
        vo.vit_pooled(tsd, torch.as_tensor(nb["pixel_values"], dtype=torch.float32), attentions=ref)
    errs = [float((a.cpu() - r).abs().max()) for a, r in zip(att, ref)]
    parity_report["vit_attention_maps_max_abs"] = errs
    assert len(errs) == 12 and max(errs) <= 2e-3, errs   # measured 1.3e-4 (bf16 q|k through 12 layers)


@pytest.mark.parametrize("m,n,k", [(300, 512, 768), (8192, 4096, 256)])     # 64x128 / 256x256 kernels
def test_gelu_tanh_epilogues(cuda, pkg, m, n, k):
    ops = pkg.ops
    g = torch.Generator().manual_seed(3)
    x = _bf(torch.randn(m, k, generator=g)).cuda()
    w = _bf(torch.randn(n, k, generator=g) * 0.05).cuda()
    b = (torch.randn(n, generator=g) * 0.1).cuda()
    for act, fn in ((2, torch.nn.functional.gelu), (3, torch.tanh)):
        out = torch.zeros(m, n, dtype=torch.float32, device="cuda")
        d = ops.gemm_desc(x, w, m, n, k, lda=k, ldb=k, c32=out, ldc32=n, bias=b, relu=act)
        ops.gemm_call(d, [x, w, out, b])(pkg.lib.stream_handle())
        torch.cuda.synchronize()
        ref = fn(x.float() @ w.float().T + b)
        assert float((out - ref).abs().max()) <= 2e-3, act


def test_vit_data_movement_kernels(cuda, pkg):
    L_ = pkg.lib
    lib = L_.load()
    s = L_.stream_handle()
    g = torch.Generator().manual_seed(5)
    img = torch.rand(2, 3, 64, 48, generator=g).cuda()
    out = torch.zeros(2 * 4 * 3, 768, dtype=torch.bfloat16, device="cuda")
    L_.check(lib.vqa_vit_patchify(img.data_ptr(), out.data_ptr(), 2, 64, 48, 16, s), "patchify")
    ref = torch.nn.functional.unfold(img, 16, stride=16).transpose(1, 2).reshape(-1, 768)
    torch.cuda.synchronize()
    assert torch.equal(out, ref.to(torch.bfloat16))
    # gather / scatter rows, last index
    src = torch.randn(10, 64, generator=g).cuda()
    idx = torch.tensor([3, 0, 9], dtype=torch.int64, device="cuda")
    dst = torch.zeros(3, 64, device="cuda")
    L_.check(lib.vqa_gather_rows(src.data_ptr(), 64, idx.data_ptr(), 0, 0, dst.data_ptr(), 64, 3, 64, 4, s), "g")
    back = torch.zeros(10, 64, device="cuda")
    L_.check(lib.vqa_scatter_rows(dst.data_ptr(), 64, None, 4, 1, back.data_ptr(), 64, 3, 64, 4, s), "s")
    mask = torch.tensor([[1, 1, 0, 0], [1, 1, 1, 1], [0, 0, 0, 0]], dtype=torch.int64, device="cuda")
    last = torch.zeros(3, dtype=torch.int64, device="cuda")
    L_.check(lib.vqa_last_index(mask.data_ptr(), 3, 4, last.data_ptr(), s), "last")
    torch.cuda.synchronize()
    assert torch.equal(dst, src[idx])
    assert torch.equal(back[[1, 5, 9]], dst) and float(back[[0, 2, 3, 4, 6, 7, 8]].abs().sum()) == 0.0
    assert last.tolist() == [1, 7, 8]
    # single-token cross-attention, dropout off: broadcast and its query-order sum
    v = _bf(torch.randn(2, 768, generator=g)).cuda()
    ctx = torch.zeros(2 * 5, 768, dtype=torch.bfloat16, device="cuda")
    L_.check(lib.vqa_xattn1_fwd(v.data_ptr(), 768, ctx.data_ptr(), 768, 2, 5, 12, 64, None, s), "xf")
    dctx = _bf(torch.randn(10, 768, generator=g)).cuda()
    dv = torch.zeros(2, 768, device="cuda")
    L_.check(lib.vqa_xattn1_bwd(dctx.data_ptr(), 768, dv.data_ptr(), None, 768, 2, 5, 12, 64, None, s), "xb")
    torch.cuda.synchronize()
    assert torch.equal(ctx.view(2, 5, 768), v[:, None].expand(2, 5, 768))
    assert torch.allclose(dv, dctx.float().view(2, 5, 768).sum(1), atol=1e-5)


def test_vit_engine_matches_reference_golden(cuda, pkg, parity_report):
    fix = np.load(GOLDEN, allow_pickle=False)
    vm = pkg.vit_model
    B, L = int(fix["B"]), int(fix["L"])
    nb = vm.make_batch(B, L, seed=1)
    eng = pkg.vit_engine.VitVQAEngine(vm.make_state_dict(seed=0), batch=B, seq_len=L, warmup=int(fix["warmup"]),
                                      total=int(fix["total"]), dropout=0.0)
    losses, norms, gnorms, lp_err, pool_err = [], [], [], None, None
    for s in range(len(fix["losses"])):
        lp, loss = eng.forward_backward(nb)
        if s == 0:
            lp_err = float(np.abs(lp - fix["log_probs"]).max())
            pool = eng.vit_pooled().cpu().numpy()
            pool_err = float(np.abs(pool - fix["vit_pooled"]).max() / np.abs(fix["vit_pooled"]).max())
        gn = eng.group_grad_norms()
        gnorms.append([gn[k] for k in GROUPS])
        eng.optimizer_step()
        torch.cuda.synchronize()
        losses.append(loss)
        norms.append(eng.last_grad_norm())
    lrel = np.abs(np.array(losses) - fix["losses"]) / np.abs(fix["losses"])
    nrel = np.abs(np.array(norms) - fix["grad_norms"]) / fix["grad_norms"]
    grel = np.abs(np.array(gnorms) - fix["group_grad_norms"]) / fix["group_grad_norms"]
    post = eng.state_dict()
    init = vm.make_state_dict(seed=0)
    serr = {}
    for f, k in (("post_cls_w", "classification_layer.weight"), ("post_fuse_w", "fusing_layer.0.weight"),
                 ("post_dec_wi0", "lang_model.decoder.block.0.layer.2.DenseReluDense.wi.weight"),
                 ("post_dec_xv0", "lang_model.decoder.block.0.layer.1.EncDecAttention.v.weight"),
                 ("post_enc_q0", "lang_model.encoder.block.0.layer.0.SelfAttention.q.weight")):
        du = post[k][:4, :16].astype(np.float64) - init[k][:4, :16]
        dr = fix[f].astype(np.float64) - init[k][:4, :16]
        serr[f] = float(np.linalg.norm(du - dr) / max(np.linalg.norm(dr), 1e-30))
    # A/B: the CPU oracle fed the engine's own (bf16) ViT pooled output -- what is left is the
    # trained part's error; the rest is the frozen ViT's bf16 forward (12 pre-LN layers)
    from oracle import vit_oracle as orc
    ot = orc.VitOracleTrainer(vm.make_state_dict(seed=0), warmup=int(fix["warmup"]), total=int(fix["total"]))
    tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
    eng0 = pkg.vit_engine.VitVQAEngine(vm.make_state_dict(seed=0), batch=B, seq_len=L, dropout=0.0)
    lp0, loss0 = eng0.forward_backward(nb)
    olp, oloss = ot.forward_backward(tb, pooled=eng0.vit_pooled().cpu())
    og = ot.group_grad_norms()
    g0 = eng0.group_grad_norms()
    grads = {k: (ot.sd[k].grad.numpy() if ot.sd[k].grad is not None else np.zeros(tuple(ot.sd[k].shape), np.float32))
             for k in ot.sd if not k.startswith("vision_model.")}
    go = eng0.lay.pack(grads)
    ge = eng0.G32.cpu().numpy()
    ab = {"log_prob_max_abs": float(np.abs(lp0 - olp.numpy()).max()),
          "loss_rel": abs(loss0 - float(oloss)) / float(oloss),
          "group_grad_norm_rel": {k: abs(g0[k] - og[k]) / og[k] for k in GROUPS},
          "gradient_rel_l2": float(np.linalg.norm(ge - go) / np.linalg.norm(go))}
    del eng0
    # the same A/B over the whole 3-step trajectory: the ViT is frozen and the batch fixed, so its
    # pooled output is the same every step -- the oracle trained on the engine's pooled output
    # separates the trained part's error from the frozen ViT's bf16 forward (op for op equal to
    # bf16-operand arithmetic: tools/vit_layer_diag.py, profiles/r04_vit_layer_diag.json)
    ot2 = orc.VitOracleTrainer(vm.make_state_dict(seed=0), warmup=int(fix["warmup"]), total=int(fix["total"]))
    pe = torch.as_tensor(pool)
    g2, n2, l2 = [], [], []
    for _ in range(len(fix["losses"])):
        _, lo = ot2.forward_backward(tb, pooled=pe)
        gg = ot2.group_grad_norms()
        g2.append([gg[k] for k in GROUPS])
        n2.append(float(ot2.clip_and_step()))
        l2.append(float(lo))
    grel2 = np.abs(np.array(gnorms) - np.array(g2)) / np.array(g2)
    nrel2 = np.abs(np.array(norms) - np.array(n2)) / np.array(n2)
    lrel2 = np.abs(np.array(losses) - np.array(l2)) / np.abs(np.array(l2))
    parity_report["vit_golden_b4_l16"] = {
        "with_engine_vit_pooled": ab,
        "trajectory_with_engine_vit_pooled": {"group_grad_norm_rel_per_step": [dict(zip(GROUPS, r)) for r in grel2.tolist()],
                                              "grad_norm_rel": nrel2.tolist(), "loss_rel": lrel2.tolist()},
        "vit_pooled_rel": pool_err, "log_prob_max_abs": lp_err, "loss_rel": lrel.tolist(),
        "grad_norm_rel": nrel.tolist(), "group_grad_norm_rel_per_step": [dict(zip(GROUPS, r)) for r in grel.tolist()],
        "post_slice_err_over_update": serr}
    # the frozen ViT in bf16 (pooled max-abs 1.2e-2 of its max, measured) moves the fused token
    # and with it every downstream gradient: step 0 grad norms 4-6e-3 (measured); with the
    # engine's own pooled output the oracle agrees to the ResNet path's level (A/B above)
    # measured (r03 / r04): pooled 1.24e-2, log-probs 1.07e-2, step-0 loss 1.2e-4 / grad norm 4.3e-3,
    # step-0/1 groups <= 5.6e-3; step 2 (after the first nonzero-lr update, lr up to 5e-3 on T5):
    # lang_model 0.114, classifier 0.025, fusing 0.017, grad norm 3.2e-2, loss 4.9e-3
    assert pool_err <= 2e-2, pool_err
    assert lp_err <= 2e-2, lp_err
    assert lrel[0] <= 3e-4 and nrel[0] <= 1e-2, (lrel, nrel)
    for s_, lim in ((0, 1e-2), (1, 1e-2), (2, 0.2)):
        assert (grel[s_] <= lim).all(), (s_, dict(zip(GROUPS, grel[s_])))
    # A/B: the oracle trained on the engine's own (bf16) pooled ViT output.  Measured (r04):
    # steps 0-1 unchanged (grad norm 4.3e-3, loss 9e-5); step 2 grad norm 3.2e-2 -> 2.4e-2,
    # loss 4.9e-3 -> 2.8e-3 -- the frozen ViT's bf16 output is ~40 % of the step-2 drift; the rest
    # (lang_model group 0.114 -> 0.131) is the T5 / SGA path's own bf16 arithmetic amplified by
    # the first nonzero-lr AdamW step (profiles/r04_vit_layer_diag.json: every engine op is
    # within bf16 rounding of the same op on bf16 operands)
    assert (grel2[:2] <= 1e-2).all() and (grel2[2] <= 0.2).all(), grel2
    assert (nrel2[:2] <= 1e-2).all() and nrel2[2] <= 3e-2 and (lrel2[:2] <= 1e-3).all() and lrel2[2] <= 4e-3, \
        (nrel2, lrel2)
    assert nrel2[2] < nrel[2] and lrel2[2] < lrel[2], (nrel, nrel2, lrel, lrel2)
    assert ab["log_prob_max_abs"] <= 2e-2 and ab["loss_rel"] <= 1e-3, ab
    # at B = 4 the T5 gradient enters through 4 answer rows and 4 CLS rows only, so the bf16
    # rounding does not average out (group norms 5e-3 at B = 4, 1.5e-3 at B = 32, measured
    # with tools/vit_grad_diag.py); the whole gradient vector: relative L2 5.3e-2 at both
    # (cosine 0.9986), the bf16-vs-fp32 floor of the path (ReLU units within rounding of 0)
    assert max(ab["group_grad_norm_rel"].values()) <= 1e-2, ab
    assert ab["gradient_rel_l2"] <= 0.1, ab
    # after two AdamW updates (lr up to 5e-3 on T5): m / sqrt(v) turns near-zero gradients'
    # rounding into O(lr) update differences
    assert (lrel <= 1e-2).all() and (nrel <= 5e-2).all(), (lrel, nrel)
    assert max(serr.values()) <= 0.5, serr          # measured <= 0.35 (post_dec_xv0)


@pytest.mark.parametrize("planned", [3, 5])
def test_vit_engine_vs_oracle_train_mode(cuda, pkg, parity_report, planned):
    """Dropout on (p = 0.1 at the T5 sites, 0.5 at the fusing layer), masks from the shared
    counter hash; two steps, the second through a captured graph.  planned = 5: the engine is
    planned for 5 rows and trains on 3-row batches (a loader's short last batch: padded rows,
    ignore_index targets), against the oracle on the 3 rows."""
    from oracle import vit_oracle as orc
    vm = pkg.vit_model
    B, L, Ld = 3, 24, 12
    sd = vm.make_state_dict(seed=4)
    eng = pkg.vit_engine.VitVQAEngine(sd, batch=planned, seq_len=L, dec_len=Ld, warmup=1, total=40, dropout=0.1,
                                      seed=9)
    ot = orc.VitOracleTrainer(sd, warmup=1, total=40, dropout=0.1, seed=9)
    rec = []
    for step in range(2):
        nb = vm.make_batch(B, L, dec_len=Ld, seed=20 + step)
        tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
        if step == 0:
            lp, loss = eng.forward_backward(nb)
            eng.optimizer_step()
        else:
            eng.load_batch(nb)
            eng.capture()
            eng.train_step()
            torch.cuda.synchronize()
            lp, loss = eng.LOGP[:eng.rows].cpu().numpy(), float(eng.LOSS.item())
        assert lp.shape == (B, eng.A)
        olp, oloss, ogn = ot.train_one_step(tb)
        torch.cuda.synchronize()
        rec.append({"log_prob_max_abs": float(np.abs(lp - olp.numpy()).max()),
                    "loss_rel": abs(loss - float(oloss)) / abs(float(oloss)),
                    "grad_norm_rel": abs(eng.last_grad_norm() - float(ogn)) / float(ogn)})
    parity_report[f"vit_oracle_train_mode_planned{planned}"] = rec
    for step, r in enumerate(rec):
        assert r["log_prob_max_abs"] <= 2e-2 * (1 + step), (step, r)
        assert r["loss_rel"] <= 1e-3 * (1 + 2 * step), (step, r)
        # B = 3: the gradient enters through 3 answer rows (see the golden test: measured 4.6e-3)
        assert r["grad_norm_rel"] <= 1e-2 * (1 + step), (step, r)


def test_vit_model_api_and_trainer(cuda, pkg, tmp_path):
    """The VitVQAModel mirror: forward(**batch), generate_answers, state_dict round trip through
    torch.save / torch.load(weights_only=True), and VQATrainer steps with the ViT groups."""
    vm = pkg.vit_model
    B, L, Ld = 2, 16, 12
    model = pkg.model.VitVQAModel(answer_spaces=170, batch_size=B, seq_len=L, dec_len=Ld, dropout=0.1)
    nb = {k: (None if v is None else torch.as_tensor(v).cuda()) for k, v in
          vm.make_batch(B, L, dec_len=Ld, seed=3).items()}
    model.eval()
    lp, loss = model(**nb)
    lp2, loss2, att = model.generate_answers(**nb)
    assert torch.equal(lp, lp2) and float(loss) == float(loss2)
    assert len(att) == 12 and all(a.shape == (B, 12, 197, 197) for a in att)
    assert model.convert_logits_to_predictions(lp).shape == (B,)
    names = [n for n, _ in model.lang_model.named_parameters()]
    assert "shared.weight" in names and "decoder.block.0.layer.1.EncDecAttention.v.weight" in names
    path = tmp_path / "vit.pt"
    torch.save(model.state_dict(), path)
    sd = torch.load(path, weights_only=True)
    model2 = pkg.model.VitVQAModel(batch_size=B, seq_len=L, dec_len=Ld, state_dict=sd)
    model2.eval()
    lp3, _ = model2(**nb)
    assert torch.equal(lp, lp3)
    model.train()
    tr = pkg.trainer.VQATrainer(model, {"type": "AdamW", "lm_encoder_lr": 1e-4, "classifier_lr": 1e-4,
                                        "kwargs": {"weight_decay": 0.1, "amsgrad": True}},
                                {"num_warmup_steps": 1}, num_training_steps=10, logger=None)
    l0, _ = tr.train_one_step(nb)
    l1, _ = tr.train_one_step(nb)
    assert np.isfinite(l0) and np.isfinite(l1) and tr.grad_norm() > 0
    res = tr.valid_one_epoch([nb])
    assert 0.0 <= res["accuracy"] <= 1.0 and len(res["predictions"]) == B


def test_vit_optimizer_checkpoint_resumes_bit_identically(cuda, pkg, tmp_path):
    """The ViT trainer's optimizer checkpoint (vit_vqa_trainer.py:298-331: four groups -- vision,
    language, fusion, classifier -- resumed from state_dict_checkpoint.pt): save after two steps,
    rebuild model + trainer from the weights file and the checkpoint (weights_only loads), and
    the next two steps equal the uninterrupted run's bit for bit; the saved optimizer entry loads
    into torch.optim.AdamW over reference-shaped parameters."""
    vm = pkg.vit_model
    B, L, Ld = 2, 16, 12
    batches = [{k: (None if v is None else torch.as_tensor(v).cuda()) for k, v in
                vm.make_batch(B, L, dec_len=Ld, seed=60 + i).items()} for i in range(4)]
    okw = {"type": "AdamW", "lm_encoder_lr": 5e-3, "classifier_lr": 1e-5, "vision_lr": 8e-3,
           "kwargs": {"weight_decay": 0.1, "amsgrad": True}}

    def fresh(sd=None):
        m = pkg.model.VitVQAModel(answer_spaces=170, batch_size=B, seq_len=L, dec_len=Ld, dropout=0.1, state_dict=sd)
        return m, pkg.trainer.VQATrainer(m, okw, {"num_warmup_steps": 2}, num_training_steps=20, logger=None)
    m, tr = fresh()
    for b in batches[:2]:
        tr.train_one_step(b)
    torch.save(m.state_dict(), tmp_path / "best-model.pt")
    tr.save_state_dict_checkpoint(tmp_path / "state_dict_checkpoint.pt", epoch=1)
    ref_losses = [tr.train_one_step(b)[0] for b in batches[2:]]
    ref_p, ref_m = m.state_dict(), m.engine.optimizer_state()[0]
    m2, tr2 = fresh(torch.load(tmp_path / "best-model.pt", weights_only=True))
    assert tr2.load_state_dict_checkpoint(tmp_path / "state_dict_checkpoint.pt") == 1
    losses = [tr2.train_one_step(b)[0] for b in batches[2:]]
    assert losses == ref_losses, (losses, ref_losses)
    p2, m2m = m2.state_dict(), m2.engine.optimizer_state()[0]
    for k in ref_p:
        assert torch.equal(p2[k], ref_p[k]), k
    for k in ref_m:
        assert np.array_equal(m2m[k], ref_m[k]), k
    ck = torch.load(tmp_path / "state_dict_checkpoint.pt", weights_only=True)
    specs = vm.model_specs(170)
    groups = [{"params": [torch.zeros(specs[k]) for k in keys], "lr": lr} for _, lr, keys in tr._param_groups()]
    assert [g for g, _, _ in tr._param_groups()] == ["Vision Model", "Language Model", "Fusion Layer",
                                                       "Classifier Layer"]
    opt = torch.optim.AdamW(groups, weight_decay=0.1, amsgrad=True)
    opt.load_state_dict(ck["optimizer"])
    assert len(opt.state_dict()["state"]) == len(ck["optimizer"]["state"]) > 0 and ck["scheduler"]["last_epoch"] == 2


def test_vit_trained_path_is_bf16_operand_arithmetic(cuda, pkg, parity_report):
    """Config 4's trained path (T5 encoder, fusing layer, T5 decoder, answer gather, head) at step 0
    on the golden batch (B = 4, L = 16, decoder 20, eval mode): the engine's error against the fp32
    oracle equals what bf16 MFMA operands alone give -- the same oracle under
    oracle/bf16_mode.Bf16Operands -- both fed the engine's pooled ViT output (the frozen ViT is
    checked op by op by tools/vit_layer_diag.py).  Measured (r05, tools/vit_trained_diag.py,
    profiles/r05_vit_trained_diag.json): the whole gradient's relative L2 vs fp32 5.26e-2 (engine)
    vs 5.27e-2 (bf16 operands); per parameter tensor the engine / bf16-operand ratio 0.75-1.25;
    every decoder layer's hidden state within 1.06x."""
    from oracle import vit_oracle as orc
    from oracle.bf16_mode import Bf16Operands
    vm = pkg.vit_model
    B, L = 4, 16
    nb = vm.make_batch(B, L, seed=1)
    sd = vm.make_state_dict(seed=0)
    eng = pkg.vit_engine.VitVQAEngine(sd, batch=B, seq_len=L, dropout=0.0)
    lp, loss = eng.forward_backward(nb)
    pooled = eng.vit_pooled().cpu()
    ge = eng.G32.cpu().numpy().astype(np.float64)
    tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
    res = {}
    for mode in ("fp32", "bf16"):
        ot = orc.VitOracleTrainer(sd)
        if mode == "bf16":
            with Bf16Operands():
                olp, oloss = ot.forward_backward(tb, pooled=pooled)
        else:
            olp, oloss = ot.forward_backward(tb, pooled=pooled)
        grads = {k: ot.sd[k].grad.numpy() for k in ot.keys}
        res[mode] = (olp.numpy().astype(np.float64), float(oloss), eng.lay.pack(grads).astype(np.float64))
    (lp32, l32, g32), (lp16, l16, g16) = res["fp32"], res["bf16"]
    rl = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))   # noqa: E731
    rep = {"grad_rel_l2": {"engine": rl(ge, g32), "bf16_operands": rl(g16, g32)},
           "log_probs_rel_l2": {"engine": rl(lp.astype(np.float64), lp32), "bf16_operands": rl(lp16, lp32)},
           "group_grad_rel_l2": {}}
    for g, (a, e) in eng.lay.groups.items():
        rep["group_grad_rel_l2"][g] = {"engine": rl(ge[a:e], g32[a:e]), "bf16_operands": rl(g16[a:e], g32[a:e])}
    parity_report["vit_trained_path_vs_bf16_operands"] = rep
    # the engine's error is bf16 arithmetic: within 1.5x of the bf16-operand oracle's (measured ~1.0x),
    # for the whole gradient, each group's and the log-probs
    for k in ("grad_rel_l2", "log_probs_rel_l2"):
        assert rep[k]["engine"] <= 1.5 * rep[k]["bf16_operands"], (k, rep[k])
    for g, v in rep["group_grad_rel_l2"].items():
        assert v["engine"] <= 1.5 * v["bf16_operands"] + 1e-6, (g, v)
