"""Parity of config 4's benched step (BASELINE configs[3], VitVQAModel) on the GPU.

The engine built exactly as `bench.py --model vit` builds it (B = 64, L = 32, decoder 20, the
tuned tile / split-K table, captured hipGraph step, train-mode dropout 0.1 at the T5 sites and
0.5 at the fusing layer from the shared counter hash) against the CPU fp32 oracle
(oracle/vit_oracle.py, pinned to a reference-generated fixture) fed the same batches and
dropout masks, three steps: log-probs, loss, total and per-group grad norms, then the
parameter updates per group (model/vit_vqa_model.py:168-227; trainer/vit_vqa_trainer.py:450-464).
Runs in the session process after the other GPU tests (this file sorts last)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json")
GROUPS = ("lang_model", "fusing_layer", "classification_layer")


def test_vit_bench_step_b64_matches_oracle(pkg, parity_report):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from oracle import vit_oracle as orc
    torch.set_num_threads(16)
    vm = pkg.vit_model
    B, L, Ld = 64, 32, 20
    sd = vm.make_state_dict(seed=0)
    eng = pkg.vit_engine.VitVQAEngine(sd, batch=B, seq_len=L, dec_len=Ld, warmup=10, total=100000, dropout=0.1)
    nbs = [vm.make_batch(B, L, dec_len=Ld, seed=1 + i) for i in range(3)]
    dev = lambda nb: {k: (None if v is None else torch.as_tensor(v).cuda()) for k, v in nb.items()}
    # bench_vit: load, one eager step's activations for the tuner, tune, capture
    eng.load_batch(dev(nbs[0]))
    eng.forward()
    eng.backward()
    eng.autotune(table=TABLE)
    eng.capture()
    ot = orc.VitOracleTrainer(sd, warmup=10, total=100000, dropout=0.1, seed=0)
    # the A/B (tools/drift_ab_vit.py, tools/vit_layer_diag.py): the same oracle trained on the
    # engine's own bf16 ViT pooled output of each batch -- what is left is the trained part's error
    ot2 = orc.VitOracleTrainer(sd, warmup=10, total=100000, dropout=0.1, seed=0)
    p0 = {k: v.detach().clone() for k, v in ot.sd.items() if not k.startswith("vision_model.")}
    rep, rep2 = {}, {}

    def cmp(lp, loss, gn, ggn, olp, oloss, ogn, ogg):
        return {"log_prob_max_abs": float(np.abs(lp - olp.numpy()).max()),
                "loss_rel": abs(loss - float(oloss)) / abs(float(oloss)), "grad_norm_rel": abs(gn - ogn) / ogn,
                "group_grad_norm_rel": {g: abs(ggn[g] - ogg[g]) / ogg[g] for g in GROUPS}}
    for i, nb in enumerate(nbs):
        ot.rng_counter = ot2.rng_counter = int(eng.RNG[1].item())   # the same dropout draw (engine bumps, then uses)
        eng.load_batch(dev(nb))
        eng.train_step()
        torch.cuda.synchronize()
        lp, loss, gn = eng.LOGP.cpu().numpy(), float(eng.LOSS.item()), eng.last_grad_norm()
        ggn = eng.group_grad_norms()
        pooled = eng.vit_pooled().cpu()
        tb = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
        olp, oloss = ot.forward_backward(tb)
        ogg = ot.group_grad_norms()
        ogn = float(ot.clip_and_step())
        rep[f"step{i}"] = cmp(lp, loss, gn, ggn, olp, oloss, ogn, ogg)
        olp, oloss = ot2.forward_backward(tb, pooled=pooled)
        ogg = ot2.group_grad_norms()
        ogn = float(ot2.clip_and_step())
        rep2[f"step{i}"] = cmp(lp, loss, gn, ggn, olp, oloss, ogn, ogg)
    post = eng.state_dict()

    def upd(o):
        delta = {}
        for g in GROUPS:
            num = den = 0.0
            for k, v0 in p0.items():
                if orc.group_of(k) != g or k not in post:
                    continue
                do = (o.sd[k].detach() - v0).double().numpy()
                de = post[k].astype(np.float64) - v0.double().numpy()
                num += float(((de - do) ** 2).sum())
                den += float((do ** 2).sum())
            delta[g] = (num / den) ** 0.5 if den > 0 else 0.0
        return delta
    delta = upd(ot)
    rep["update_rel_l2"] = delta
    rep2["update_rel_l2"] = upd(ot2)
    rep["with_engine_vit_pooled"] = rep2
    parity_report["vit_bench_b64"] = rep
    for i in range(3):
        r = rep[f"step{i}"]
        # bf16 arithmetic: the fp32 oracle under oracle/bf16_mode.Bf16Operands (every matmul on
        # bf16 operands) against the plain fp32 oracle on these batches measures log-probs
        # 1.7e-2 / 1.7e-2 / 8.8e-2, loss <= 1.6e-4, grad norm <= 1.9e-3, groups <= 1.6e-2 (fusing
        # layer, step 2) (tools/drift_ab_vit.py, profiles/r05_drift_ab_vit.json); the engine
        # measured 1.9e-2 / 1.6e-2 / 0.10, loss <= 2.6e-4, grad norm <= 1.2e-3, groups <= 7.8e-3:
        # the bounds are ~1.5x the bf16-operand oracle's own error (step 2 follows the first
        # nonzero-lr AdamW update, which moves every weight by ~lr * sign(g): a near-zero
        # gradient's rounding becomes an O(lr) difference in either arithmetic)
        assert r["log_prob_max_abs"] <= (3e-2 if i < 2 else 0.13), rep
        assert r["loss_rel"] <= 5e-4, rep
        assert r["grad_norm_rel"] <= 2.5e-3, rep
        assert max(r["group_grad_norm_rel"].values()) <= (5e-3 if i < 2 else 2.5e-2), rep
    # relative L2 of the per-group update vectors after three steps: measured 0.04 (classifier),
    # 0.16 (T5), 0.19 (fusing layer); the bf16-operand oracle: 0.037 / 0.14 / 0.19
    assert max(delta.values()) <= 0.25, delta
    # A/B with the engine's pooled outputs fed to the oracle: at B = 64 it does NOT bring the
    # oracle closer (measured r04: step-2 log-probs 0.110 vs 0.100, grad norm 2.6e-3 vs 1.2e-3):
    # the step-2 log-prob error is the first nonzero-lr AdamW update moving every weight by
    # ~lr * sign(g) on near-zero gradient entries, not the frozen ViT's bf16 forward
    r2 = rep2["step2"]
    assert r2["log_prob_max_abs"] <= 0.13 and r2["grad_norm_rel"] <= 4e-3, rep2
    assert max(rep2["update_rel_l2"].values()) <= 0.25, rep2
