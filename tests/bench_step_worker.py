"""The benched step (BASELINE configs[1]) against the CPU oracle.

  python tests/bench_step_worker.py OUT.json [dp|c5]   (stand-alone: writes the report to OUT.json)

`run()` is called in the pytest session process by
tests/test_z_bench_step_gpu.py::test_bench_step_b64_matches_oracle, after every other GPU
test.  The engine is built exactly as bench.py main() builds it (R50, B=64, 224x224, L=32,
pipelined frozen ResNet, tuned tile / split-K table, captured hipGraph step, deferred AdamW,
dropout 0.1 from the shared counter hash) and stepped against the CPU oracle
(trainer/faster_rcnn_vqa_trainer.py:391-406)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from oracle import vqa_oracle as orc  # noqa: E402  (test infrastructure: the checker)

TABLE = os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json")
GROUPS = ("lang_model", "scaler", "sga_modules", "attention_pooler", "classification_layer")
# bf16 GEMM operands / fp32 accumulate vs the fp32 oracle (log-probs 5e-2, loss
# 5e-3, total grad-norm 1e-3, per-group 5e-3), tightened to what is met with margin (measured
# at B=64: log-probs <= 1.2e-2, loss <= 4.4e-5, grad-norm <= 6.2e-4, per-group <= 9.7e-4).
# Train-mode steps with identical dropout masks.
LP_TOL, LOSS_RTOL, GN_RTOL, GROUP_RTOL = 2e-2, 5e-4, 1e-3, 5e-3


def _dev(nb):
    return {k: torch.as_tensor(v).cuda() for k, v in nb.items() if v is not None}


def _world1_group():
    """A world-1 RCCL process group for the DP mode (bench.py --dp), unless one exists."""
    import socket
    import torch.distributed as dist
    if dist.is_initialized():
        return False
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    return True


# config 5 (fp8 engine vs the fp8 restatement in the oracle): bf16 operands outside the e4m3
# linears and flips of an e4m3 rounding wherever the engine's bf16 activations differ from the
# oracle's by an ulp (tests/test_config5_gpu.py measured at B = 2: log-probs <= 6.2e-2, loss
# <= 2.5e-3, grad norm <= 9.9e-4); the same bounds at the benched B = 64
C5_LP_TOL, C5_LOSS_RTOL, C5_GN_RTOL, C5_GROUP_RTOL, C5_POOLER_RTOL = 0.1, 5e-3, 2e-3, 1e-2, 3e-2


def run(mode="engine"):
    """Build, tune, capture and step the benched engine against the oracle; returns (report, fails).
    mode "dp": the N > 1 step at world 1 -- dp.DataParallelStep over a world-1 RCCL group on the
    DP engine (T5 weight-gradient groups dp.DP_T5_DW_GROUPS), built as `bench.py --dp` builds it;
    mode "c5": BASELINE configs[4] as `bench.py --config5` builds it (T5-large, 6 SGA blocks at
    width 1024, 384 x 384 images, e4m3 forward weight GEMMs) against the oracle's fp8 restatement,
    2 steps."""
    pkg = load_package()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    dp, c5 = mode == "dp", mode == "c5"
    B, L, H = 64, 32, (384 if c5 else 224)
    NB, lm = (6, "t5-large") if c5 else (3, "t5-base")
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=NB, language_model=lm)
    own_pg = _world1_group() if dp else False
    # bench.py main(): same constructor arguments, same priming / tuning / capture sequence
    eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=L, image_size=H, warmup=10, total=100000,
                               dropout=0.1, seed=0, pipeline=True, num_blocks=NB, language_model=lm, fp8=c5,
                               t5_dw_group=pkg.dp.DP_T5_DW_GROUPS if dp else None)
    assert eng.defer_opt and eng.pipeline and eng.dw_stream
    nsteps = 2 if c5 else 3
    nbs = [pkg.synthetic.make_batch(B, L, H, seed=1 + i) for i in range(nsteps + 1)]
    pool = [_dev(nb) for nb in nbs]
    eng.prime(pool[0]["image_tensors"])
    eng.F4.copy_(eng.F4N)
    eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
    eng.forward()
    eng.backward()
    eng.autotune(table=TABLE)
    if dp:
        dps = pkg.dp.DataParallelStep(eng, use_graph=True)
        step = dps.step
    else:
        eng.capture()
        step = eng.train_step
    eng.prime(pool[0]["image_tensors"])
    splitk = sum(1 for c in eng.res_calls + eng.fwd_calls + eng.bwd_calls if c.name == "vqa_gemm" and c.desc.splitk > 1)

    ot = orc.OracleTrainer(sd, "resnet50", warmup=10, total=100000, dropout=0.1, seed=0, num_blocks=NB, fp8=c5)
    p0 = {k: v.detach().clone() for k, v in ot.sd.items() if k in ot.keys}
    rep = {"splitk_launches": splitk}
    fails = []
    for i in range(nsteps):
        ot.rng_counter = int(eng.RNG[1].item())             # the same dropout draw (engine bumps, then uses)
        eng.load_batch(pool[i], next_images=pool[i + 1]["image_tensors"])
        step()
        torch.cuda.synchronize()
        lp, loss, gn = eng.LOGP.cpu().numpy(), float(eng.LOSS.item()), eng.last_grad_norm()
        ggn = eng.group_grad_norms()
        olp, oloss = ot.forward_backward(orc.to_torch_batch(nbs[i]))
        ogg = ot.group_grad_norms()
        ogn = float(ot.clip_and_step())
        lp_err = float(np.abs(lp - olp.numpy()).max())
        loss_rel = abs(loss - float(oloss)) / abs(float(oloss))
        gn_rel = abs(gn - ogn) / ogn
        grp = {g: abs(ggn[g] - ogg[g]) / ogg[g] for g in GROUPS}
        rep[f"step{i}"] = {"log_prob_max_abs": lp_err, "loss_rel": loss_rel, "grad_norm_rel": gn_rel,
                           "group_grad_norm_rel": grp, "loss": loss, "grad_norm": gn}
        if c5:
            other = max(v for g, v in grp.items() if g != "attention_pooler")
            checks = (("log_probs", lp_err > C5_LP_TOL), ("loss", loss_rel > C5_LOSS_RTOL),
                      ("grad_norm", gn_rel > C5_GN_RTOL * (1 + i)), ("group_grad_norms", other > C5_GROUP_RTOL * (1 + i)),
                      ("pooler_grad_norm", grp["attention_pooler"] > C5_POOLER_RTOL * (1 + i)))
        else:
            checks = (("log_probs", lp_err > LP_TOL), ("loss", loss_rel > LOSS_RTOL),
                      ("grad_norm", gn_rel > GN_RTOL * (1 + i)),
                      ("group_grad_norms", max(grp.values()) > GROUP_RTOL * (1 + i)))
        fails += [(i, what) for what, bad in checks if bad]
    # parameters after the updates (deferred update flushed), per group: L2 error of the
    # update vectors relative to the oracle's update
    post = eng.state_dict()
    delta = {}
    for g in GROUPS:
        num = den = 0.0
        for k in ot.keys:
            if orc.group_of(k) != g:
                continue
            do = (ot.sd[k].detach() - p0[k]).double().numpy()
            de = post[k].astype(np.float64) - p0[k].double().numpy()
            num += float(((de - do) ** 2).sum())
            den += float((do ** 2).sum())
        delta[g] = (num / den) ** 0.5 if den > 0 else 0.0
    rep["update_rel_l2"] = delta
    rep["mode"] = mode
    if dp:
        rep["buckets"] = len(dps.buckets)
    torch.cuda.synchronize()
    if own_pg:
        import torch.distributed as dist
        dist.destroy_process_group()
    return rep, fails


def main(out_path, mode="engine"):
    rep, fails = run(mode)
    json.dump({"report": rep, "fails": fails}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:3])
