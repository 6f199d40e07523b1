"""Parity of single blocks on the GPU (the benched step: tests/test_a_bench_step_gpu.py).

* test_sga_block_matches_reference / test_t5_encoder_matches_reference: one
  SGA block (forward + backward from a given output gradient) and the T5
  encoder output, through the HIP kernels, against the fixtures the reference
  modules wrote (tests/golden/make_golden.py: sga_case, t5_case;
  model/multi_head_vision_text_attn.py:145-158, TF T5Stack).

Every measured error is recorded (conftest.parity_report ->
gpurun_out/parity_report.json -> profiles/r02_parity_*.json).  Tolerances are
bf16-MFMA-vs-fp32 bounds, stated next to each check."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _sga_engine(pkg, lm="t5-base"):
    # 7x7 = 49 vision tokens (sga_block's y) at 224; 12x12 = 144 (sga1024_block's) at 384
    B, L, H = 2, 32, (224 if lm == "t5-base" else 384)
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=1, language_model=lm)
    eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=L, image_size=H, warmup=2, total=10,
                               num_blocks=1, dropout=0.0, language_model=lm)
    eng.load_batch(pkg.synthetic.make_batch(B, L, H, seed=1))
    eng.forward()
    eng.backward()
    torch.cuda.synchronize()
    return eng


@pytest.mark.parametrize("case,lm", [("sga_block", "t5-base"), ("sga1024_block", "t5-large")])
def test_sga_block_matches_reference(cuda, pkg, golden, parity_report, case, lm):
    """SGA block 0 (x = given text, y = given vision tokens) through the HIP kernels:
    output, dL/dx, dL/dy and every parameter-gradient norm for dL/dout = gout.
    sga1024_block: the reference SGA at config 5's width (1024, 8 heads of 128, 144 keys)."""
    g = golden(case)
    eng = _sga_engine(pkg, lm)
    T = eng.T
    x = torch.as_tensor(g["x"]).reshape(T, -1).cuda()
    y = torch.as_tensor(g["y"]).reshape(eng.V_TOK, -1).cuda()
    eng.TXT32.copy_(x)
    eng.TXT16.copy_(x.bfloat16())
    eng.VIS32.copy_(y)
    eng.VIS16.copy_(y.bfloat16())
    eng._run(eng.sga_vision_calls)                           # block 0's k|v projection of y
    eng._run(eng.fwd_calls[eng._fsplit[2]:])                 # the SGA block (+ the head, unused here)
    b = eng.bwd_calls
    assert b[1].name == "vqa_head_bwd"
    eng._run(b[:2])
    eng.dY[0].copy_(torch.as_tensor(g["gout"]).reshape(T, -1).cuda())   # replace dL/dout by the fixture's
    eng._run(b[2:eng._bsplit[0]])
    torch.cuda.synchronize()
    out = eng.sga[0]["OUT"].cpu().numpy().reshape(g["out"].shape)
    dx = eng.dTXT.cpu().numpy().reshape(g["dx"].shape)
    dy = eng.dVIS32.cpu().numpy().reshape(g["dy"].shape)
    grads = eng.lay.unpack(eng.G32.cpu().numpy())
    names = [str(n) for n in g["param_names"]]
    pn = np.array([np.linalg.norm(grads["sga_modules.0." + n].astype(np.float64)) for n in names])

    def rel(a, r):
        return float(np.abs(a - r).max() / np.abs(r).max())
    rep = {"out_max_rel": rel(out, g["out"]), "dx_max_rel": rel(dx, g["dx"]), "dy_max_rel": rel(dy, g["dy"])}
    ref = g["param_grad_norms"]
    big = ref > 1e-3 * ref.max()                             # linear_k biases: mathematically zero gradient
    prel = np.abs(pn - ref)[big] / ref[big]
    rep["param_grad_norm_rel_max"] = float(prel.max())
    rep["param_grad_norm_rel"] = dict(zip([n for n, k in zip(names, big) if k], map(float, prel)))
    parity_report[case] = rep
    # bf16 GEMM operands (8 bits of mantissa) through a post-LN block: a few 1e-3 of the range
    assert rep["out_max_rel"] <= 2e-2 and rep["dx_max_rel"] <= 3e-2 and rep["dy_max_rel"] <= 3e-2, rep
    assert rep["param_grad_norm_rel_max"] <= 2e-2, rep


@pytest.mark.parametrize("case,lm", [("t5_encoder", "t5-base"), ("t5_large_encoder", "t5-large")])
def test_t5_encoder_matches_reference(cuda, pkg, golden, parity_report, case, lm):
    """T5-base / T5-large encoder last_hidden_state (eval) through the HIP kernels vs the fixture."""
    g = golden(case)
    B, L, H = 2, 32, 32
    nb = pkg.synthetic.make_batch(B, L, H, seed=3)
    np.testing.assert_array_equal(nb["question_input_ids"], g["ids"])
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, language_model=lm)
    eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=L, image_size=H, warmup=2, total=10,
                               dropout=0.0, language_model=lm)
    eng.load_batch(nb)
    eng.forward()
    torch.cuda.synchronize()
    h = eng.TXT32.cpu().numpy().reshape(g["hidden"].shape)
    ref = g["hidden"]
    err = float(np.abs(h - ref).max() / np.abs(ref).max())
    cos = float((h * ref).sum() / np.sqrt((h * h).sum() * (ref * ref).sum()))
    parity_report[case] = {"hidden_max_rel": err, "cosine": cos}
    assert err <= 3e-2 and cos >= 0.9995, (err, cos)
