"""Pin the CPU oracle against golden vectors produced by the reference modules
(tests/golden/make_golden.py).  CPU only."""
import hashlib

import numpy as np
import pytest
import torch

from oracle import vqa_oracle as orc

torch.set_num_threads(8)


def _sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def test_relative_position_buckets(golden):
    g = golden("t5_encoder")
    got = orc.t5_relative_position_bucket(torch.as_tensor(g["rel"])).numpy()
    np.testing.assert_array_equal(got, g["buckets"])


@pytest.mark.parametrize("case,lm", [("t5_encoder", "t5-base"), ("t5_large_encoder", "t5-large")])
def test_t5_encoder_matches_reference(golden, pkg, case, lm):
    """t5-large: transformers' T5Stack built from a T5Config of the published t5-large sizes
    (24 layers, d 1024, 16 heads, d_ff 4096; BASELINE configs[4])."""
    g = golden(case)
    keys = {k for k in pkg.synthetic.model_specs("resnet50", language_model=lm) if k.startswith("lang_model.")}
    sd = {k: torch.as_tensor(v)
          for k, v in pkg.synthetic.make_state_dict("resnet50", keys=keys, language_model=lm).items()}
    h = orc.t5_encoder(sd, torch.as_tensor(g["ids"]), torch.as_tensor(g["mask"]))
    np.testing.assert_allclose(h.numpy(), g["hidden"], atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("case,lm", [("sga_block", "t5-base"), ("sga1024_block", "t5-large")])
def test_sga_block_matches_reference(golden, pkg, case, lm):
    """sga1024_block: the reference SGA built from configuration instances with HIDDEN_SIZE =
    FF_SIZE = 1024 (8 heads of 128), x [2, 32, 1024], y [2, 144, 1024] (config 5's 12 x 12 map)."""
    g = golden(case)
    keys = {k for k in pkg.synthetic.model_specs("resnet50", language_model=lm) if k.startswith("sga_modules.0.")}
    sd = {k: torch.as_tensor(v).requires_grad_(True)
          for k, v in pkg.synthetic.make_state_dict("resnet50", keys=keys, language_model=lm).items()}
    x = torch.tensor(g["x"], requires_grad=True)
    y = torch.tensor(g["y"], requires_grad=True)
    out = orc.sga_block(sd, "sga_modules.0", x, y)
    (out * torch.as_tensor(g["gout"])).sum().backward()
    np.testing.assert_allclose(out.detach().numpy(), g["out"], atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(x.grad.numpy(), g["dx"], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(y.grad.numpy(), g["dy"], atol=5e-5, rtol=1e-4)
    names = [str(n) for n in g["param_names"]]
    got = np.array([float(sd["sga_modules.0." + n].grad.norm()) for n in names])
    # linear_k biases have a mathematically zero gradient (softmax shift invariance): compare with atol
    np.testing.assert_allclose(got, g["param_grad_norms"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("case,vision,blocks,lm", [("model_r50_224_l32", "resnet50", 3, "t5-base"),
                                                    ("model_r34_256_l16", "resnet34", 3, "t5-base"),
                                                    ("model_r18_256_l16", "resnet18", 3, "t5-base"),
                                                    ("model_c5_r50_384_l32", "resnet50", 6, "t5-large")])
def test_full_step_matches_reference(golden, pkg, case, vision, blocks, lm):
    """model_c5_*: BASELINE configs[4] widths -- the reference ResnetVQAModel with its
    width-dependent children rebuilt at 1024 (t5-large encoder, 6 SGA blocks from 1024-wide
    configuration instances, ConvTranspose2d 2048 -> 1024, pooler and classifier at 1024) and
    its own forward, at 384 x 384 images (tests/golden/make_golden.py build_model_c5)."""
    g = golden(case)
    B, L, H = int(g["B"]), int(g["L"]), int(g["H"])
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    assert _sha(nb["image_tensors"]) == g["image_sha"], "synthetic image generator drifted"
    np.testing.assert_array_equal(nb["question_input_ids"], g["ids"])
    np.testing.assert_array_equal(nb["question_attention_masks"], g["mask"])
    np.testing.assert_array_equal(nb["annotation_ids"], g["targets"])
    sd = pkg.synthetic.make_state_dict(vision, seed=0, num_attention_blocks=blocks, language_model=lm)
    tr = orc.OracleTrainer(sd, vision, warmup=int(g["warmup"]), total=int(g["total"]), num_blocks=blocks)
    batch = orc.to_torch_batch(nb)
    losses, norms, gnorms = [], [], []
    for s in range(len(g["losses"])):
        lp, loss = tr.forward_backward(batch)
        if s == 0:
            np.testing.assert_allclose(lp.numpy(), g["log_probs"], atol=2e-4)
            with torch.no_grad():
                f = orc.resnet_features(tr.sd, batch["image_tensors"], vision).numpy()
            np.testing.assert_allclose(f[:, :8], g["feat_slice"], atol=1e-4, rtol=1e-4)
        gn = tr.group_grad_norms()
        gnorms.append([gn["lang_model"], gn["scaler"], gn["sga_modules"], gn["attention_pooler"],
                       gn["classification_layer"]])
        norms.append(float(tr.clip_and_step()))
        losses.append(float(loss))
    np.testing.assert_allclose(losses, g["losses"], rtol=2e-5)
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=2e-4)
    np.testing.assert_allclose(np.array(gnorms), g["group_grad_norms"], rtol=5e-4)
    sdp = tr.sd
    np.testing.assert_allclose(sdp["lang_model.block.0.layer.0.SelfAttention.q.weight"][:4, :16].detach().numpy(),
                               g["post_t5_q0"], atol=1e-5, rtol=1e-4)  # Adam step ~5e-3: 0.2% of one update
    np.testing.assert_allclose(sdp["classification_layer.weight"][:4, :16].detach().numpy(), g["post_cls_w"],
                               atol=1e-7, rtol=1e-5)
    np.testing.assert_allclose(sdp[f"sga_modules.{blocks - 1}.ffn.mlp.fc1.weight"][:4, :16].detach().numpy(),
                               g["post_sga_fc1"], atol=1e-5, rtol=1e-4)
