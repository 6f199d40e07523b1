"""Config 4 (VitVQAModel): the CPU oracle against the fixture generated from the reference
model itself (tests/golden/make_golden_vit.py), and the flat-arena layout round trip."""
import os

import numpy as np
import pytest
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vit_model_b4_l16.npz")


@pytest.fixture(scope="module")
def fix():
    return np.load(GOLDEN, allow_pickle=False)


def test_vit_layout_round_trip(pkg):
    vm = pkg.vit_model
    sd = vm.make_state_dict(seed=0)
    lay = vm.VitLayout()
    flat = lay.pack(sd)
    back = lay.unpack(flat)
    for k in lay.trainable_keys:
        assert np.array_equal(back[k], sd[k]), k
    specs = vm.model_specs()
    trainable = [k for k in specs if not k.startswith("vision_model.")]
    assert sorted(set(lay.trainable_keys)) == sorted(trainable)
    assert lay.num_params == sum(int(np.prod(specs[k])) for k in trainable if k not in vm.TIED)


def test_causal_bucket_map_matches_transformers(pkg):
    from transformers.models.t5.modeling_t5 import T5Attention
    L = 40
    rel = torch.arange(L)[None, :] - torch.arange(L)[:, None]
    ref = T5Attention._relative_position_bucket(rel, bidirectional=False, num_buckets=32, max_distance=128).numpy()
    got = pkg.vit_model.causal_bucket_map(L)
    keep = np.tril(np.ones((L, L), bool))
    assert np.array_equal(got[keep], ref[keep])
    assert (got[~keep] == -1).all()


def test_vit_oracle_matches_reference(pkg, fix):
    from oracle import vit_oracle as orc
    vm = pkg.vit_model
    B, L = int(fix["B"]), int(fix["L"])
    nb = vm.make_batch(B, L, seed=1)
    assert np.array_equal(nb["question_input_ids"], fix["ids"])
    assert np.array_equal(nb["decoder_question_input_ids"], fix["dec_ids"])
    batch = {k: (None if v is None else torch.as_tensor(v)) for k, v in nb.items()}
    tr = orc.VitOracleTrainer(vm.make_state_dict(seed=0), warmup=int(fix["warmup"]), total=int(fix["total"]))
    with torch.no_grad():
        pooled = orc.vit_pooled(tr.sd, batch["pixel_values"]).numpy()
    assert np.abs(pooled - fix["vit_pooled"]).max() <= 2e-5 * max(1.0, np.abs(fix["vit_pooled"]).max())
    losses, norms = [], []
    for s in range(len(fix["losses"])):
        lp, loss = tr.forward_backward(batch)
        if s == 0:
            assert np.abs(lp.numpy() - fix["log_probs"]).max() <= 2e-5
        g = tr.group_grad_norms()
        got = np.array([g["lang_model"], g["fusing_layer"], g["classification_layer"]])
        assert np.allclose(got, fix["group_grad_norms"][s], rtol=2e-4, atol=1e-7), (s, got, fix["group_grad_norms"][s])
        norms.append(float(tr.clip_and_step()))
        losses.append(float(loss))
    assert np.allclose(losses, fix["losses"], rtol=1e-5), (losses, fix["losses"])
    assert np.allclose(norms, fix["grad_norms"], rtol=2e-4), (norms, fix["grad_norms"])
    post = {"post_cls_w": "classification_layer.weight", "post_fuse_w": "fusing_layer.0.weight",
            "post_dec_wi0": "lang_model.decoder.block.0.layer.2.DenseReluDense.wi.weight",
            "post_dec_xv0": "lang_model.decoder.block.0.layer.1.EncDecAttention.v.weight",
            "post_enc_q0": "lang_model.encoder.block.0.layer.0.SelfAttention.q.weight"}
    for f, k in post.items():
        got = tr.sd[k].detach()[:4, :16].numpy()
        assert np.allclose(got, fix[f], rtol=1e-4, atol=1e-6), (f, np.abs(got - fix[f]).max())
