"""Host-side logic: flat arena layout <-> reference state_dict, bucket map,
BN folding.  CPU only."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("vision,count", [("resnet50", 141_648_171), ("resnet34", 141_648_171 - 14_156_544 + 3_539_712),
                                          ("resnet18", 141_648_171 - 14_156_544 + 3_539_712)])
def test_trainable_count_and_roundtrip(pkg, vision, count):
    lay = pkg.layout.ParamLayout(vision)
    assert lay.num_params == count
    keys = set(lay.trainable_keys)
    sd = pkg.synthetic.make_state_dict(vision, seed=3, keys=keys)
    flat = lay.pack(sd)
    back = lay.unpack(flat)
    assert set(back) == keys
    for k in keys:
        np.testing.assert_array_equal(back[k], sd[k])
    ends, lrs = lay.group_of_element()
    assert ends == sorted(ends) and ends[-1] == lay.total and lrs == [1e-5, 5e-4, 5e-4, 5e-4, 5e-3]
    for s in lay.segments.values():
        assert s.offset % 64 == 0


def test_t5_large_config5_layout_roundtrip(pkg):
    """BASELINE configs[4] widths (t5-large encoder, 6 SGA blocks, scaler / pooler / classifier at
    1024): the arena holds exactly the trainable entries of the reference state dict built at that
    width, and packs / unpacks them bit for bit."""
    S = pkg.synthetic
    lay = pkg.layout.ParamLayout("resnet50", 170, 6, "t5-large")
    specs = S.model_specs("resnet50", 170, 6, "t5-large")
    trainable = {k: v for k, v in specs.items() if not k.startswith(("vision_model.", "upscale_layer."))}
    assert set(lay.trainable_keys) == set(trainable)
    assert lay.num_params == sum(int(np.prod(v)) for v in trainable.values()) == 417_003_179
    assert specs["lang_model.block.23.layer.1.DenseReluDense.wi.weight"] == (4096, 1024)
    assert specs["lang_model.block.0.layer.0.SelfAttention.relative_attention_bias.weight"] == (32, 16)
    keys = {k for k in trainable if k.startswith(("sga_modules.5.", "lang_model.block.23.", "classification"))}
    sd = S.make_state_dict("resnet50", seed=5, num_attention_blocks=6, language_model="t5-large")
    back = lay.unpack(lay.pack(sd))
    for k in keys:
        np.testing.assert_array_equal(back[k], sd[k])


def test_convT_repack_is_equivalent_conv(pkg):
    lay = pkg.layout
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 16, 5, 5, generator=g)
    w = torch.randn(16, 8, 3, 3, generator=g)
    ref = F.conv_transpose2d(x, w, stride=1, padding=1)
    wc = torch.as_tensor(lay._convT_to_conv(w.numpy()))              # [Cout, kh, kw, Cin]
    got = F.conv2d(x, wc.permute(0, 3, 1, 2), padding=1)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(lay._conv_to_convT(wc.numpy()), w.numpy())


def test_bucket_map_matches_reference(pkg, golden):
    g = golden("t5_encoder")
    rel, buckets = g["rel"], g["buckets"]
    L = 41
    bm = pkg.layout.t5_bucket_map(L, 2 * L - 1)           # rel = j - i covers -40..80
    got = {int(j - 40): int(bm[40, j]) for j in range(0, 81)}   # row i=40 -> rel = j - 40
    for r, b in zip(rel, buckets):
        assert got[int(r)] == int(b), (r, got[int(r)], b)
    from oracle import vqa_oracle as orc
    for L in (16, 32, 49, 64):
        ref = orc.t5_relative_position_bucket(torch.arange(L)[None, :] - torch.arange(L)[:, None]).numpy()
        np.testing.assert_array_equal(pkg.layout.t5_bucket_map(L, L), ref)


def test_bn_fold(pkg):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 4, 6, 6, generator=g)
    w = torch.randn(5, 4, 3, 3, generator=g)
    bw, bb, rm, rv = torch.rand(5, generator=g) + .5, torch.randn(5, generator=g), torch.randn(5, generator=g), \
        torch.rand(5, generator=g) + .5
    ref = F.batch_norm(F.conv2d(x, w, padding=1), rm, rv, bw, bb, training=False, eps=1e-5)
    wf, bf = pkg.layout.fold_bn(w.numpy(), bw.numpy(), bb.numpy(), rm.numpy(), rv.numpy())
    got = F.conv2d(x, torch.as_tensor(wf), torch.as_tensor(bf), padding=1)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_stem_space_to_depth_equals_7x7_stride2(pkg):
    """engine.stem_s2d_weight + the vqa_image_to_s2d16 layout (restated here in torch):
    the 4x4 stride-1 pad-1 conv over the space-to-depth image is the torchvision stem
    conv (7x7, stride 2, pad 3, resnet_vqa_model.py:51-58 via torchvision) exactly."""
    import torch
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(0)
    for hw in (16, 30):
        img = torch.rand(2, 3, hw, hw, generator=g, dtype=torch.float64)
        w = torch.randn(8, 3, 7, 7, generator=g, dtype=torch.float64)
        hz = hw // 2 + 1
        xp = F.pad(img, (1, 1, 1, 1))
        z = torch.zeros(2, 16, hz, hz, dtype=torch.float64)
        for p in range(2):
            for q in range(2):
                z[:, (2 * p + q) * 3:(2 * p + q) * 3 + 3] = xp[:, :, p:p + 2 * hz:2, q:q + 2 * hz:2]
        w2 = torch.from_numpy(pkg.engine.stem_s2d_weight(w.permute(0, 2, 3, 1).float().numpy())).double()
        y = F.conv2d(z, w2.permute(0, 3, 1, 2), padding=1)
        ref = F.conv2d(img, w.float().double(), stride=2, padding=3)
        torch.testing.assert_close(y, ref, rtol=1e-12, atol=1e-12)
