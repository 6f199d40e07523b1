"""Train-mode dropout: the oracle's restatement of the counter-hash masks
(include/vqa_hip.h "dropout") and its use in the oracle step (CPU only; the
device side is checked bit for bit against this in test_kernels_gpu.py)."""
import numpy as np
import torch

from oracle import vqa_oracle as orc


def test_mix32_known_answers():
    # values of the device function (common.h vqa_mix32) compiled with gcc, uint32 arithmetic
    assert orc._mix32(0) == 0
    assert orc._mix32(1) == 0x688990C0
    assert orc._mix32(0xDEADBEEF) == 0xE628C683
    assert orc._mix32((orc._mix32(7) + 0x9E3779B9) & 0xFFFFFFFF) == 0xCED1D009
    xs = np.arange(1 << 16, dtype=np.uint64)
    hs = orc._mix32(xs)
    assert len(np.unique(hs)) == len(xs)                       # a bijection: no collisions


def test_mask_law_and_independence():
    n = 1 << 20
    m = orc.dropout_multiplier(0.1, 0, 1, 16, n)
    keep = (m > 0).mean()
    assert abs(keep - 0.9) < 2e-3
    scale = np.float32(1) / (np.float32(1) - np.float32(0.1))
    assert set(np.unique(m).tolist()) == {0.0, float(scale)}
    # different site / counter / seed -> independent masks
    for other in (orc.dropout_multiplier(0.1, 0, 1, 17, n), orc.dropout_multiplier(0.1, 0, 2, 16, n),
                  orc.dropout_multiplier(0.1, 1, 1, 16, n)):
        both = ((m > 0) & (other > 0)).mean()
        assert abs(both - 0.81) < 3e-3
    # deterministic
    np.testing.assert_array_equal(m, orc.dropout_multiplier(0.1, 0, 1, 16, n))
    # no run structure along the row: neighbouring elements are uncorrelated
    a, b = (m[:-1] > 0).astype(np.float64), (m[1:] > 0).astype(np.float64)
    assert abs(np.corrcoef(a, b)[0, 1]) < 5e-3


def test_engine_and_oracle_share_site_numbering(pkg):
    E = pkg.engine
    assert (E.SITE_EMBED, E.SITE_FINAL) == (orc.SITE_EMBED, orc.SITE_FINAL)
    sites = {E.SITE_EMBED, E.SITE_FINAL}
    for i in range(12):
        for kind in range(4):
            assert E.t5_site(i, kind) == orc.t5_site(i, kind)
            sites.add(E.t5_site(i, kind))
    for n in range(3):
        for kind in range(6):
            assert E.sga_site(n, kind) == orc.sga_site(n, kind)
            sites.add(E.sga_site(n, kind))
    assert len(sites) == 2 + 48 + 18                              # every dropout application has its own key


def test_oracle_train_mode_step_uses_dropout(pkg):
    """Same batch, lr 0 (first scheduler step): eval mode repeats exactly, train mode draws new masks."""
    sd = pkg.synthetic.make_state_dict("resnet34", seed=0)
    nb = orc.to_torch_batch(pkg.synthetic.make_batch(2, 8, 64, seed=1))
    tr = orc.OracleTrainer(sd, "resnet34", warmup=5, total=10, dropout=0.1, seed=4)
    l1 = tr.forward_backward(nb)[0]
    tr2 = orc.OracleTrainer(sd, "resnet34", warmup=5, total=10, dropout=0.1, seed=4)
    l2 = tr2.forward_backward(nb)[0]
    torch.testing.assert_close(l1, l2, rtol=0, atol=0)               # same seed+counter: identical
    l3 = tr2.forward_backward(nb)[0]                                 # counter 2: new masks
    assert not torch.equal(l2, l3)
    e0 = orc.OracleTrainer(sd, "resnet34", warmup=5, total=10, dropout=0.0)
    assert not torch.equal(e0.forward_backward(nb)[0], l1)


def test_torch_hash_equals_uint32_hash():
    """dropout_multiplier (int64 torch arithmetic, masked to 32 bits) == the numpy uint64 form,
    element for element, across keys and sizes (incl. indices past 2^31)."""
    for p, seed, counter, site, n in ((0.1, 0, 1, 16, 1 << 18), (0.5, 7, 123456, 5, 77777), (0.1, 3, 9, 131, 4099)):
        np.testing.assert_array_equal(orc.dropout_multiplier(p, seed, counter, site, n),
                                      orc.dropout_multiplier_np(p, seed, counter, site, n))
    # the top of the index range: e * 0x9E3779B9 overflows int64 and must wrap like uint32 math
    e = np.array([2**31 - 1, 2**31, 2**32 - 2], dtype=np.uint64)
    key = orc.dropout_key(1, 2, 3)
    ref = orc._mix32(((e * np.uint64(0x9E3779B9)) + np.uint64(key)) & np.uint64(0xFFFFFFFF))
    x = ((torch.tensor(e.astype(np.int64)) * 0x9E3779B9) + key) & 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    assert (x ^ (x >> 16)).numpy().astype(np.uint64).tolist() == ref.tolist()
