"""The CPU restatement of the collate's image path (oracle/image_oracle.py: OpenCV
INTER_LINEAR for 8-bit images + ToTensor) and the question padding of the GPU collate.
Parity against cv2 itself is unpinned (cv2 is not importable here): these are the
properties the restated algorithm must have."""
import numpy as np
import pytest
import torch

from oracle import image_oracle as io


def rnd(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_same_size_is_a_copy():
    a = rnd(13, 17, 0)
    assert np.array_equal(io.resize_linear_u8(a, 13, 17), a)


def test_constant_image_stays_constant():
    for oh, ow in ((256, 256), (3, 5), (100, 7)):
        assert (io.resize_linear_u8(np.full((37, 41, 3), 201, np.uint8), oh, ow) == 201).all()


def test_exact_half_is_the_2x2_box_average():
    """cv::resize turns an exact 2x INTER_LINEAR downscale into INTER_AREA; the 8-bit
    linear arithmetic gives the same (a + b + c + d + 2) >> 2."""
    a = rnd(64, 48, 1).astype(np.int64)
    ref = (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
    assert np.array_equal(io.resize_linear_u8(a.astype(np.uint8), 32, 24), ref)


@pytest.mark.parametrize("h,w,oh,ow", [(480, 640, 256, 256), (31, 29, 256, 256), (300, 200, 224, 224)])
def test_close_to_float_bilinear(h, w, oh, ow):
    """Within one level of the exact half-pixel bilinear (11-bit weights, 8-bit rounding)."""
    a = rnd(h, w, 2)
    x = torch.tensor(a.transpose(2, 0, 1)[None].astype(np.float32))
    f = torch.nn.functional.interpolate(x, size=(oh, ow), mode="bilinear", align_corners=False)[0]
    got = io.resize_linear_u8(a, oh, ow).astype(np.float32).transpose(2, 0, 1)
    assert np.abs(got - f.numpy()).max() <= 1.0


def test_to_tensor_and_collate_layout():
    imgs = [rnd(20, 30, 3), rnd(50, 10, 4)]
    t = io.collate_images(imgs, 16, 16)
    assert t.shape == (2, 3, 16, 16) and t.dtype == np.float32
    assert t.min() >= 0.0 and t.max() <= 1.0
    assert np.array_equal(t[0] * np.float32(255), np.rint(t[0] * np.float32(255)))   # k / 255 exactly


def test_question_padding(pkg):
    data = pkg.data
    ids, mask = data.pad_question_ids([[32100, 5, 6, 1], list(range(2, 40)) + [1]], max_length=16)
    assert ids.shape == (2, 16) and mask.dtype == np.int64
    assert list(ids[0, :5]) == [32100, 5, 6, 1, 0] and list(mask[0, :5]) == [1, 1, 1, 1, 0]
    assert mask[1].all() and ids[1, -1] == 1 and list(ids[1, :15]) == list(range(2, 17))
