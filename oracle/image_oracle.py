"""CPU restatement of the reference collate's image path -- TEST INFRASTRUCTURE
ONLY (tests/ and the checkers may import it; the product path never does).

dataset_utils/resnet_vqa_daquar_dataset.py:145-163 runs, per image,
    cv2.imread -> cv2.cvtColor(BGR2RGB) -> cv2.resize((W, H), INTER_LINEAR) -> ToTensor()
opencv-python is not a dependency the reference pins (requirements.txt has no
cv2 line; the collate imports it) and it is not importable here, so this file
restates OpenCV's published algorithm for an 8-bit INTER_LINEAR resize (OpenCV
4.x imgproc/src/resize.cpp, generic fixed-point path: INTER_RESIZE_COEF_BITS =
11, HResizeLinear + VResizeLinear<uchar, int, short, FixedPtCast<int, uchar,
22>> whose uchar form is ((b0*(S0>>4))>>16) + ((b1*(S1>>4))>>16) + 2) >> 2) and
torchvision's ToTensor (functional.to_tensor: float(x) / 255, CHW).
Parity unpinned against cv2 itself (no cv2 outputs exist in the reference or
here); an IPP-accelerated OpenCV build may differ by one level at a few pixels.
"""
import numpy as np

COEF_SCALE = 2048          # 1 << INTER_RESIZE_COEF_BITS


def _weights(dst, src, clamp):
    """Per destination index: (i0, i1, w0, w1, one) in OpenCV's float32 / rounding."""
    scale = 1.0 / (float(dst) / float(src))                       # cv::resize: 1 / inv_scale
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    i = np.floor(f).astype(np.int64)
    f = (f - i.astype(np.float32)).astype(np.float32)
    one = np.zeros(dst, bool)
    if clamp:                                                      # horizontal: fx = 0 at the borders
        lo, hi = i < 0, i >= src - 1
        i = np.where(lo, 0, np.where(hi, src - 1, i))
        f = np.where(lo | hi, np.float32(0), f).astype(np.float32)
        one = lo | hi
        i1 = np.where(one, i, i + 1)
    else:                                                          # vertical: rows clipped, weights kept
        i1 = np.clip(i + 1, 0, src - 1)
        i = np.clip(i, 0, src - 1)
    w0 = np.rint((np.float32(1) - f) * np.float32(COEF_SCALE)).astype(np.int64)
    w1 = np.rint(f * np.float32(COEF_SCALE)).astype(np.int64)
    return i, i1, w0, w1, one


def resize_linear_u8(img, oh, ow):
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_LINEAR) for uint8 HWC."""
    img = np.asarray(img, np.uint8)
    h, w = img.shape[:2]
    x0, x1, a0, a1, one = _weights(ow, w, True)
    y0, y1, b0, b1, _ = _weights(oh, h, False)
    s = img.astype(np.int64)
    rows = np.unique(np.concatenate([y0, y1]))
    t = np.zeros((h, ow) + img.shape[2:], np.int64)
    a0e = a0.reshape((1, ow) + (1,) * (img.ndim - 2))
    a1e = a1.reshape((1, ow) + (1,) * (img.ndim - 2))
    onee = one.reshape((1, ow) + (1,) * (img.ndim - 2))
    t[rows] = np.where(onee, s[rows][:, x0] * COEF_SCALE, s[rows][:, x0] * a0e + s[rows][:, x1] * a1e)
    b0e = b0.reshape((oh, 1) + (1,) * (img.ndim - 2))
    b1e = b1.reshape((oh, 1) + (1,) * (img.ndim - 2))
    v = (((b0e * (t[y0] >> 4)) >> 16) + ((b1e * (t[y1] >> 4)) >> 16) + 2) >> 2
    return v.astype(np.uint8)


def to_tensor(img):
    """torchvision ToTensor: HWC uint8 -> CHW float32 / 255."""
    return (np.asarray(img).transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)).astype(np.float32)


def collate_images(images, oh, ow):
    """The collate's image_tensors: stack of ToTensor(resize(img)) -> [B, 3, oh, ow] float32."""
    return np.stack([to_tensor(resize_linear_u8(im, oh, ow)) for im in images])
