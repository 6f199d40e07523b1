"""Input pipeline of the reference collate on the GPU.

`DaquarFasterRcnnT5CollateFn.collect_preprocessed_data`
(dataset_utils/resnet_vqa_daquar_dataset.py:145-231) decodes, converts,
resizes and ToTensor's every image on the host, one at a time, then tokenizes
the questions.  Here:

* decode stays on the host (JPEG entropy decoding is serial): `decode_image`
  returns the RGB uint8 HWC array cv2.imread + cvtColor(BGR2RGB) gives (PIL is
  the decoder available offline);
* `ImageBatcher` packs a batch of variable-size uint8 images into one pinned
  buffer, copies it to HBM in one async transfer (uint8: 4x fewer PCIe bytes
  than the fp32 tensors the reference moves, `:327-329` of the trainer) and one
  `vqa_resize_linear_u8` launch writes the resized ToTensor batch straight into
  the destination (e.g. the engine's static image buffer);
* questions arrive pre-tokenized (the t5-base tokenizer files cannot be fetched
  offline): `DaquarCollate` pads / truncates them exactly as
  `tokenizer(..., padding="max_length", max_length=16, truncation=True)` lays
  out ids and masks, and returns the reference batch dict.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import lib as L


def decode_image(path):
    """cv2.imread(path) + cv2.cvtColor(BGR2RGB): an RGB uint8 [H, W, 3] array."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


class ImageBatcher:
    """Resize + ToTensor of a batch of uint8 RGB images on the GPU (cv2 INTER_LINEAR numerics).

    Buffers grow on demand and are reused; `__call__` is asynchronous on the current
    stream (the pinned staging buffer is not rewritten before the previous copy ended)."""

    def __init__(self, out_h=256, out_w=256, device="cuda"):
        self.oh, self.ow = int(out_h), int(out_w)
        self.dev = torch.device(device)
        self._host = self._dev_src = None
        self._hdesc = self._ddesc = None
        self._done = None
        L.load()

    def _ensure(self, nbytes, batch):
        if self._host is None or self._host.numel() < nbytes:
            cap = max(nbytes, 1 << 20)
            self._host = torch.empty(cap, dtype=torch.uint8).pin_memory()
            self._dev_src = torch.empty(cap, dtype=torch.uint8, device=self.dev)
        if self._hdesc is None or self._hdesc.numel() < batch * 16:
            self._hdesc = torch.empty(batch * 16, dtype=torch.uint8).pin_memory()
            self._ddesc = torch.empty(batch * 16, dtype=torch.uint8, device=self.dev)

    def __call__(self, images, out=None):
        """images: list of [H_i, W_i, 3] uint8 arrays; out: optional [B, 3, oh, ow] fp32 CUDA
        tensor to write (else a new one).  Returns the batch tensor."""
        B = len(images)
        if B == 0:
            raise ValueError("empty image batch")
        arrs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        for a in arrs:
            if a.ndim != 3 or a.shape[2] != 3 or a.shape[0] < 1 or a.shape[1] < 1:
                raise ValueError(f"expected [H, W, 3] uint8 images, got {a.shape}")
        sizes = [a.nbytes for a in arrs]
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        total = int(sum(sizes))
        if self._done is not None:
            self._done.synchronize()                      # the last copy out of the staging buffer ended
        self._ensure(total, B)
        host = self._host.numpy()
        for a, o in zip(arrs, offs):
            host[o:o + a.nbytes] = a.reshape(-1)
        desc = (L.ImageDesc * B)(*[L.ImageDesc(int(o), a.shape[0], a.shape[1]) for a, o in zip(arrs, offs)])
        ctypes.memmove(self._hdesc.data_ptr(), ctypes.addressof(desc), ctypes.sizeof(desc))
        self._dev_src[:total].copy_(self._host[:total], non_blocking=True)
        self._ddesc[:B * 16].copy_(self._hdesc[:B * 16], non_blocking=True)
        if out is None:
            out = torch.empty(B, 3, self.oh, self.ow, dtype=torch.float32, device=self.dev)
        if tuple(out.shape) != (B, 3, self.oh, self.ow) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous [{B}, 3, {self.oh}, {self.ow}] fp32 tensor")
        rc = L.load().vqa_resize_linear_u8(self._dev_src.data_ptr(), self._ddesc.data_ptr(), B, self.oh, self.ow,
                                           out.data_ptr(), L.stream_handle())
        L.check(rc, "vqa_resize_linear_u8")
        self._done = torch.cuda.Event()
        self._done.record()
        return out


def pad_question_ids(token_ids, max_length=16, pad_id=0):
    """tokenizer(..., padding="max_length", max_length, truncation=True) layout of already
    tokenized questions: ids truncated (keeping the final EOS, as T5's tokenizer does) or
    right-padded with pad_id; attention mask 1 on real tokens."""
    B = len(token_ids)
    ids = np.full((B, max_length), pad_id, np.int64)
    mask = np.zeros((B, max_length), np.int64)
    for b, t in enumerate(token_ids):
        t = list(t)
        if len(t) > max_length:
            t = t[:max_length - 1] + [t[-1]]
        ids[b, :len(t)] = t
        mask[b, :len(t)] = 1
    return ids, mask


class DaquarCollate:
    """`DaquarFasterRcnnT5CollateFn` (resnet_vqa_daquar_dataset.py:92-231) with the image
    path on the GPU.  A data point is a dict with `image` (uint8 RGB array) or `image_path`,
    `question_ids` (token ids, ending in EOS), and `annotation_id` (answer index)."""

    # cv2 flags the reference collate accepts as `interpolation_strategy` (:156-164); only
    # INTER_LINEAR (the default, cv2 constant 1) has a GPU kernel here
    INTERPOLATIONS = {"linear": 1, "INTER_LINEAR": 1, 1: 1}

    def __init__(self, resizing_dimensions=(256, 256), max_question_length=16, device="cuda", eval_mode=False,
                 interpolation_strategy="linear", decode_workers=0):
        if interpolation_strategy not in self.INTERPOLATIONS:
            raise NotImplementedError(f"interpolation_strategy {interpolation_strategy!r}: only cv2.INTER_LINEAR is "
                                      "implemented on the GPU (vqa_resize_linear_u8); LANCZOS4 / CUBIC would train "
                                      "on different pixels")
        w, h = resizing_dimensions                      # the reference unpacks (width, height) (:132)
        self.batcher = ImageBatcher(h, w, device)
        self.max_len = int(max_question_length)
        self.eval_mode = eval_mode
        self.dev = torch.device(device)
        # host JPEG decode is serial per image; decode_workers > 0 decodes a batch on a thread
        # pool (PIL releases the GIL while it decodes)
        self._pool = None
        if decode_workers and decode_workers > 0:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=int(decode_workers))

    def _decode(self, data_points):
        get = lambda dp: dp["image"] if "image" in dp else decode_image(dp["image_path"])
        if self._pool is None:
            return [get(dp) for dp in data_points]
        return list(self._pool.map(get, data_points))

    def __call__(self, data_points, out=None):
        images = self._decode(data_points)
        ids, mask = pad_question_ids([dp["question_ids"] for dp in data_points], self.max_len)
        B = len(data_points)
        dec = np.zeros((B, 20), np.int64)                 # decoder_* / answer_* (ignored by the model)
        batch = {
            "question_input_ids": torch.from_numpy(ids).to(self.dev),
            "decoder_question_input_ids": torch.from_numpy(dec).to(self.dev),
            "question_attention_masks": torch.from_numpy(mask).to(self.dev),
            "decoder_question_attention_masks": torch.from_numpy(dec).to(self.dev),
            "annotation_ids": torch.as_tensor([int(dp["annotation_id"]) for dp in data_points],
                                              dtype=torch.int64).to(self.dev),
            "pixel_values": None,
            "image_tensors": self.batcher(images, out=out),
            "question_type_ids": None,
            "answer_input_ids": torch.from_numpy(dec).to(self.dev),
            "answer_attention_masks": torch.from_numpy(dec).to(self.dev),
        }
        if self.eval_mode:
            batch["image_fns"] = [dp.get("image_path") for dp in data_points]
        return batch


def synthetic_images(batch, seed=0, min_side=200, max_side=640):
    """DAQUAR-like variable-size RGB uint8 images (NYU-Depth frames are 640 x 480)."""
    g = np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, 0x1A6E]))
    out = []
    for _ in range(batch):
        h, w = int(g.integers(min_side, max_side + 1)), int(g.integers(min_side, max_side + 1))
        out.append(g.integers(0, 256, (h, w, 3), dtype=np.uint8))
    return out


__all__ = ["decode_image", "ImageBatcher", "pad_question_ids", "DaquarCollate", "synthetic_images"]
