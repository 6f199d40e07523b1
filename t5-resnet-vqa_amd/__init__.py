"""vqa_amd — MI355X-native (gfx950) training path for the ResNet+T5+SGA VQA model
of shiv-vignesh/T5-Resnet-VQA (`model/resnet_vqa_model.py`,
`model/multi_head_vision_text_attn.py`).

Layout:
  csrc/          hand-written HIP kernels + the extern "C" ABI (libvqa_hip.so)
  lib.py         ctypes binding of that ABI (fails loudly when the .so is absent)
  engine.py      flat parameter/gradient/optimizer arenas, the explicit
                 forward/backward schedule, fused clip+AdamW, hipGraph capture
  layout.py      the flat arena <-> reference state_dict mapping
  ops.py         prepared C-ABI calls (descriptors built once, replayed)
  model.py       mirror of the reference module API (ResnetVQAModel)
  trainer.py     train_one_step / epoch loops of the reference trainer
  dp.py          the data-parallel (RCCL over xGMI) step
  data.py        the collate's image path on the GPU (resize + ToTensor)
  synthetic.py   deterministic weights / batches (no network)
"""
import importlib

from . import synthetic  # noqa: F401  (numpy only)

_LAZY = ("lib", "ops", "engine", "layout", "model", "trainer", "dp", "data", "vit_model", "vit_engine")


def __getattr__(name):
    if name in _LAZY:
        mod = importlib.import_module(f"{__name__}.{name}")
        globals()[name] = mod
        return mod
    raise AttributeError(name)
