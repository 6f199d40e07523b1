"""ctypes binding of libvqa_hip.so (include/vqa_hip.h).

The HIP library is the product path: there is no CPU or PyTorch fallback.  If
the shared object is missing, or does not export every symbol the header
declares, `load()` raises.  torch is imported first so that the library binds
to the HIP runtime torch already loaded (same SONAME libamdhip64.so.7), which
lets us pass torch's stream handles and device pointers straight through.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must be loaded before the HIP library)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libvqa_hip.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "vqa_hip.h")

c_void_p, c_int, c_float, c_ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_longlong


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("n", "h", "w", "c", "oh", "ow", "kh", "kw", "stride", "pad")]


class Dropout(ctypes.Structure):
    """vqa_dropout: p (0 = off), site id, device uint32[2] {seed, counter}."""
    _fields_ = [("p", c_float), ("site", ctypes.c_uint), ("rng", c_void_p)]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("a", c_void_p), ("lda", c_ll), ("a_trans", c_int),
        ("b", c_void_p), ("ldb", c_ll), ("b_trans", c_int),
        ("m", c_int), ("n", c_int), ("k", c_int),
        ("c32", c_void_p), ("ldc32", c_ll),
        ("c16", c_void_p), ("ldc16", c_ll),
        ("bias", c_void_p),
        ("res32", c_void_p), ("res16", c_void_p), ("ldres", c_ll),
        ("mask16", c_void_p), ("ldmask", c_ll),
        ("alpha", c_float), ("beta", c_float), ("relu", c_int),
        ("a_conv", c_int), ("ga", ConvGeom),
        ("b_conv", c_int), ("gb", ConvGeom),
        ("batch", c_int), ("stride_a", c_ll), ("stride_b", c_ll), ("stride_c32", c_ll),
        ("stride_c16", c_ll), ("stride_res", c_ll), ("config", c_int),
        ("drop", Dropout),
        ("splitk", c_int), ("workspace", c_void_p), ("workspace_bytes", c_ll),
        ("stride_bias", c_ll), ("drop_site_stride", c_int),
        ("fp8", c_int), ("scale_a", c_void_p), ("scale_b", c_void_p),
        ("stride_scale_a", c_ll), ("stride_scale_b", c_ll),
    ]


class ImageDesc(ctypes.Structure):
    """vqa_image_desc: byte offset of an image in the packed uint8 buffer, its height, width."""
    _fields_ = [("offset", c_ll), ("h", c_int), ("w", c_int)]


class ColsumJob(ctypes.Structure):
    _fields_ = [("ws", c_void_p), ("out", c_void_p), ("stride", c_ll), ("parts", c_int), ("cols", c_int),
                ("beta", c_float), ("first_block", c_int)]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("q", c_void_p), ("ldq", c_ll), ("k", c_void_p), ("ldk", c_ll), ("v", c_void_p), ("ldv", c_ll),
        ("o", c_void_p), ("ldo", c_ll), ("p", c_void_p), ("bias", c_void_p), ("key_mask", c_void_p),
        ("batch", c_int), ("heads", c_int), ("lq", c_int), ("lk", c_int), ("dh", c_int), ("scale", c_float),
        ("dout", c_void_p), ("lddo", c_ll), ("dq", c_void_p), ("lddq", c_ll), ("dk", c_void_p), ("lddk", c_ll),
        ("dv", c_void_p), ("lddv", c_ll), ("dbias", c_void_p),
        ("drop", Dropout),
        ("groups", c_int), ("gstride_qkv", c_ll), ("gstride_o", c_ll), ("gstride_p", c_ll), ("gstride_dout", c_ll),
        ("gdrop_site_stride", c_int),
    ]


# vqa_gemm tile configs (gemm.hip dispatch_tile): config -> (BM, BN, LDS stages)
# config -> (BM, BN, stages); 1-8 run 4 waves (2x2), 9-12 run 8 waves (include/vqa_hip.h)
GEMM_TILES = {1: (128, 128, 3), 2: (128, 64, 4), 3: (64, 64, 4), 4: (64, 64, 2), 5: (64, 64, 3), 6: (128, 64, 2),
              7: (64, 128, 2), 8: (128, 128, 2), 9: (256, 128, 2), 10: (128, 256, 2), 11: (256, 256, 2),
              12: (256, 128, 3), 13: (64, 192, 2), 14: (128, 192, 2), 15: (64, 192, 3), 16: (128, 192, 3),
              17: (128, 64, 2), 18: (128, 128, 2), 19: (64, 64, 2), 20: (64, 128, 2),
              21: (64, 64, 2), 22: (64, 128, 2), 23: (128, 64, 2), 24: (64, 128, 2), 25: (128, 128, 3),
              26: (64, 128, 1), 27: (128, 64, 1), 28: (64, 64, 1)}
GEMM_PATCH_ONLY = (17, 18, 19, 20, 25)   # the LDS-patch 3x3 convolution (a_conv = 2) and nothing else
GEMM_KC_B_ONLY = (13, 14, 15, 16)        # tile configs that need a k-contiguous B operand (b_trans = 0)
GEMM_BK128 = (21, 22, 23, 24)            # 128-deep k-tiles: no implicit im2col operand, no split-K
GEMM_K64_ONLY = (26, 27, 28)             # one k-tile in a single-stage ring: k <= 64, no implicit im2col, no split-K
GEMM_FP8 = (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 21, 22, 23)   # tile configs with an e4m3 form (gemm_fp8.hip)
GEMM_WAVES = {c: ((4, 2) if c in (9, 12, 25) else (2, 4) if c in (10, 11, 24) else (2, 2)) for c in GEMM_TILES}

ATTN_MFMA, ATTN_LONG, ATTN_VALU = 0, 1, 2          # vqa_attn_path
MAX_GROUPS = 8
ST_STEP, ST_GRAD_NORM, ST_CLIP_COEF, ST_LR_SCALE, ST_BC1, ST_BC2_SQRT = range(6)
ST_PENDING, ST_FLOATS = 8, 16


class AdamWDesc(ctypes.Structure):
    _fields_ = [
        ("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
        ("max_exp_avg_sq", c_void_p), ("param16", c_void_p), ("n", c_ll), ("ngroups", c_int),
        ("group_end", c_ll * MAX_GROUPS), ("group_lr", c_float * MAX_GROUPS),
        ("beta1", c_float), ("beta2", c_float), ("eps", c_float), ("weight_decay", c_float),
        ("grad_scale", c_float), ("state", c_void_p),
    ]


_lib = None


def header_symbols():
    """Every `int vqa_*(` / `long long vqa_*(` / `const char* vqa_*(` export declared in include/vqa_hip.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|long long|const char\*)\s+(vqa_\w+)\s*\(", txt, re.M)))


def abi_version():
    return int(re.search(r"#define VQA_ABI_VERSION (\d+)", open(HEADER).read()).group(1))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libvqa_hip.so not built at {LIB_PATH}: run `python __graft_entry__.py` "
                           "(make -C t5-resnet-vqa_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    if missing:
        raise RuntimeError(f"libvqa_hip.so lacks exported symbols {missing}")
    lib.vqa_last_error.restype = ctypes.c_char_p
    if lib.vqa_abi_version() != abi_version():
        raise RuntimeError(f"libvqa_hip.so ABI {lib.vqa_abi_version()} != header ABI {abi_version()}: rebuild it")
    lib.vqa_gemm.argtypes = [ctypes.POINTER(GemmDesc), c_void_p]
    lib.vqa_gemm_select.argtypes = [ctypes.POINTER(GemmDesc)]
    lib.vqa_gemm_workspace_bytes.argtypes = [ctypes.POINTER(GemmDesc)]
    lib.vqa_gemm_workspace_bytes.restype = c_ll
    lib.vqa_gemm_pair.argtypes = [ctypes.POINTER(GemmDesc), ctypes.POINTER(GemmDesc), c_void_p]
    lib.vqa_attn_fwd.argtypes = [ctypes.POINTER(AttnDesc), c_void_p]
    lib.vqa_attn_bwd.argtypes = [ctypes.POINTER(AttnDesc), c_void_p]
    lib.vqa_attn_path.argtypes = [ctypes.POINTER(AttnDesc), c_int]
    lib.vqa_attn_probs.argtypes = [ctypes.POINTER(AttnDesc), c_void_p]
    lib.vqa_adamw_amsgrad.argtypes = [ctypes.POINTER(AdamWDesc), c_void_p]
    lib.vqa_adamw_rows.argtypes = [ctypes.POINTER(AdamWDesc), c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]
    for name in ("vqa_norm_bwd_workspace_floats", "vqa_colsum_workspace_floats"):
        getattr(lib, name).argtypes = [c_int, c_int]
    lib.vqa_head_workspace_floats.argtypes = [c_int] * 4
    lib.vqa_norm_bwd_parts.argtypes = [c_int]
    lib.vqa_colsum_parts.argtypes = [c_int]
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int
    _lib = lib
    return lib


_SIGS: dict = {}          # filled by register() below for the plain-argument kernels


def register(name, *argtypes):
    _SIGS[name] = list(argtypes) + [c_void_p]      # every export ends with the stream


P = c_void_p
register("vqa_rmsnorm_fwd", P, P, P, P, P, c_int, c_int, c_float, P)
register("vqa_rmsnorm_bwd", P, P, P, P, P, P, P, P, c_float, P, c_int, c_int, P, P, P)
register("vqa_layernorm_fwd", P, P, P, P, P, P, P, c_int, c_int, c_float)
register("vqa_layernorm_bwd", P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, P, P)
register("vqa_rng_advance", P)
register("vqa_dropout_mask", P, P, c_ll)
register("vqa_colsum_partials", P, c_int, c_ll, c_int, P, c_float)
register("vqa_image_to_nhwc8", P, P, c_int, c_int, c_int)
register("vqa_image_to_s2d16", P, P, c_int, c_int, c_int)
register("vqa_resize_linear_u8", P, P, c_int, c_int, c_int, P)
register("vqa_maxpool3x3s2_nhwc", P, P, c_int, c_int, c_int, c_int, c_int, c_int)
register("vqa_subsample_nhwc", P, c_int, c_int, c_int, c_int, c_int, P, c_ll)
register("vqa_stem_s2d_conv", P, P, P, P, c_int, c_int, c_int)
register("vqa_stem_pool_s2d", P, P, P, P, c_int, c_int, c_int)
register("vqa_stem_pool_img", P, P, P, P, c_int, c_int)
register("vqa_colsum", P, c_int, c_int, c_int, c_ll, P, c_float, P)
register("vqa_embedding_fwd", P, P, P, c_int, c_int, c_int, P)
register("vqa_embedding_bwd", P, P, P, c_int, c_int, c_int, P)
register("vqa_embedding_zero_rows", P, P, c_int, P, c_int, c_int)
register("vqa_colsum_batched", P, c_int, c_int)
register("vqa_t5_relbias_fwd", P, P, P, c_int, c_int, c_int)
register("vqa_t5_relbias_bwd", P, P, P, c_int, c_int, c_int, c_int)
register("vqa_batch_sum", P, c_int, c_ll, P, c_float)
register("vqa_cast_f32_bf16", P, P, c_ll)
register("vqa_zero", P, c_ll)
register("vqa_copy", P, P, c_ll)
register("vqa_tap_shift", P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int)
register("vqa_quant_rows_fp8", P, c_int, c_ll, c_int, c_int, P, c_ll, P)
register("vqa_head_fwd", P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int)
register("vqa_head_bwd", P, P, P, P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, c_float)
register("vqa_count_targets", P, c_int, P)
register("vqa_embed_mark", P, c_int, c_int, P, P)
register("vqa_grad_sqnorm", P, c_ll, P, c_int)
register("vqa_vit_patchify", P, P, c_int, c_int, c_int, c_int)
register("vqa_gather_rows", P, c_ll, P, c_ll, c_ll, P, c_ll, c_int, c_int, c_int)
register("vqa_scatter_rows", P, c_ll, P, c_ll, c_ll, P, c_ll, c_int, c_int, c_int)
register("vqa_last_index", P, c_int, c_int, P)
register("vqa_xattn1_fwd", P, c_ll, P, c_ll, c_int, c_int, c_int, c_int, P)
register("vqa_xattn1_bwd", P, c_ll, P, P, c_ll, c_int, c_int, c_int, c_int, P)
register("vqa_optim_finalize", P, c_int, c_float, c_float, c_int, c_int, c_float, c_float, P)


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.vqa_last_error().decode()}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def hip_runtime():
    """The HIP runtime library this process already runs (torch's copy), for the few runtime
    entry points torch does not wrap (hipExtStreamCreateWithCUMask)."""
    import torch
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
    if not paths:
        raise RuntimeError("libamdhip64.so is not mapped in this process")
    return ctypes.CDLL(sorted(paths)[0])


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def call(name, *args, stream=None):
    lib = load()
    rc = getattr(lib, name)(*args, stream_handle(stream))
    check(rc, name)
