"""Thin Python constructors for the C-ABI calls.

Descriptors are built once (the engine's buffers have fixed addresses) and the
prepared call is replayed every step, so the per-step host cost is one ctypes
call per kernel (and zero under hipGraph replay).
"""
from __future__ import annotations

import ctypes

import torch

from . import lib as L


def addr(x, offset_elems=0):
    """Device address of a tensor (+ element offset), a raw int address, or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr() + offset_elems * x.element_size()


def conv_geom(n, h, w, c, oh, ow, kh, kw, stride, pad):
    return L.ConvGeom(n, h, w, c, oh, ow, kh, kw, stride, pad)


def gemm_desc(a, b, m, n, k, *, lda, ldb, a_trans=False, b_trans=False, c32=None, ldc32=0, c16=None, ldc16=0,
              bias=None, res32=None, res16=None, ldres=0, mask16=None, ldmask=0, alpha=1.0, beta=0.0,
              relu=False, ga=None, gb=None, batch=1, stride_a=0, stride_b=0, stride_c32=0, stride_c16=0,
              stride_res=0, splitk=0, workspace=None, stride_bias=0, drop_site_stride=0, a_patch=False,
              fp8=False, scale_a=None, scale_b=None, stride_scale_a=0, stride_scale_b=0):
    """fp8: a / b are e4m3 byte tensors (lda, ldb, k, strides in bytes = elements) with fp32 row
    scales scale_a [m] / scale_b [n] (vqa_gemm_desc.fp8)."""
    op_t = torch.uint8 if fp8 else torch.bfloat16
    for t in (a, b):
        assert not isinstance(t, torch.Tensor) or t.dtype == op_t, f"{op_t} operand expected"
    for t in (c16, res16, mask16):
        assert not isinstance(t, torch.Tensor) or t.dtype == torch.bfloat16, "bf16 operand expected"
    for t in (c32, bias, res32):
        assert not isinstance(t, torch.Tensor) or t.dtype == torch.float32, "fp32 tensor expected"
    d = L.GemmDesc()
    d.a, d.lda, d.a_trans = addr(a), lda, int(a_trans)
    d.b, d.ldb, d.b_trans = addr(b), ldb, int(b_trans)
    d.m, d.n, d.k = m, n, k
    d.c32, d.ldc32 = addr(c32), ldc32
    d.c16, d.ldc16 = addr(c16), ldc16
    d.bias = addr(bias)
    d.res32 = addr(res32)
    d.res16 = addr(res16)
    d.ldres = ldres
    d.mask16 = addr(mask16)
    d.ldmask = ldmask
    d.alpha, d.beta, d.relu = alpha, beta, int(relu)
    d.a_conv = (2 if a_patch else 1) if ga is not None else 0
    if ga is not None:
        d.ga = ga
    d.b_conv = int(gb is not None)
    if gb is not None:
        d.gb = gb
    d.batch, d.stride_a, d.stride_b = batch, stride_a, stride_b
    d.stride_c32, d.stride_c16, d.stride_res = stride_c32, stride_c16, stride_res
    d.stride_bias, d.drop_site_stride = stride_bias, drop_site_stride
    d.fp8, d.scale_a, d.scale_b = int(fp8), addr(scale_a), addr(scale_b)
    d.stride_scale_a, d.stride_scale_b = stride_scale_a, stride_scale_b
    set_splitk(d, splitk, workspace)
    return d


def set_splitk(d, splitk, workspace=None):
    """Split-K of a descriptor: `workspace` (a zero-filled device tensor, see
    vqa_gemm_workspace_bytes) holds the fp32 partials and arrival counters."""
    d.splitk = int(splitk)
    d.workspace = addr(workspace)
    d.workspace_bytes = 0 if workspace is None else workspace.numel() * workspace.element_size()


def splitk_workspace(d, device="cuda"):
    """A zero-filled workspace large enough for descriptor `d` as configured now."""
    n = int(L.load().vqa_gemm_workspace_bytes(ctypes.byref(d)))
    return torch.zeros(max(n, 16) // 4 + 4, dtype=torch.int32, device=device)


class Call:
    """A prepared library call: fixed argument list, replayed on a stream.

    `keep` must reference every tensor whose device address is baked into
    `args`: the call only stores raw addresses, and a tensor freed behind its
    back would hand its memory to the next allocation (use-after-free)."""
    __slots__ = ("fn", "args", "name", "keep", "desc", "side")

    def __init__(self, name, *args, keep=None, desc=None):
        lib = L.load()
        self.name = name
        self.fn = getattr(lib, name)
        self.args = args
        self.keep = keep            # tensors (and structures) that must outlive the call
        self.desc = desc            # ctypes descriptor passed by reference, if any
        self.side = False           # may run on a side stream (off the critical chain), see engine

    def __call__(self, stream_ptr):
        rc = self.fn(*self.args, stream_ptr)
        if rc != 0:
            L.check(rc, self.name)


_PTR_FIELDS = {"GemmDesc": ("a", "b", "c32", "c16", "bias", "res32", "res16", "mask16", "workspace", "scale_a",
                            "scale_b"),
               "AttnDesc": ("q", "k", "v", "o", "p", "bias", "key_mask", "dout", "dq", "dk", "dv", "dbias"),
               "AdamWDesc": ("param", "grad", "exp_avg", "exp_avg_sq", "max_exp_avg_sq", "param16", "state")}


def _pointers(call):
    """(where, address) of every device / host address a prepared call passes: plain
    integer arguments that can only be addresses, and the pointer fields of the descriptors
    it passes by reference (with their dropout RNG pointers)."""
    out = []
    for i, a in enumerate(call.args):
        if isinstance(a, int) and a >= 1 << 36:
            out.append((f"arg{i}", a))
        obj = getattr(a, "_obj", None)                      # ctypes.byref(desc)
        if obj is not None:
            for f in _PTR_FIELDS.get(type(obj).__name__, ()):
                v = getattr(obj, f)
                if v:
                    out.append((f"arg{i}.{f}", v))
            drop = getattr(obj, "drop", None)
            if drop is not None and drop.rng:
                out.append((f"arg{i}.drop.rng", drop.rng))
    return out


def uncovered_pointers(call):
    """Addresses baked into `call` that no object in its `keep` owns (Call docstring: a
    tensor freed behind a prepared call's back hands its memory to the next allocation).
    A tensor covers its whole storage; a ctypes structure its own bytes."""
    spans = []

    def add(o):
        if isinstance(o, torch.Tensor):
            st = o.untyped_storage()
            spans.append((st.data_ptr(), st.data_ptr() + st.nbytes()))
        elif isinstance(o, ctypes.Structure):
            spans.append((ctypes.addressof(o), ctypes.addressof(o) + ctypes.sizeof(o)))
        elif isinstance(o, (tuple, list)):
            for x in o:
                add(x)
    add(call.keep or ())
    add(call.desc if call.desc is not None else ())
    return [(w, hex(p)) for w, p in _pointers(call) if not any(a <= p < b for a, b in spans)]


def gemm_call(desc, tensors=()):
    return Call("vqa_gemm", ctypes.byref(desc), keep=tuple(tensors), desc=desc)


def run(call_or_desc, stream=None):
    s = L.stream_handle(stream)
    if isinstance(call_or_desc, L.GemmDesc):
        call_or_desc = gemm_call(call_or_desc)
    call_or_desc(s)


# ------------------------------------------------------------------ conveniences (tests, API mirror)
def linear(x16, w16, bias=None, relu=False, out32=None, out16=None):
    """y = x @ w^T (+bias) ; x [M,K] bf16, w [N,K] bf16."""
    M, K = x16.shape
    N = w16.shape[0]
    if out32 is None and out16 is None:
        out32 = torch.empty(M, N, device=x16.device, dtype=torch.float32)
    d = gemm_desc(x16, w16, M, N, K, lda=K, ldb=K, c32=out32, ldc32=N, c16=out16, ldc16=N, bias=bias, relu=relu)
    run(d)
    return out32 if out32 is not None else out16
