"""ORACLE -- test infrastructure only, never the product path.

bf16-operand arithmetic for the CPU oracles: inside `Bf16Operands()`, every matmul (`@`,
torch.matmul, Tensor.matmul) and the ViT patch convolution run on bf16-rounded operands with
fp32 accumulation, and their backward rounds the output gradient too -- the operands the
engine's MFMA GEMMs see.  The oracle run under this mode against the plain fp32 oracle is what
bf16 arithmetic alone moves (tools/drift_ab_vit.py, tools/vit_trained_diag.py,
tests/test_vit_gpu.py::test_vit_trained_path_is_bf16_operand_arithmetic).
"""
import torch
from torch.overrides import TorchFunctionMode

F = torch.nn.functional


def r16(t):
    return t.bfloat16().float()


class _Bf16MM(torch.autograd.Function):
    """a @ b on bf16-rounded operands, fp32 accumulation; the backward rounds dY too."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return torch.matmul(r16(a), r16(b))

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        # (run under the mode when backward() is called inside it: the operands are rounded
        # already, so the mode's second rounding changes nothing)
        d = r16(dy)
        da = torch.matmul(d, r16(b).transpose(-1, -2)) if ctx.needs_input_grad[0] else None
        db = torch.matmul(r16(a).transpose(-1, -2), d) if ctx.needs_input_grad[1] else None
        if db is not None and db.dim() > b.dim():                  # broadcast weight: sum the batch dims
            db = db.reshape(-1, *b.shape).sum(0)
        if da is not None and da.shape != a.shape:                 # broadcast activation
            da = da.reshape(-1, *a.shape).sum(0)
        return da, db


_MATMULS = (torch.matmul, torch.Tensor.__matmul__, torch.Tensor.matmul, torch._C.TensorBase.matmul)


class Bf16Operands(TorchFunctionMode):
    """Round every matmul's operands to bf16.  `a @ b` reaches a mode as
    `torch._C.TensorBase.matmul` in this torch (2.10), not as `Tensor.__matmul__`: r04's mode
    matched only the latter, so its "bf16-operand oracle" rounded none of the oracle's `@`
    products (only the patch convolution) -- test_bf16_operand_mode_rounds_every_matmul."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in _MATMULS and all(torch.is_tensor(x) for x in args[:2]) \
                and args[0].dim() >= 2 and args[1].dim() >= 2:
            return _Bf16MM.apply(args[0], args[1])
        if func is F.conv2d:                                      # the ViT patch embedding (frozen)
            x, w = args[0], args[1]
            return func(r16(x), r16(w), *args[2:], **kwargs)
        return func(*args, **kwargs)
