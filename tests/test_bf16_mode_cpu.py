"""The bf16-operand oracle mode (oracle/bf16_mode.py) must round EVERY matmul the oracles
write: r04's mode matched only `Tensor.__matmul__`, which `a @ b` never reaches in this torch
(it arrives as `TensorBase.matmul`), so its "bf16-operand oracle" was the fp32 oracle and the
config-4 parity A/B built on it was wrong (profiles/r05_vit_trained_diag.json)."""
import torch

from oracle.bf16_mode import Bf16Operands, r16


def test_bf16_operand_mode_rounds_every_matmul():
    g = torch.Generator().manual_seed(0)
    a = torch.randn(3, 5, 64, generator=g, requires_grad=True)
    w = torch.randn(48, 64, generator=g, requires_grad=True)
    ref = r16(a) @ r16(w).T
    with Bf16Operands():
        outs = [a @ w.T, torch.matmul(a, w.T), a.matmul(w.T)]
    for o in outs:
        assert torch.equal(o, ref)
    assert not torch.equal(outs[0], a @ w.T)                 # outside the mode: fp32 operands
    dy = torch.randn(3, 5, 48, generator=g)
    with Bf16Operands():
        (a @ w.T).backward(dy)
    torch.testing.assert_close(a.grad, r16(dy) @ r16(w), rtol=0, atol=0)
    torch.testing.assert_close(w.grad, (r16(dy).reshape(-1, 48).T @ r16(a).reshape(-1, 64)), rtol=1e-6, atol=1e-5)
