"""3x3 stride-1 backbone convs on the split MFMA kernel (dd_conv3x3_forward).

Used by `resnet.ResNet.run(..., fast=True)` for every Conv2d with kernel 3, stride 1, pad 1
whose spatial shape the kernel supports (W in {8, 16, 32}); other convs stay on MIOpen.
`Conv3x3Fn` is an autograd Function whose backward is the same kernel on the transposed,
flipped weight pack (backward-data only: the scoring passes never need weight gradients).
"""
from __future__ import annotations

import torch

from . import _capi

ROWS = {32: 4, 16: 8, 8: 8}  # row block of the kernel per width (4x4: whole images)


def supported(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    if conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1):
        return False
    if conv.groups != 1 or conv.dilation != (1, 1) or x.dim() != 4:
        return False
    h, w = x.shape[2], x.shape[3]
    if not x.is_cuda:
        return False
    return (w in ROWS and h % ROWS[w] == 0) or (h == 4 and w == 4)


# Operand halves (include/dd_capi.h DD_OPERANDS_*): every forward pack takes fp16 halves by
# default, ~2^-22 relative per product instead of bf16's ~2^-17 at the same MFMA rate -- the
# raw weights' packs (the EL2N forward, batch-normalised activations; ScoreConfig.el2n_operands)
# and the BN-folded ones (the GraNd forward; ScoreConfig.grand_operands, whose eval-BN
# activations are not bounded by batch statistics: ScoringEngine.run falls back to bf16 halves
# if one leaves fp16's range).  Only the backward-data packs stay bf16 (gradients span many
# octaves below fp16's normal range).


class Packs:
    """Forward and backward-data packs of one 3x3 weight (computed once per checkpoint)."""

    def __init__(self, weight: torch.Tensor, fwd_operands: str = "bf16x3"):
        w = weight.detach().float().contiguous()
        self.cout, self.cin = w.shape[0], w.shape[1]
        self.fwd = _capi.conv3x3_pack(w, operands=fwd_operands)
        self.bwd = _capi.conv3x3_pack(w, transpose_flip=True)


class DownPacks:
    """Packs of a downsampling head: the stride-2 3x3 conv and its 1x1 stride-2 projection
    (forward: dd_down_forward; backward-data: dd_down_backward)."""

    def __init__(self, w3: torch.Tensor, w1: torch.Tensor, fwd_operands: str = "bf16x3"):
        w3 = w3.detach().float().contiguous()
        w1 = w1.detach().float().contiguous()
        self.cout, self.cin = w3.shape[0], w3.shape[1]
        self.fwd3 = _capi.conv3x3_pack(w3, operands=fwd_operands)
        self.fwd1 = _capi.conv1x1_pack(w1, operands=fwd_operands)
        self.bwd3 = _capi.conv3x3_pack(w3, transpose_flip=True)
        self.bwd1 = _capi.conv1x1_pack(w1, transpose=True)


class Packs1x1:
    """Forward and backward-data packs of one 1x1 weight [cout, cin(, 1, 1)] for
    dd_conv1x1_forward (the Bottleneck convs and projection shortcuts)."""

    def __init__(self, weight: torch.Tensor, fwd_operands: str = "bf16x3"):
        w = weight.detach().float().reshape(weight.shape[0], weight.shape[1]).contiguous()
        self.cout, self.cin = w.shape
        self.fwd = _capi.conv1x1_pack(w, operands=fwd_operands)
        self.bwd = _capi.conv1x1_pack(w, transpose=True)


class Down3Packs:
    """A stride-2 3x3 conv without a fused shortcut (ResNet-50 Bottleneck conv2 at stride 2,
    reference models/resnet.py:42): dd_down_forward / dd_down_backward with no 1x1 part."""

    def __init__(self, w3: torch.Tensor, fwd_operands: str = "bf16x3"):
        w3 = w3.detach().float().contiguous()
        self.cout, self.cin = w3.shape[0], w3.shape[1]
        self.fwd3 = _capi.conv3x3_pack(w3, operands=fwd_operands)
        self.bwd3 = _capi.conv3x3_pack(w3, transpose_flip=True)


def supported1x1(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    """A 1x1 conv dd_conv1x1_forward runs (stride 1, or 2 over an even map)."""
    if conv.kernel_size != (1, 1) or conv.padding != (0, 0) or conv.groups != 1:
        return False
    s = conv.stride[0]
    if conv.stride[1] != s or s not in (1, 2) or not x.is_cuda or x.dim() != 4:
        return False
    return s == 1 or (x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)


class Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, packs: Packs, bias):
        ctx.packs = packs
        return _capi.conv3x3(x.contiguous(), packs.fwd, packs.cout, bias=bias)

    @staticmethod
    def backward(ctx, gy):
        p = ctx.packs
        gx = _capi.conv3x3(gy.contiguous(), p.bwd, p.cin)
        return gx, None, None


def conv3x3(x: torch.Tensor, packs: Packs, bias=None) -> torch.Tensor:
    if torch.is_grad_enabled() and x.requires_grad:
        return Conv3x3Fn.apply(x, packs, bias)
    return _capi.conv3x3(x.contiguous(), packs.fwd, packs.cout, bias=bias)
