"""Building blocks for the NHWC CNN towers (face / OCR): conv with BatchNorm folded into
the implicit-GEMM epilogue, depthwise conv, pre-conv BN as a channel affine, SE, linear.

Every parameter is stored in the layout its kernel consumes (conv weights
[Cout, KH, KW, Cin_pad] bf16, folded BN as an fp32 bias), so a forward pass is
nothing but kernel launches.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
from torch import nn

from .. import ops
from ..ops import cnn


def _pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def _pad16(c: int) -> int:
    return (c + 15) // 16 * 16


def fold_bn(w: torch.Tensor, b: Optional[torch.Tensor], bn: dict, eps: float = 1e-5):
    """Fold an inference BatchNorm (after the conv) into conv weights [Cout, ...] / bias."""
    g = bn["weight"].float() if bn.get("weight") is not None else torch.ones_like(bn["running_mean"]).float()
    beta = bn["bias"].float() if bn.get("bias") is not None else torch.zeros_like(g)
    scale = g / torch.sqrt(bn["running_var"].float() + eps)
    wf = w.float() * scale.view(-1, *([1] * (w.dim() - 1)))
    bf = (b.float() if b is not None else torch.zeros_like(g)) * scale + beta - bn["running_mean"].float() * scale
    return wf, bf


class ConvBN(nn.Module):
    """conv (+folded BN) -> act -> PReLU -> (+residual), NHWC."""

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, pad: Optional[int] = None, act=None,
                 prelu: bool = False, dilation: int = 1, dtype=torch.bfloat16, post_act=None):
        super().__init__()
        self.cin, self.cout, self.k = cin, cout, k
        self.post_act = post_act
        self.cin_p, self.cout_p = _pad8(cin), _pad16(cout)
        self.stride, self.dilation = stride, dilation
        self.pad = k // 2 * dilation if pad is None else pad
        self.act = act
        self.w = nn.Parameter(torch.zeros(self.cout_p, k, k, self.cin_p, dtype=dtype), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(self.cout_p, dtype=torch.float32), requires_grad=False)
        self.prelu = nn.Parameter(torch.full((self.cout_p,), 0.25, dtype=dtype), requires_grad=False) if prelu else None

    def random_init(self, g: torch.Generator, gain: float = 1.0):
        fan_in = self.cin * self.k * self.k
        w = torch.randn(self.cout, self.k, self.k, self.cin, generator=g) * gain * math.sqrt(2.0 / fan_in)
        self.w.data.zero_()
        self.w.data[: self.cout, :, :, : self.cin] = w.to(self.w.dtype)
        self.b.data.zero_()
        self.b.data[: self.cout] = torch.randn(self.cout, generator=g) * 0.01

    def load_torch(self, w: torch.Tensor, b: Optional[torch.Tensor] = None, bn: Optional[dict] = None,
                   prelu: Optional[torch.Tensor] = None):
        """w: PyTorch [Cout, Cin, KH, KW] (+ BN dict to fold)."""
        if bn is not None:
            w, b = fold_bn(w, b, bn)
        wt = w.float().permute(0, 2, 3, 1)
        self.w.data.zero_()
        self.w.data[: self.cout, :, :, : self.cin] = wt.to(self.w.dtype)
        self.b.data.zero_()
        if b is not None:
            self.b.data[: self.cout] = b.float()
        if prelu is not None and self.prelu is not None:
            self.prelu.data[: self.cout] = prelu.float().flatten().to(self.prelu.dtype)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                out_dtype=None, aff: Optional[tuple] = None, aff_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``aff`` / ``aff_out``: the next layer's channel affine produced by this conv's epilogue
        (ops.cnn.conv2d)."""
        assert x.shape[-1] == self.cin_p, f"ConvBN expects {self.cin_p} input channels, got {x.shape[-1]}"
        return cnn.conv2d(x, self.w, self.b, self.stride, self.pad, self.dilation, act=self.act, residual=residual,
                          prelu=self.prelu, out=out, out_dtype=out_dtype, post_act=self.post_act, aff=aff,
                          aff_out=aff_out)


class DWConvBN(nn.Module):
    def __init__(self, c: int, k: int, stride: int = 1, act=None, dtype=torch.bfloat16):
        super().__init__()
        self.c, self.k, self.stride, self.act = c, k, stride, act
        self.w = nn.Parameter(torch.zeros(k, k, c, dtype=dtype), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(c, dtype=torch.float32), requires_grad=False)

    def random_init(self, g):
        self.w.data.copy_((torch.randn(self.k, self.k, self.c, generator=g) * math.sqrt(2.0 / (self.k * self.k)))
                          .to(self.w.dtype))

    def load_torch(self, w, b=None, bn=None):
        if bn is not None:
            w, b = fold_bn(w, b, bn)
        self.w.data.copy_(w.float().reshape(self.c, self.k, self.k).permute(1, 2, 0).to(self.w.dtype))
        if b is not None:
            self.b.data.copy_(b.float())

    def forward(self, x):
        return cnn.conv2d_dw(x, self.w, self.b, self.stride, self.k // 2, 1, act=self.act)


class ChannelAffine(nn.Module):
    """Inference BatchNorm that cannot be folded (it precedes a zero-padded conv)."""

    def __init__(self, c: int, act=None, prelu: bool = False):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(c), requires_grad=False)
        self.shift = nn.Parameter(torch.zeros(c), requires_grad=False)
        self.act = act
        self.prelu = nn.Parameter(torch.full((c,), 0.25, dtype=torch.bfloat16), requires_grad=False) if prelu else None

    def load_bn(self, bn: dict, eps: float = 1e-5):
        g = bn.get("weight")
        g = g.float() if g is not None else torch.ones_like(bn["running_mean"]).float()
        s = g / torch.sqrt(bn["running_var"].float() + eps)
        beta = bn.get("bias")
        beta = beta.float() if beta is not None else torch.zeros_like(s)
        self.scale.data.copy_(s)
        self.shift.data.copy_(beta - bn["running_mean"].float() * s)

    def random_init(self, g):
        self.scale.data.copy_(1.0 + 0.05 * torch.randn(self.scale.shape, generator=g))
        self.shift.data.copy_(0.05 * torch.randn(self.shift.shape, generator=g))

    def forward(self, x):
        return cnn.channel_affine(x, self.scale, self.shift, act=self.act, prelu=self.prelu)


class Linear(nn.Module):
    def __init__(self, cin: int, cout: int, bias: bool = True, act=None, dtype=torch.bfloat16):
        super().__init__()
        self.cin_p = (cin + 63) // 64 * 64
        self.cout_p = _pad16(cout)
        self.cin, self.cout, self.act = cin, cout, act
        self.w = nn.Parameter(torch.zeros(self.cout_p, self.cin_p, dtype=dtype), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(self.cout_p), requires_grad=False) if bias else None

    def random_init(self, g, std=None):
        std = std or self.cin ** -0.5
        self.w.data.zero_()
        self.w.data[: self.cout, : self.cin] = (torch.randn(self.cout, self.cin, generator=g) * std).to(self.w.dtype)

    def load_torch(self, w, b=None):
        self.w.data.zero_()
        self.w.data[: self.cout, : self.cin] = w.float().to(self.w.dtype)
        if self.b is not None and b is not None:
            self.b.data.zero_()
            self.b.data[: self.cout] = b.float()

    def forward(self, x, out_dtype=None, residual=None):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.shape[1] != self.cin_p:
            x2 = torch.nn.functional.pad(x2, (0, self.cin_p - x2.shape[1]))
        y = ops.linear(x2, self.w, self.b, act=self.act, residual=residual, out_dtype=out_dtype)
        return y[:, : self.cout] if self.cout_p != self.cout else y
