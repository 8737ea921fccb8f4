"""CNN ops on NHWC activations (HIP kernels on GPU, PyTorch fp32 reference on CPU).

Layout conventions: activations are NHWC ``[N, H, W, C]`` (C a multiple of 8 on the
GPU path, 16-byte channel vectors); dense conv weights are ``[Cout, KH, KW, Cin]``
(K-contiguous, the implicit-GEMM B operand); depthwise weights are ``[KH, KW, C]``.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from .._native import hip_ops
from . import _act_ref, act_id


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _pads4(padding) -> tuple:
    """int | (ph, pw) | ONNX (top, left, bottom, right) -> (top, left, bottom, right)."""
    if isinstance(padding, (tuple, list)) and len(padding) == 4:
        return tuple(int(v) for v in padding)
    p = _pair(padding)
    return (p[0], p[1], p[0], p[1])


def _pad_arg(padding) -> list:
    q = _pads4(padding)
    return [q[0], q[1]] if (q[0], q[1]) == (q[2], q[3]) else list(q)


def conv_out_hw(H, W, KH, KW, stride, padding, dilation):
    s, d = _pair(stride), _pair(dilation)
    pt, pl, pb, pr = _pads4(padding)
    return ((H + pt + pb - d[0] * (KH - 1) - 1) // s[0] + 1, (W + pl + pr - d[1] * (KW - 1) - 1) // s[1] + 1)


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, stride=1, padding=0, dilation=1,
           act=None, residual: Optional[torch.Tensor] = None, prelu: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, out_dtype=None, tile: int = -1, post_act=None,
           aff: Optional[tuple] = None, aff_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = post_act(prelu(act(conv(x, w) + bias)) + residual)   (NHWC; w [Cout, KH, KW, Cin]).

    ``aff`` = (scale, shift) fp32 [Cout]: a per-channel affine of the bf16-rounded result -- the
    next layer's pre-conv BatchNorm -- written to ``aff_out`` (a second output; ``True``: allocate
    it and return ``(out, aff_out)``) or, when ``aff_out`` is None, to ``out`` in place of the
    plain result."""
    N, H, W, Cin = x.shape
    Cout, KH, KW, _ = w.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, padding, dilation)
    if out is None:
        out = torch.empty((N, Ho, Wo, Cout), device=x.device, dtype=out_dtype or x.dtype)
    if aff_out is True:
        ao = torch.empty_like(out)
        conv2d(x, w, bias, stride, padding, dilation, act, residual, prelu, out, out_dtype, tile, post_act, aff, ao)
        return out, ao
    a = act_id(act)
    if x.is_cuda:
        hip_ops().conv2d(x, w, bias, residual, prelu, a, list(_pair(stride)), _pad_arg(padding),
                         list(_pair(dilation)), out, int(tile), act_id(post_act),
                         aff[0] if aff is not None else None, aff[1] if aff is not None else None, aff_out)
        return out
    pt, pl, pb, pr = _pads4(padding)
    y = F.conv2d(F.pad(x.float().permute(0, 3, 1, 2), (pl, pr, pt, pb)), w.float().permute(0, 3, 1, 2), None,
                 _pair(stride), 0, _pair(dilation)).permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    y = _act_ref(y, a)
    if prelu is not None:
        y = torch.where(y > 0, y, y * prelu.float())
    if residual is not None:
        y = y + residual.float()
    y = _act_ref(y, act_id(post_act))
    if aff is not None:
        z = y.to(out.dtype).float() * aff[0].float() + aff[1].float()
        if aff_out is None:
            y = z
        else:
            aff_out.copy_(z.to(aff_out.dtype))
    out.copy_(y.to(out.dtype))
    return out


def conv2d_dw(x, w, bias=None, stride=1, padding=0, dilation=1, act=None, out=None):
    """Depthwise conv, NHWC; w [KH, KW, C]."""
    N, H, W, C = x.shape
    KH, KW, _ = w.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, padding, dilation)
    if out is None:
        out = torch.empty((N, Ho, Wo, C), device=x.device, dtype=x.dtype)
    a = act_id(act)
    if x.is_cuda:
        pt, pl = _pads4(padding)[:2]            # bottom / right follow from the out size
        hip_ops().conv2d_dw(x.contiguous(), w.contiguous(), bias, a, list(_pair(stride)), [pt, pl],
                            list(_pair(dilation)), out)
        return out
    wt = w.float().permute(2, 0, 1).unsqueeze(1)  # [C, 1, KH, KW]
    pt, pl, pb, pr = _pads4(padding)
    y = F.conv2d(F.pad(x.float().permute(0, 3, 1, 2), (pl, pr, pt, pb)), wt, None, _pair(stride), 0, _pair(dilation),
                 groups=C)
    y = y.permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    out.copy_(_act_ref(y, a).to(out.dtype))
    return out


def channel_affine(x, scale, shift, act=None, prelu=None, out=None):
    """y = x * scale[c] + shift[c] (-> act -> PReLU) — un-foldable BatchNorm (pre-conv BN)."""
    if out is None:
        out = torch.empty_like(x)
    a = act_id(act)
    if x.is_cuda:
        hip_ops().channel_affine(x.contiguous(), scale.float().contiguous(), shift.float().contiguous(), out, a, prelu)
        return out
    y = _act_ref(x.float() * scale.float() + shift.float(), a)
    if prelu is not None:
        y = torch.where(y > 0, y, y * prelu.float())
    out.copy_(y.to(out.dtype))
    return out


def pool2d(x, kernel, stride, padding=0, is_max=True):
    N, H, W, C = x.shape
    k, s, p = _pair(kernel), _pair(stride), _pair(padding)
    Ho, Wo = (H + 2 * p[0] - k[0]) // s[0] + 1, (W + 2 * p[1] - k[1]) // s[1] + 1
    if x.is_cuda:
        out = torch.empty((N, Ho, Wo, C), device=x.device, dtype=x.dtype)
        hip_ops().pool2d(x.contiguous(), out, list(k), list(s), list(p), bool(is_max))
        return out
    xn = x.float().permute(0, 3, 1, 2)
    y = F.max_pool2d(xn, k, s, p) if is_max else F.avg_pool2d(xn, k, s, p, count_include_pad=True)
    return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()


def global_avgpool(x) -> torch.Tensor:
    """NHWC -> fp32 [N, C]."""
    if x.is_cuda:
        out = torch.empty((x.shape[0], x.shape[3]), device=x.device, dtype=torch.float32)
        hip_ops().global_avgpool(x.contiguous(), out)
        return out
    return x.float().mean(dim=(1, 2))


def upsample_add(x, add=None, factor=2, out=None):
    """nearest-upsample x by ``factor`` (+ add) -> out (may be a channel slice of a concat buffer)."""
    N, H, W, C = x.shape
    if out is None:
        out = torch.empty((N, H * factor, W * factor, C), device=x.device, dtype=x.dtype)
    if x.is_cuda:
        hip_ops().upsample_add(x.contiguous(), add, out, int(factor))
        return out
    y = x.float().repeat_interleave(factor, 1).repeat_interleave(factor, 2)
    if add is not None:
        y = y + add.float()
    out.copy_(y.to(out.dtype))
    return out


def channel_scale_(x, s):
    """SE re-weighting in place: x[n, h, w, c] *= s[n, c] (s fp32 [N, C])."""
    if x.is_cuda:
        hip_ops().channel_scale_(x, s.float().contiguous())
        return x
    x.copy_((x.float() * s.float()[:, None, None, :]).to(x.dtype))
    return x


def pixel_shuffle_up(y, C, factor=2):
    """[N, H, W, f*f*C] (ConvTranspose-as-GEMM output) -> [N, H*f, W*f, C]."""
    N, H, W, _ = y.shape
    out = torch.empty((N, H * factor, W * factor, C), device=y.device, dtype=y.dtype)
    if y.is_cuda:
        hip_ops().pixel_shuffle_up(y.contiguous(), out, int(factor))
        return out
    t = y.reshape(N, H, W, factor, factor, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H * factor, W * factor, C)
    out.copy_(t)
    return out


def db_head_up(h, w1, b1, w2p, b2):
    """DBNet head tail fused (csrc/conv.hip db_head_up): h [N, H4, W4, C] bf16 (C 16 or 32) through
    up1 (2x2 s2 ConvTranspose C -> C + ReLU, weights w1 [4C, C] bf16 / b1 [4C] fp32) and up2 (2x2 s2
    ConvTranspose C -> 1 + sigmoid, MFMA-packed w2p [4, 64, 8] from :func:`db_head_pack_up2`, b2 [4])
    -> probability map [N, 4*H4, 4*W4] fp32."""
    N, H4, W4, _ = h.shape
    out = torch.empty((N, 4 * H4, 4 * W4), device=h.device, dtype=torch.float32)
    hip_ops().db_head_up(h, w1, b1, w2p, b2, out)
    return out


def db_head_pack_up2(w2: torch.Tensor) -> torch.Tensor:
    """up2's weights [4 (kh*2 + kw), C] -> the A fragments of db_head_up's four k-steps [4, 64, 8] bf16:
    k-step s1, lane l holds row l & 15 (= 4*s1 + s2 when nonzero) at the permuted channels
    c(l >> 4, j) = 4*(l >> 4) + j for j < 4, 12 + 4*(l >> 4) + j for j >= 4 (see the kernel)."""
    C = w2.shape[1]
    lane = np.arange(64)
    row, hq = lane & 15, lane >> 4
    j = np.arange(8)
    c = np.where(j[None, :] < 4, 4 * hq[:, None] + j[None, :], 12 + 4 * hq[:, None] + j[None, :])    # [64, 8]
    w = w2.float().cpu().numpy()
    out = np.zeros((4, 64, 8), np.float32)
    for s1 in range(4):
        sel = (row >> 2) == s1
        ok = sel[:, None] & (c < C)
        vals = w[(row & 3)[:, None].repeat(8, 1), np.minimum(c, C - 1)]
        out[s1] = np.where(ok, vals, 0.0)
    return torch.from_numpy(out).to(torch.bfloat16)


def conv_weight_from_torch(w: torch.Tensor, cin_pad: Optional[int] = None) -> torch.Tensor:
    """[Cout, Cin, KH, KW] -> [Cout, KH, KW, Cin(_pad)] (zero-padded input channels)."""
    wt = w.permute(0, 2, 3, 1).contiguous()
    if cin_pad is not None and cin_pad > wt.shape[3]:
        wt = F.pad(wt, (0, cin_pad - wt.shape[3]))
    return wt.contiguous()
