"""Compute ops of lumen_amd.

Every op has exactly two implementations:

* GPU tensors -> the hand-written gfx950 HIP kernel (``torch.ops.lumen.*``); the
  native library is *required* (no silent PyTorch fallback on a GPU).
* CPU tensors -> a plain PyTorch fp32 reference with identical semantics.  This
  is the "CPU reference path" used for plumbing tests (BASELINE config #1) and
  as the numerical oracle the GPU kernels are tested against.
"""
from __future__ import annotations

import functools
import math
import threading
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from .._native import hip_ops
from ..utils.h2d import h2d

ACTS = {
    None: 0, "none": 0, "gelu": 1, "quick_gelu": 2, "relu": 3, "silu": 4, "gelu_tanh": 5,
    "hardswish": 6, "sigmoid": 7, "leaky": 8, "hardsigmoid": 9,
}


# Held around every hipGraph capture in the process (models/vlm.py, runtime/engine.py):
# torch.cuda.graph() enters with a device-wide synchronize + empty_cache, which fails (or
# invalidates) a capture another thread has in progress, thread_local mode or not.
CAPTURE_LOCK = threading.RLock()


def private_stream(device) -> "torch.cuda.Stream":
    """A HIP stream that nothing else in the process uses (never from PyTorch's recycled pool):
    kernels key their split-K tickets / workspaces by stream (csrc/workspace.h), and a hipGraph
    captured on a stream keeps those buffers; a pool stream could later be handed to another
    thread's eager work, or another model's graph, that would then share them."""
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    try:
        return torch.cuda.ExternalStream(int(hip_ops().private_stream(idx)), device=torch.device("cuda", idx))
    except (AttributeError, RuntimeError):   # extension without the op
        return torch.cuda.Stream(device=torch.device("cuda", idx))


def _act_ref(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == 0:
        return x
    if act == 1:
        return F.gelu(x)
    if act == 2:
        return x * torch.sigmoid(1.702 * x)
    if act == 3:
        return F.relu(x)
    if act == 4:
        return F.silu(x)
    if act == 5:
        return F.gelu(x, approximate="tanh")
    if act == 6:
        return F.hardswish(x)
    if act == 7:
        return torch.sigmoid(x)
    if act == 8:
        return F.leaky_relu(x, 0.1)
    if act == 9:
        return torch.clamp(x / 6.0 + 0.5, 0.0, 1.0)
    raise ValueError(act)


def act_id(act) -> int:
    if isinstance(act, int):
        return act
    return ACTS[act]


def apply_act(x: torch.Tensor, act) -> torch.Tensor:
    """Standalone activation (reference semantics) — used by conv paths on CPU."""
    return _act_ref(x.float(), act_id(act)).to(x.dtype)


# --------------------------------------------------------------------------- GEMM
def linear(
    x: torch.Tensor,
    w: torch.Tensor,
    bias: Optional[torch.Tensor] = None,
    act=None,
    residual: Optional[torch.Tensor] = None,
    table: Optional[torch.Tensor] = None,
    table_period: int = 0,
    table_offset: int = 0,
    alpha: float = 1.0,
    out: Optional[torch.Tensor] = None,
    out_dtype: Optional[torch.dtype] = None,
    out_group: int = 0,
    out_group_stride: int = 0,
    out_row_offset: int = 0,
    tile: int = -1,
    glu: bool = False,
    w_scale: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """y = epi(alpha * x @ w.T): (+bias) -> act -> (+table[m % P + off]) -> (+residual[orow]).

    ``w`` may be an OCP ``torch.float8_e4m3fn`` weight with per-output-row fp32
    ``w_scale`` [N] (weight-only fp8, :func:`quantize_fp8_rows`): the HIP kernels widen
    it to bf16 in registers and apply the scale in the fp32 epilogue.

    ``x`` is [M, K] (or [..., K]), ``w`` is [N, K].  With ``out_group`` > 0 row m is
    written to ``(m // G) * GS + RO + m % G`` of ``out`` (patch rows into a token
    buffer).  ``residual`` is indexed by the *output* row.  ``glu``: the rows of ``w``
    interleave [gate 8 | up 8] per 16 (see :func:`glu_interleave`) and the output is
    silu(gate) * up with N/2 columns (SwiGLU fused into the epilogue).
    """
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    a = act_id(act)
    NO = N // 2 if glu else N
    if out is None:
        assert out_group == 0, "out_group needs an explicit out tensor"
        out = torch.empty((M, NO), device=x.device, dtype=out_dtype or x.dtype)
        ret_shape = (*lead, NO)
    else:
        ret_shape = None
    out2 = out if out.dim() == 2 else out.view(-1, out.shape[-1])
    if w.dtype == torch.float8_e4m3fn:
        assert w_scale is not None, "fp8 weights need w_scale"
        assert table is None and out_group == 0 and alpha == 1.0, "fp8 GEMM: bias / act / SwiGLU / residual epilogues"
        if x.is_cuda:
            if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0:
                x2 = x2.contiguous()
            res2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
            hip_ops().gemm_w8(x2, w, w_scale, bias, res2, a, out2, int(bool(glu)))
            return out.view(ret_shape) if ret_shape is not None else out
        w = w.float() * w_scale.float()[:, None]
    if x.is_cuda:
        if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0:
            x2 = x2.contiguous()
        res2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
        hip_ops().gemm(x2, w, bias, res2, table, int(table_period), int(table_offset), a, float(alpha), out2,
                       int(out_group), int(out_group_stride), int(out_row_offset), int(tile), None, int(bool(glu)))
    else:
        y = (x2.float() @ w.float().t()) * alpha
        if bias is not None:
            y = y + bias.float()[:N]
        if glu:
            gu = y.view(M, N // 16, 2, 8)
            out2[:, :NO] = (F.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, NO).to(out2.dtype)
            return out.view(ret_shape) if ret_shape is not None else out
        y = _act_ref(y, a)
        m = torch.arange(M)
        orow = (m // out_group) * out_group_stride + out_row_offset + m % out_group if out_group > 0 else m
        if table is not None:
            y = y + table.float()[(m % table_period) + table_offset, :N]
        if residual is not None:
            r2 = residual.reshape(-1, residual.shape[-1])
            y = y + r2.float()[orow, :N]
        out2[orow, :N] = y.to(out2.dtype)
    if ret_shape is not None:
        return out.view(ret_shape)
    return out


FP8_E4M3_MAX = 448.0


def quantize_fp8_rows(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """[N, K] weight -> (OCP e4m3fn [N, K], fp32 per-row scale [N]) with w ~= w8 * scale[:, None]."""
    wf = w.float()
    s = (wf.abs().amax(dim=1) / FP8_E4M3_MAX).clamp_min(1e-12)
    return (wf / s[:, None]).clamp(-FP8_E4M3_MAX, FP8_E4M3_MAX).to(torch.float8_e4m3fn), s.contiguous()


def quant_rows_fp8(x: torch.Tensor, out: Optional[torch.Tensor] = None,
                   scale: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-token dynamic fp8: bf16 rows [M, K] -> (e4m3fn [M, K], fp32 scale [M]) with
    x ~= x8 * scale[:, None] (scale = max|x_m| / 448)."""
    M, K = x.shape
    if out is None:
        out = torch.empty((M, K), device=x.device, dtype=torch.float8_e4m3fn)
    if scale is None:
        scale = torch.empty((M,), device=x.device, dtype=torch.float32)
    if x.is_cuda:
        hip_ops().quant_rows_fp8(x, out, scale)
    else:
        xf = x.float()
        s = (xf.abs().amax(dim=1) / FP8_E4M3_MAX).clamp_min(1e-12 / FP8_E4M3_MAX)
        out[:M].copy_((xf / s[:, None]).clamp(-FP8_E4M3_MAX, FP8_E4M3_MAX).to(torch.float8_e4m3fn))
        scale[:M].copy_(s)
    return out, scale


def rms_norm_quant_fp8(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-6, add: Optional[torch.Tensor] = None,
                       resid_out: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                       scale: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
    """RMSNorm(x [+ add], stored to ``resid_out``) quantised per token to fp8 in the same
    kernel: the input of an fp8 x fp8 projection (:func:`linear_f8`)."""
    M, K = x.shape
    if out is None:
        out = torch.empty((M, K), device=x.device, dtype=torch.float8_e4m3fn)
    if scale is None:
        scale = torch.empty((M,), device=x.device, dtype=torch.float32)
    if x.is_cuda:
        hip_ops().rms_norm_quant_fp8(x, add, resid_out, w, float(eps), out, scale)
        return out, scale
    xf = x.float() + (add.float() if add is not None else 0.0)
    if resid_out is not None:
        resid_out.copy_(xf.to(resid_out.dtype))
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return quant_rows_fp8(y, out, scale)


def linear_dec(x: torch.Tensor, w: torch.Tensor, w_scale: Optional[torch.Tensor] = None,
               bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None, glu: bool = False, norm_eps: Optional[float] = None,
               ssq_in: Optional[torch.Tensor] = None, ssq_out: Optional[torch.Tensor] = None,
               out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Decode projection (M <= 32 rows) on the skinny kernels with RMSNorm folding:

    * ``norm_eps`` set: y = rstd(x) * (x @ w^T) (+bias ...), i.e. ``linear(rms_norm(x), w)``
      for a ``w`` whose norm gamma is already folded in (``LLM.fold_norms``).  rstd comes
      from ``ssq_in`` ([>= M, K / 16] per-tile sums of squares written by the GEMM that
      produced x) or is computed from x.
    * ``ssq_out`` ([>= M, N / 16] fp32): this GEMM (bf16 residual-stream output) writes the
      per-16-column sums of squares of its stored rows for the next norm-folded GEMM.

    CPU (and M > 32): plain ``rms_norm`` (unit gamma) + :func:`linear`; ``ssq_*`` unused."""
    M, K = x.shape
    N = w.shape[0]
    NO = N // 2 if glu else N
    if out is None:
        out = torch.empty((M, NO), device=x.device, dtype=out_dtype or x.dtype)
    if x.is_cuda and 0 < M <= 32:
        if x.stride(-1) != 1 or x.stride(0) % 8 != 0:
            x = x.contiguous()
        hip_ops().gemm_dec(x, w, w_scale, bias, residual, out, int(bool(glu)), int(norm_eps is not None),
                           float(norm_eps or 0.0), ssq_in if norm_eps is not None else None, ssq_out)
        return out
    if norm_eps is not None:
        x = rms_norm(x, torch.ones(K, dtype=x.dtype, device=x.device), norm_eps)
    return linear(x, w, bias=bias, residual=residual, out=out, glu=glu, w_scale=w_scale)


def linear_f8(x8: torch.Tensor, x_scale: torch.Tensor, w8: torch.Tensor, w_scale: torch.Tensor,
              bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, glu: bool = False,
              out_dtype: torch.dtype = torch.bfloat16, splits: int = -1, variant: int = 0) -> torch.Tensor:
    """W8A8 projection on the gfx950 fp8 matrix cores (csrc/gemm_f8.hip):
    y = epi((x8 @ w8^T) * x_scale[m] * w_scale[n]) with fp32 bias, SwiGLU (``glu``, see
    :func:`glu_interleave`) or + residual.  x8 / w8 are e4m3fn, K % 128 == 0."""
    M, K = x8.shape
    N = w8.shape[0]
    NO = N // 2 if glu else N
    if out is None:
        out = torch.empty((M, NO), device=x8.device, dtype=out_dtype)
    if x8.is_cuda:
        hip_ops().gemm_f8(x8, x_scale, w8, w_scale, bias, residual, out, int(bool(glu)), int(splits), int(variant))
        return out
    y = (x8.float() @ w8.float().t()) * x_scale.float()[:M, None] * w_scale.float()[None, :]
    if bias is not None:
        y = y + bias.float()[:N]
    if glu:
        gu = y.view(M, N // 16, 2, 8)
        out[:, :NO] = (F.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, NO).to(out.dtype)
        return out
    if residual is not None:
        y = y + residual.float()[:M, :N]
    out[:M, :N] = y.to(out.dtype)
    return out


def mx_planes(qs_rows: torch.Tensor) -> torch.Tensor:
    """E8M0 bytes [M, K/32] (row-major) -> the kernels' K-step planes [K/128, M, 4]: the byte of
    (row m, 32-column block b) at [b // 4, m, b % 4], so a GEMM's per-K-step load of 64 rows'
    scales is 256 contiguous bytes."""
    M, nb = qs_rows.shape
    out = torch.empty((nb // 4, M, 4), dtype=qs_rows.dtype, device=qs_rows.device)   # standard strides
    out.copy_(qs_rows.reshape(M, nb // 4, 4).permute(1, 0, 2))
    return out


def mx_rows(qs: torch.Tensor) -> torch.Tensor:
    """Scale planes [K/128, M, 4] -> row-major E8M0 bytes [M, K/32]."""
    P, M, _ = qs.shape
    return qs.permute(1, 0, 2).reshape(M, P * 4)


def mx_quant_ref(x: torch.Tensor):
    """MX fp8 of rows x [M, K] (K % 128 == 0), the arithmetic of the GPU producers: per 32
    columns e = the smallest exponent with amax / 2^e <= 448 (E8M0 byte e + 127), values
    x * 2^-e saturated to e4m3fn.  -> (q8 [M, K] float8_e4m3fn, qs [K/128, M, 4] uint8 scale
    planes, see :func:`mx_planes`)."""
    M, K = x.shape
    xb = x.float().reshape(M, K // 32, 32)
    t = xb.abs().amax(-1) * torch.tensor(1.0 / 448.0, dtype=torch.float32)
    m, ex = torch.frexp(t)
    e = torch.where(m == 0.5, ex - 1, ex)
    e = torch.where(t == 0, torch.full_like(e, -127), e)
    e = torch.where((t > 0) & (t < 2.0 ** -126), torch.full_like(e, -126), e).clamp(-127, 126)
    q = (xb * torch.exp2(-e.float())[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.reshape(M, K), mx_planes((e + 127).to(torch.uint8))


def mx_dequant(q8: torch.Tensor, qs: torch.Tensor) -> torch.Tensor:
    """MX fp8 [M, K] + E8M0 scale planes [K/128, >= M, 4] -> fp32 [M, K]."""
    M, K = q8.shape
    s = torch.exp2(mx_rows(qs[:, :M]).float() - 127.0)
    return (q8.float().reshape(M, K // 32, 32) * s[..., None]).reshape(M, K)


def quant_rows_mx(x: torch.Tensor, q8: Optional[torch.Tensor] = None, qs: Optional[torch.Tensor] = None,
                  ssq: Optional[torch.Tensor] = None):
    """bf16 rows [M, K] -> MX fp8 (q8 [M, K] e4m3fn, qs [K/128, M, 4] E8M0 planes) and, when ``ssq`` is given,
    its per-(row, 128-column) sums of squares [M, K/128] (the rstd source of a norm-folded
    consumer, ops.linear_mx(ssq_in=...)).  Returns (q8, qs)."""
    M, K = x.shape
    if q8 is None:
        q8 = torch.empty((M, K), device=x.device, dtype=torch.float8_e4m3fn)
    if qs is None:
        qs = torch.empty((K // 128, M, 4), device=x.device, dtype=torch.uint8)
    if x.is_cuda:
        hip_ops().quant_rows_mx(x, q8, qs, ssq)
        return q8, qs
    a, b = mx_quant_ref(x)
    q8[:M].copy_(a)
    qs[:, :M].copy_(b)
    if ssq is not None:
        ssq[:M, :K // 128] = (x.float() ** 2).reshape(M, K // 128, 128).sum(-1)
    return q8, qs


def linear_mx(x8: torch.Tensor, xs: torch.Tensor, w8: torch.Tensor, w_scale: torch.Tensor,
              bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, glu: bool = False, ssq_in: Optional[torch.Tensor] = None,
              norm_eps: float = 0.0, q_out: Optional[tuple] = None, ssq_out: Optional[torch.Tensor] = None,
              write_out: bool = True, variant: int = 0, act=None, row_aff: Optional[torch.Tensor] = None,
              col_aff: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """W8A8 projection with MX (block-scaled) activations on the gfx950 matrix cores
    (csrc/gemm_f8.hip::gemm_mx): A = x8 * 2^(xs - 127) per 32 columns feeds the MFMA scale operand,
    so producers quantise with block-local scales and no per-row quantisation pass runs.

    y = epi(rstd[m] * (A @ w8^T) * w_scale[n]): ``ssq_in`` [M, K/128] (the producer's sums of
    squares) gives rstd = rsqrt(sum / K + norm_eps) -- the RMSNorm whose gamma was folded into w8;
    then fp32 bias, SwiGLU or + residual.  Outputs: bf16 ``out`` (skipped with ``write_out=False``,
    SwiGLU only), ``q_out = (q8, qs)`` an MX fp8 copy of the output for the next projection,
    ``ssq_out`` [M, N/128] per-(row, 128-column) sums of squares of the stored bf16 values."""
    M, K = x8.shape
    N = w8.shape[0]
    NO = N // 2 if glu else N
    if out is None and write_out:
        out = torch.empty((M, NO), device=x8.device, dtype=torch.bfloat16)
    q8, qs = q_out if q_out is not None else (None, None)
    a = act_id(act)
    if x8.is_cuda:
        hip_ops().gemm_mx(x8, xs, w8, w_scale, bias, residual, out if write_out else None, int(bool(glu)), ssq_in,
                          float(norm_eps), q8, qs, ssq_out, int(variant), a, row_aff, col_aff)
        return out
    y = (mx_dequant(x8, xs) @ w8.float().t()) * w_scale.float()[None, :N]
    if ssq_in is not None:
        y = y * torch.rsqrt(ssq_in.float()[:M].sum(1, keepdim=True) / K + norm_eps)
    if row_aff is not None:
        y = y * row_aff[:M, :1] + row_aff[:M, 1:] * col_aff[0] + col_aff[1]
    if bias is not None:
        y = y + bias.float()[:N]
    if a and not glu:
        y = _act_ref(y, a)
    if glu:
        gu = y.view(M, N // 16, 2, 8)
        r = (F.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, NO)
        if write_out:
            out[:M, :NO] = r.to(out.dtype)
        if q8 is not None:
            a, b = mx_quant_ref(r)
            q8[:M].copy_(a)
            qs[:, :M].copy_(b)
        return out
    if residual is not None:
        y = y + residual.float()[:M, :N]
    yb = y.to(torch.bfloat16) if write_out else y
    if write_out:
        out[:M, :N] = yb
    if q8 is not None:
        a, b = mx_quant_ref(yb.float())
        q8[:M].copy_(a)
        qs[:, :M].copy_(b)
    if ssq_out is not None:
        ssq_out[:M, :N // 128] = (yb.float() ** 2).reshape(M, N // 128, 128).sum(-1)
    return out


def glu_interleave(w_gate: torch.Tensor, w_up: torch.Tensor) -> torch.Tensor:
    """[I, K] gate / up projections -> [2I, K] rows grouped [gate 8 | up 8] per 16 (``linear(glu=True)``)."""
    I, K = w_gate.shape
    assert I % 8 == 0 and w_up.shape == w_gate.shape
    return torch.stack([w_gate.reshape(I // 8, 8, K), w_up.reshape(I // 8, 8, K)], 1).reshape(2 * I, K)


# --------------------------------------------------------------------------- norms
def _norm_ref(x, w, b, eps, mode):
    xf = x.float()
    if mode == 0:
        mu = xf.mean(-1, keepdim=True)
        var = ((xf - mu) ** 2).mean(-1, keepdim=True)
        y = (xf - mu) * torch.rsqrt(var + eps) * w.float()
        if b is not None:
            y = y + b.float()
    else:
        y = xf * torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps) * w.float()
    return y


def _norm(x, w, b, eps, mode, row_idx=None, add=None, resid_out=None, out=None, out_dtype=None):
    D = x.shape[-1]
    x2 = x.reshape(-1, D)
    rows = row_idx.numel() if row_idx is not None else x2.shape[0]
    if out is None:
        out = torch.empty((rows, D), device=x.device, dtype=out_dtype or x.dtype)
    if x.is_cuda:
        add2 = add.reshape(-1, D) if add is not None else None
        hip_ops().norm(x2, row_idx, add2, resid_out, w, b, out.view(-1, D), float(eps), int(mode))
    else:
        src = x2[row_idx] if row_idx is not None else x2
        h = src.float()
        if add is not None:
            a2 = add.reshape(-1, D)
            h = h + (a2[row_idx] if row_idx is not None else a2).float()
        if resid_out is not None:
            resid_out.copy_(h.to(resid_out.dtype))
        out.view(-1, D).copy_(_norm_ref(h, w, b, eps, mode).to(out.dtype))
    return out


def layer_norm(x, w, b=None, eps=1e-5, row_idx=None, out=None, out_dtype=None, add=None, resid_out=None):
    """LayerNorm(x [+ add]); when ``resid_out`` is given the pre-norm sum is stored there
    (the residual-stream update of a pre-LN block fused into the next norm)."""
    out = _norm(x, w, b, eps, 0, row_idx=row_idx, add=add, resid_out=resid_out, out=out, out_dtype=out_dtype)
    if row_idx is None and out.shape != x.shape and out.numel() == x.numel():
        return out.view(x.shape)
    return out


def ln_row_stats(x: torch.Tensor, eps: float = 1e-5, out: Optional[torch.Tensor] = None,
                 q_out: Optional[tuple] = None) -> torch.Tensor:
    """LayerNorm statistics of the rows of x [R, D]: fp32 [R, 2] = (rstd, -mean * rstd), the
    row half of a LayerNorm folded into the next projection (:func:`linear_lnf`).  ``q_out``
    = (q8 [R, D], qs [D/128, R, 4]): the raw rows also as MX fp8 (the W8A8 :func:`linear_mx`
    operand of that projection)."""
    x2 = x.reshape(-1, x.shape[-1])
    if out is None:
        out = torch.empty((x2.shape[0], 2), device=x.device, dtype=torch.float32)
    if x.is_cuda:
        if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0:
            x2 = x2.contiguous()
        q8, qs = q_out if q_out is not None else (None, None)
        hip_ops().ln_row_stats(x2, out, float(eps), q8, qs)
        return out
    if q_out is not None:
        quant_rows_mx(x2, q_out[0], q_out[1])
    xf = x2.float()
    mean = xf.mean(-1)
    rstd = torch.rsqrt(((xf - mean[:, None]) ** 2).mean(-1) + eps)
    out[:, 0] = rstd
    out[:, 1] = -mean * rstd
    return out


def ln_fold_weights(w: torch.Tensor, bias: Optional[torch.Tensor], gamma: torch.Tensor,
                    beta: Optional[torch.Tensor]) -> tuple[torch.Tensor, torch.Tensor]:
    """Fold LayerNorm(gamma, beta) into the projection (w [N, K], bias [N]) that consumes it:
    returns w' = w * gamma (w's dtype) and col_aff fp32 [2, N] = (colsum(w'), bias + w . beta),
    colsum taken over the rounded w' the GEMM multiplies with."""
    wf = (w.float() * gamma.float()[None, :]).to(w.dtype)
    cs = wf.float().sum(1)
    cb = bias.float().clone() if bias is not None else torch.zeros(w.shape[0], device=w.device)
    if beta is not None:
        cb += w.float() @ beta.float()
    return wf, torch.stack([cs, cb]).contiguous()


def linear_lnf(x: torch.Tensor, wf: torch.Tensor, col_aff: torch.Tensor, row_aff: torch.Tensor, act=None,
               out: Optional[torch.Tensor] = None, tile: int = -1) -> torch.Tensor:
    """act(LayerNorm(x) . w^T + b) with the norm folded in (:func:`ln_fold_weights`,
    :func:`ln_row_stats`): act(rstd * (x . w'^T) - mean * rstd * colsum(w') + b') over the raw rows
    of x [M, K] (bf16 on the GPU), so no normalised copy of x is written."""
    M, N = x.shape[0], wf.shape[0]
    if out is None:
        out = torch.empty((M, N), device=x.device, dtype=x.dtype)
    a = act_id(act)
    if x.is_cuda:
        hip_ops().gemm_lnf(x, wf, col_aff, row_aff, a, out, int(tile))
        return out
    y = (x.float() @ wf.float().t()) * row_aff[:M, :1] + row_aff[:M, 1:] * col_aff[0] + col_aff[1]
    out.copy_(_act_ref(y, a).to(out.dtype))
    return out


def rms_norm(x, w, eps=1e-6, add=None, resid_out=None, out=None, out_dtype=None):
    """RMSNorm(x [+ add]); when ``resid_out`` is given the pre-norm sum is stored there."""
    o = _norm(x, w, None, eps, 1, add=add, resid_out=resid_out, out=out, out_dtype=out_dtype)
    return o.view(*x.shape[:-1], x.shape[-1]) if o.numel() == x.numel() else o


def l2_normalize_(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """In-place row L2 normalisation of an fp32 [R, D] tensor."""
    if x.is_cuda:
        hip_ops().l2norm_(x, float(eps))
    else:
        x.div_(x.norm(dim=-1, keepdim=True).clamp_min(eps))
    return x


def cls_fill(x: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, seq: int) -> None:
    """x[b*seq + 0] = cls + pos[0] for every sequence in the flat [B*seq, D] buffer."""
    if x.is_cuda:
        hip_ops().cls_fill(x, cls, pos, int(seq))
    else:
        B = x.shape[0] // seq
        x.view(B, seq, -1)[:, 0] = (cls.float() + pos.reshape(-1, x.shape[-1])[0].float()).to(x.dtype)


def embed(ids: torch.Tensor, table: torch.Tensor, pos: Optional[torch.Tensor] = None, id_offset: int = 0,
          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token-embedding gather (+ positional row ``pos[s]`` for position s of each sequence)."""
    S = ids.shape[-1]
    D = table.shape[1]
    if out is None:
        out = torch.empty((*ids.shape, D), device=table.device, dtype=table.dtype)
    if table.is_cuda:
        hip_ops().embed_gather(ids.contiguous().to(torch.long), table, pos, out, int(S), int(id_offset))
    else:
        idx = ids.long() - id_offset
        valid = (idx >= 0) & (idx < table.shape[0])
        e = table.float()[idx.clamp(0, table.shape[0] - 1)] * valid.unsqueeze(-1)
        if pos is not None:
            e = e + pos.float().reshape(-1, D)[:S]
        out.copy_(e.to(out.dtype))
    return out


# --------------------------------------------------------------------------- attention
def attention(q, k, v, scale: Optional[float] = None, causal: bool = False, kv_len=None, out=None):
    """Fused softmax(q k^T * scale [+mask]) v.

    q: [B, Sq, H, D]; k, v: [B, Sk, Hkv, D] (GQA when Hkv < H); any strides with unit
    inner stride (e.g. views into a packed QKV projection).  Returns [B, Sq, H, D].
    ``kv_len`` (int32 [B]) masks padded keys; ``causal`` aligns the last query with
    the last key (prefill with a KV-cache prefix).
    """
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if out is None:
        out = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
    if q.is_cuda:
        kl = kv_len.to(torch.int32) if kv_len is not None else None
        hip_ops().attention(q, k, v, out, kl, float(scale), bool(causal))
        return out
    qf = q.float().transpose(1, 2)
    rep = H // Hkv
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    mask = torch.zeros((B, 1, Sq, Sk), dtype=torch.bool)
    if kv_len is not None:
        kl = kv_len.long().view(B, 1, 1, 1)
        mask |= torch.arange(Sk).view(1, 1, 1, Sk) >= kl
    if causal:
        qi = torch.arange(Sq).view(Sq, 1) + (Sk - Sq)
        mask |= (torch.arange(Sk).view(1, Sk) > qi).view(1, 1, Sq, Sk)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = (p @ vf).transpose(1, 2)
    out.copy_(o.to(out.dtype))
    return out


def attention_mx(q, k, v, scale: Optional[float] = None, causal: bool = False, kv_len=None,
                 q_out: Optional[tuple] = None, out=None):
    """:func:`attention` whose output leaves as MX fp8 (the W8A8 o-projection's operand,
    :func:`linear_mx`): returns (o8 [B*Sq, H*D] e4m3fn, os [H*D/128, B*Sq, 4] E8M0 planes).
    ``out`` (bf16 [B, Sq, H, D]) is also written when given.  On the CPU: attention + mx_quant_ref."""
    B, Sq, H, D = q.shape
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if q_out is None:
        q_out = (torch.empty((B * Sq, H * D), device=q.device, dtype=torch.float8_e4m3fn),
                 torch.empty((H * D // 128, B * Sq, 4), device=q.device, dtype=torch.uint8))
    o8, os_ = q_out
    if q.is_cuda:
        kl = kv_len.to(torch.int32) if kv_len is not None else None
        hip_ops().attention_mx(q, k, v, out, o8, os_, kl, float(scale), bool(causal))
        return o8, os_
    o = attention(q, k, v, scale=scale, causal=causal, kv_len=kv_len)
    if out is not None:
        out.copy_(o)
    of = attention(q.float(), k.float(), v.float(), scale=scale, causal=causal, kv_len=kv_len)
    a, b = mx_quant_ref(of.reshape(B * Sq, H * D))
    o8.copy_(a)
    os_[:, :B * Sq].copy_(b)
    return o8, os_


# --------------------------------------------------------------------------- top-k
def row_topk(scores: torch.Tensor, k: int, scale: float = 1.0, with_lse: bool = False, index_offset: int = 0):
    """Per-row top-k (descending) of fp32 scores [B, N]; optionally the row logsumexp(scale*s).

    Returns (values [B,k] f32, indices [B,k] int32, lse [B] f32 | None).
    """
    B, N = scores.shape
    k = min(k, N)
    if scores.is_cuda:
        v = torch.empty((B, k), device=scores.device, dtype=torch.float32)
        i = torch.empty((B, k), device=scores.device, dtype=torch.int32)
        lse = torch.empty((B,), device=scores.device, dtype=torch.float32) if with_lse else None
        hip_ops().row_topk(scores.contiguous().float(), int(k), float(scale), v, i, lse, int(index_offset))
        return v, i, lse
    s = scores.float()
    v, i = torch.topk(s, k, dim=-1, largest=True, sorted=True)
    lse = torch.logsumexp(s * scale, dim=-1) if with_lse else None
    return v, (i + index_offset).to(torch.int32), lse


def bank_scores(q: torch.Tensor, bank: torch.Tensor) -> torch.Tensor:
    """cosine scores [B, N] (fp32) of unit query rows q [B, D] against a unit label bank [N, D]."""
    if q.is_cuda:
        D = q.shape[1]
        qb = q.to(bank.dtype) if bank.dtype == torch.bfloat16 else q
        if D % 64 != 0 or bank.dtype != torch.bfloat16:
            return (q.float() @ bank.float().t())
        return linear(qb.contiguous(), bank, out_dtype=torch.float32)
    return q.float() @ bank.float().t()


# --------------------------------------------------------------------------- image prep
FILTERS = {"pil_bicubic": 0, "bicubic": 0, "pil_bilinear": 1, "cv2_linear": 2, "linear": 2, "cv2_cubic": 3}
LAYOUTS = {"nchw": 0, "nhwc": 1, "patches": 2, "nhwc8": 3}


class ImageGeom:
    """Geometry of one image in a ragged preprocessing batch."""

    __slots__ = ("ih", "iw", "off", "cw", "ch", "ox", "oy", "dx", "dy", "dw", "dh")

    def __init__(self, ih, iw, off, cw, ch, ox, oy, dx, dy, dw, dh):
        self.ih, self.iw, self.off = ih, iw, off
        self.cw, self.ch, self.ox, self.oy = cw, ch, ox, oy
        self.dx, self.dy, self.dw, self.dh = dx, dy, dw, dh

    def row(self):
        return [self.ih, self.iw, self.off, self.cw, self.ch, self.ox, self.oy, self.dx, self.dy, self.dw, self.dh]

    @staticmethod
    def resize(ih, iw, off, oh, ow):
        """Plain resize of the whole image to (oh, ow)."""
        return ImageGeom(ih, iw, off, iw, ih, 0, 0, 0, 0, ow, oh)

    @staticmethod
    def letterbox(ih, iw, off, oh, ow, rh, rw):
        """Resize to (rh, rw) placed top-left in an (oh, ow) canvas, rest padded."""
        return ImageGeom(ih, iw, off, iw, ih, 0, 0, 0, 0, rw, rh)

    @staticmethod
    def center_crop(ih, iw, off, size):
        """open_clip / torchvision ``Resize(size)`` (shortest side -> size, long side
        ``int(size * long / short)``) then ``CenterCrop(size)`` (offsets ``int(round(d / 2))``):
        the resized image is placed at a negative destination offset, so the output window
        is its centre (reference torch runtime, lumen-clip torch_backend.py:201-204,568-576)."""
        if iw <= ih:
            nw, nh = size, int(size * ih / iw)
        else:
            nh, nw = size, int(size * iw / ih)
        top, left = int(round((nh - size) / 2.0)), int(round((nw - size) / 2.0))
        return ImageGeom(ih, iw, off, iw, ih, 0, 0, -left, -top, nw, nh)

    @staticmethod
    def pad_square(ih, iw, off, out):
        """Centre on a black max(h, w) square, then resize the square to out x out."""
        s = max(ih, iw)
        return ImageGeom(ih, iw, off, s, s, (s - iw) // 2, (s - ih) // 2, 0, 0, out, out)


@functools.lru_cache(maxsize=256)
def _resample_matrix(in_len: int, out_len: int, filt: int) -> torch.Tensor:
    """[out_len, in_len] fp32 weights of the kernel's 1-D resample (normalised windows;
    cv2 filters replicate the border by clamping the tap index)."""
    scale = in_len / out_len
    m = torch.zeros((out_len, in_len), dtype=torch.float32)
    for i in range(out_len):
        if filt >= 2:
            center = (i + 0.5) * scale - 0.5
            r = 2 if filt == 3 else 1
            x0 = math.floor(center) - r + 1
            xs = list(range(x0, x0 + 2 * r))
            ws = [_filt(float(x) - center, filt) for x in xs]
            xs = [min(max(x, 0), in_len - 1) for x in xs]
        else:
            ss = max(scale, 1.0)
            sup = (2.0 if filt == 0 else 1.0) * ss
            center = (i + 0.5) * scale
            x0 = max(int(center - sup + 0.5), 0)
            x1 = min(int(center + sup + 0.5), in_len)
            xs = list(range(x0, x1))
            ws = [_filt((x - center + 0.5) / ss, filt) for x in xs]
        tot = sum(ws)
        for x, w in zip(xs, ws):
            m[i, x] += w / tot if tot != 0 else 0.0
    return m


def _ref_resample_axis(img: torch.Tensor, out_len: int, axis: int, filt: int) -> torch.Tensor:
    """1-D resample of float image [H, W, 3] along axis (0=H, 1=W) matching the kernel
    (one matmul with the cached weight matrix; PIL filters round to uint8 after each pass,
    cv2 filters after the vertical one)."""
    w = _resample_matrix(img.shape[axis], out_len, filt)
    out = torch.einsum("oi,iwc->owc", w, img) if axis == 0 else torch.einsum("oi,hic->hoc", w, img)
    if filt < 2 or axis == 0:
        out = out.round().clamp(0, 255)
    return out


def _filt(x, f):
    a = -0.5 if f == 0 else -0.75
    x = abs(x)
    if f in (0, 3):
        if x < 1:
            return ((a + 2) * x - (a + 3)) * x * x + 1
        if x < 2:
            return (((x - 5) * x + 8) * x - 4) * a
        return 0.0
    return 1 - x if x < 1 else 0.0


# the fused band kernel only where three workgroups fit a CU's 160 KB of LDS: ViT-L/14 b512 0.63 -> 0.35 ms;
# at one workgroup per CU (ViT-B/32: 43 KB patch image + 43 staged rows) it lost to the two passes, 0.77 vs
# 0.58 ms (profiles/r6_prep_band_v1.txt)
_PREP_BAND_LDS = 53 * 1024


def _prep_band_bounds(geoms, filt: int, lay: int, patch: int, kpad: int, OW: int, out_dtype,
                      pad: float = 0.0) -> Optional[tuple]:
    """(rcap, cwcap, taps) for the fused per-band prep kernel, or None when it does not apply: canvas rows
    one band of ``patch`` output rows reads, staged canvas columns, and taps per resampling window,
    bounded over the batch
    (windows span < 2 * support * max(scale, 1) + 1 samples; a band's windows start and end within
    (patch - 1) * scale of each other)."""
    if lay != 2 or filt not in (0, 1) or out_dtype != torch.bfloat16 or kpad % 8 or patch <= 0 or OW % patch:
        return None
    if not (float(pad).is_integer() and 0 <= pad <= 255):   # the canvas is staged as bytes
        return None
    sup = 2.0 if filt == 0 else 1.0
    taps = rcap = cwcap = 0
    for cw, dw, ch, dh in {(gg.cw, gg.dw, gg.ch, gg.dh) for gg in geoms}:
        sx, sy = cw / dw, ch / dh
        supx, supy = sup * max(sx, 1.0), sup * max(sy, 1.0)
        taps = max(taps, int(math.floor(2 * supx)) + 2, int(math.floor(2 * supy)) + 2)
        rcap = max(rcap, int(math.ceil((patch - 1) * sy + 2 * supy)) + 2)   # rows < (patch-1)s + 2 sup + 1
        cwcap = max(cwcap, cw)
    if taps > 16:
        return None
    tm = 8 if taps <= 8 else 16
    r16 = lambda n: (n + 15) // 16 * 16  # noqa: E731
    ra = r16(OW * (tm + 3) * 4) + rcap * cwcap * 4                        # csrc/image.hip image_prep_band_lds
    lds = r16(patch * (tm + 3) * 4) + r16(max(ra, (OW // patch) * kpad * 2)) + rcap * OW * 4 + 16
    return (rcap, cwcap, taps) if lds <= _PREP_BAND_LDS else None


def image_prep(
    images: Sequence[torch.Tensor] | torch.Tensor,
    out_hw: tuple[int, int],
    mean=(0.0, 0.0, 0.0),
    std=(1.0, 1.0, 1.0),
    scale: float = 1.0 / 255.0,
    filter: str = "pil_bicubic",
    layout: str = "nchw",
    patch: int = 0,
    kpad: int = 0,
    swap_rb: bool = False,
    pad: float = 0.0,
    geoms: Optional[Sequence[ImageGeom]] = None,
    out_dtype: torch.dtype = torch.float32,
    device=None,
    src: Optional[torch.Tensor] = None,
    center_crop: bool = False,
) -> torch.Tensor:
    """Resize/pad/normalise a batch of uint8 HWC RGB images into one tensor.

    ``center_crop``: shortest side -> OH then the centre OH x OW window (open_clip's
    transform, :meth:`ImageGeom.center_crop`) instead of squashing to (OH, OW).

    ``src``: the images already on the device as one flat uint8 tensor (PinnedUploader);
    ``geoms`` then carry the offsets into it and ``images`` only provide the shapes.

    ``images`` is a list of [H, W, 3] uint8 tensors (ragged sizes allowed) or a
    [B, H, W, 3] uint8 tensor.  Output value = ((px * scale) - mean) / std with the
    channel order optionally reversed (``swap_rb``).
    """
    if isinstance(images, torch.Tensor) and images.dim() == 4:
        imgs = list(images.unbind(0))
        flat_src = images.reshape(-1)
    else:
        imgs = list(images)
        flat_src = None
    B = len(imgs)
    OH, OW = out_hw
    device = device or imgs[0].device
    if geoms is None:
        off = 0
        geoms = []
        for im in imgs:
            if center_crop:
                assert OH == OW, "center_crop needs a square output"
                geoms.append(ImageGeom.center_crop(im.shape[0], im.shape[1], off, OH))
            else:
                geoms.append(ImageGeom.resize(im.shape[0], im.shape[1], off, OH, OW))
            off += im.numel()
    lay = LAYOUTS[layout]
    filt = FILTERS[filter]
    if lay == 2:
        P = (OH // patch) * (OW // patch)
        kpad = kpad or 3 * patch * patch
        out = torch.empty((B * P, kpad), device=device, dtype=out_dtype)
    elif lay == 0:
        out = torch.empty((B, 3, OH, OW), device=device, dtype=out_dtype)
    elif lay == 3:
        out = torch.empty((B, OH, OW, 8), device=device, dtype=out_dtype)
    else:
        out = torch.empty((B, OH, OW, 3), device=device, dtype=out_dtype)
    if torch.device(device).type == "cuda":
        if src is None:
            src = flat_src if flat_src is not None else torch.cat([im.reshape(-1) for im in imgs])
            src = src.to(device, non_blocking=True)
        g = h2d([gg.row() for gg in geoms], device, torch.long)
        band = _prep_band_bounds(geoms, filt, lay, patch, kpad, OW, out_dtype, pad)
        if band is not None:          # ViT patch rows, PIL filters: one fused launch (csrc/image.hip)
            hip_ops().image_prep_band(src, g, out, OH, OW, filt, bool(swap_rb), [float(m) for m in mean],
                                      [float(s) for s in std], float(scale), float(pad), int(patch), int(kpad),
                                      band[0], band[1], band[2])
            return out
        max_ch = max(gg.ch for gg in geoms)
        max_dw = max(gg.dw for gg in geoms)
        tmp = torch.empty((B, max_ch, max_dw, 3), device=device, dtype=torch.float32)
        hip_ops().image_prep(src, g, out, tmp, OH, OW, filt, bool(swap_rb), [float(m) for m in mean],
                             [float(s) for s in std], float(scale), float(pad), lay, int(patch), int(kpad),
                             int(max_ch), int(max_dw))
        return out
    # CPU reference
    outs = []
    for im, gg in zip(imgs, geoms):
        canvas = torch.full((gg.ch, gg.cw, 3), float(pad))
        canvas[gg.oy:gg.oy + gg.ih, gg.ox:gg.ox + gg.iw] = im.float()
        t = _ref_resample_axis(canvas, gg.dw, 1, filt)
        t = _ref_resample_axis(t, gg.dh, 0, filt)
        full = torch.full((OH, OW, 3), float(pad))
        y0, x0 = max(gg.dy, 0), max(gg.dx, 0)                      # crop geometries: dx, dy < 0
        y1, x1 = min(gg.dy + gg.dh, OH), min(gg.dx + gg.dw, OW)
        full[y0:y1, x0:x1] = t[y0 - gg.dy:y1 - gg.dy, x0 - gg.dx:x1 - gg.dx]
        if swap_rb:
            full = full.flip(-1)
        v = (full * scale - torch.tensor(mean, dtype=torch.float32)) / torch.tensor(std, dtype=torch.float32)
        outs.append(v)
    v = torch.stack(outs)  # B, OH, OW, 3
    if lay == 0:
        out.copy_(v.permute(0, 3, 1, 2).to(out_dtype))
    elif lay == 1:
        out.copy_(v.to(out_dtype))
    elif lay == 3:
        out.zero_()
        out[..., :3] = v.to(out_dtype)
    else:
        p = patch
        gh, gw = OH // p, OW // p
        x = v.permute(0, 3, 1, 2).reshape(B, 3, gh, p, gw, p).permute(0, 2, 4, 1, 3, 5).reshape(B * gh * gw, 3 * p * p)
        out.zero_()
        out[:, : 3 * p * p] = x.to(out_dtype)
    return out
