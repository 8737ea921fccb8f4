"""CLIP model family (OpenAI / OpenCLIP / HF CLIP naming, BioCLIP-2, ViT-B/L).

The towers are written directly against :mod:`lumen_amd.ops`, i.e. every hot op
is one hand-written gfx950 kernel on the GPU:

  image_prep (resize+normalise+im2col)  -> patch GEMM (epilogue: +pos-emb, row
  scatter into the token buffer) -> cls_fill -> ln_pre -> L x [LN -> QKV GEMM ->
  fused attention (reads the packed QKV in place) -> out-proj GEMM (+bias
  +residual in place) -> LN -> fc1 GEMM (+bias, GELU/QuickGELU) -> fc2 GEMM (+bias
  +residual)] -> ln_post on CLS rows (row gather) -> projection GEMM (fp32 out) ->
  L2 normalise.

Reference behaviour reproduced: image embedding = normalised projection of the
CLS token (packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:466-495,
torch_backend.py:520-535); text embedding pools the EOT token (argmax id) for
OpenAI-style towers (torch_backend.py:340-393).
"""
from __future__ import annotations

import logging
import math
import os
from dataclasses import dataclass, field, asdict
from typing import Optional

import torch
from torch import nn

from .. import ops
from .fastvit import FASTVIT_PRESETS, FastViTConfig, FastViTTower


@dataclass
class VisionConfig:
    image_size: int = 224
    patch_size: int = 14
    width: int = 1024
    layers: int = 24
    heads: int = 16
    mlp_ratio: float = 4.0
    act: str = "quick_gelu"
    ln_eps: float = 1e-5


@dataclass
class TextConfig:
    context_length: int = 77
    vocab_size: int = 49408
    width: int = 768
    layers: int = 12
    heads: int = 12
    mlp_ratio: float = 4.0
    act: str = "quick_gelu"
    ln_eps: float = 1e-5
    eot_token_id: Optional[int] = None  # None -> argmax(ids) pooling (OpenAI BPE: EOT is the max id)


@dataclass
class BertConfig:
    """Chinese-CLIP text tower (BERT / RoBERTa-wwm-ext, post-LN, CLS pooling)."""
    vocab_size: int = 21128
    width: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    ln_eps: float = 1e-12
    act: str = "gelu"
    context_length: int = 52
    pad_token_id: int = 0


@dataclass
class CLIPConfig:
    embed_dim: int = 768
    vision: VisionConfig = field(default_factory=VisionConfig)
    text: TextConfig = field(default_factory=TextConfig)
    image_mean: tuple = (0.48145466, 0.4578275, 0.40821073)
    image_std: tuple = (0.26862954, 0.26130258, 0.27577711)
    logit_scale: float = math.log(100.0)
    text_arch: str = "openai"                 # "openai" causal EOT-pooled | "bert" (Chinese-CLIP)
    bert: Optional[BertConfig] = None
    vision_arch: str = "vit"                  # "vit" | "fastvit" (MobileCLIP / MobileCLIP2 MCi towers)
    fastvit: Optional[FastViTConfig] = None

    def to_dict(self):
        return asdict(self)

    @property
    def context_length(self) -> int:
        return self.bert.context_length if self.text_arch == "bert" else self.text.context_length

    @staticmethod
    def from_dict(d: dict) -> "CLIPConfig":
        v = VisionConfig(**d.get("vision", {}))
        t = TextConfig(**d.get("text", {}))
        rest = {k: d[k] for k in ("embed_dim", "image_mean", "image_std", "logit_scale", "text_arch", "vision_arch")
                if k in d}
        if "image_mean" in rest:
            rest["image_mean"] = tuple(rest["image_mean"])
        if "image_std" in rest:
            rest["image_std"] = tuple(rest["image_std"])
        if d.get("bert"):
            rest["bert"] = BertConfig(**d["bert"])
        if d.get("fastvit"):
            rest["fastvit"] = FastViTConfig.from_dict(d["fastvit"])
        return CLIPConfig(vision=v, text=t, **rest)


PRESETS = {
    # OpenAI ViT-L/14 (also the BioCLIP-2 geometry), 768-d embeddings
    "ViT-L-14": CLIPConfig(),
    "ViT-B-32": CLIPConfig(
        embed_dim=512,
        vision=VisionConfig(patch_size=32, width=768, layers=12, heads=12),
        text=TextConfig(width=512, layers=12, heads=8),
    ),
    "ViT-B-16": CLIPConfig(
        embed_dim=512,
        vision=VisionConfig(patch_size=16, width=768, layers=12, heads=12),
        text=TextConfig(width=512, layers=12, heads=8),
    ),
    "ViT-L-14-336": CLIPConfig(vision=VisionConfig(image_size=336)),
    # Chinese-CLIP (reference default general CLIP: CN-CLIP_ViT-B-16 / CN-CLIP_ViT-L-14),
    # RoBERTa-wwm-ext-base-chinese text tower, 52-token context, CLS pooling
    "CN-ViT-B-16": CLIPConfig(
        embed_dim=512,
        vision=VisionConfig(patch_size=16, width=768, layers=12, heads=12),
        text_arch="bert", bert=BertConfig(),
    ),
    "CN-ViT-L-14": CLIPConfig(text_arch="bert", bert=BertConfig()),
    "cn-tiny": CLIPConfig(
        embed_dim=64,
        vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=2),
        text=TextConfig(context_length=16, vocab_size=512, width=64, layers=2, heads=2),
        text_arch="bert", bert=BertConfig(vocab_size=512, width=64, layers=2, heads=2, intermediate=128,
                                          max_position=64, context_length=16),
    ),
    # MobileCLIP2 (reference default general CLIP for region "other"): MCi image towers
    # (FastViT, reparameterised) + OpenAI-style text transformer; no pixel normalisation
    "MobileCLIP2-S2": CLIPConfig(
        embed_dim=512, vision_arch="fastvit", fastvit=FASTVIT_PRESETS["mci2"],
        vision=VisionConfig(image_size=256), text=TextConfig(width=512, layers=12, heads=8, act="gelu"),
        image_mean=(0.0, 0.0, 0.0), image_std=(1.0, 1.0, 1.0),
    ),
    "MobileCLIP2-S4": CLIPConfig(
        embed_dim=768, vision_arch="fastvit", fastvit=FASTVIT_PRESETS["mci4"],
        vision=VisionConfig(image_size=256), text=TextConfig(width=768, layers=12, heads=12, act="gelu"),
        image_mean=(0.0, 0.0, 0.0), image_std=(1.0, 1.0, 1.0),
    ),
    "mobileclip-tiny": CLIPConfig(
        embed_dim=64, vision_arch="fastvit", fastvit=FASTVIT_PRESETS["tiny"],
        vision=VisionConfig(image_size=64, patch_size=8, width=64, layers=1, heads=2),
        text=TextConfig(context_length=16, vocab_size=512, width=64, layers=2, heads=2, act="gelu"),
        image_mean=(0.0, 0.0, 0.0), image_std=(1.0, 1.0, 1.0),
    ),
    # tiny geometry used by CPU tests and synthetic model directories
    "tiny": CLIPConfig(
        embed_dim=64,
        vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=2),
        text=TextConfig(context_length=16, vocab_size=512, width=64, layers=2, heads=2),
    ),
}


def _pad64(k: int) -> int:
    return (k + 63) // 64 * 64


class _Block(nn.Module):
    """Pre-LN transformer block parameters (weights stored [out, in], bf16)."""

    def __init__(self, width: int, mlp: int, dtype, device):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.ln1_w = nn.Parameter(torch.ones(width, **kw), requires_grad=False)
        self.ln1_b = nn.Parameter(torch.zeros(width, **kw), requires_grad=False)
        self.qkv_w = nn.Parameter(torch.empty(3 * width, width, **kw), requires_grad=False)
        self.qkv_b = nn.Parameter(torch.zeros(3 * width, **kw), requires_grad=False)
        self.out_w = nn.Parameter(torch.empty(width, width, **kw), requires_grad=False)
        self.out_b = nn.Parameter(torch.zeros(width, **kw), requires_grad=False)
        self.ln2_w = nn.Parameter(torch.ones(width, **kw), requires_grad=False)
        self.ln2_b = nn.Parameter(torch.zeros(width, **kw), requires_grad=False)
        self.fc1_w = nn.Parameter(torch.empty(mlp, width, **kw), requires_grad=False)
        self.fc1_b = nn.Parameter(torch.zeros(mlp, **kw), requires_grad=False)
        self.fc2_w = nn.Parameter(torch.empty(width, mlp, **kw), requires_grad=False)
        self.fc2_b = nn.Parameter(torch.zeros(width, **kw), requires_grad=False)

    def lnf(self):
        """GPU form with both LayerNorms folded into the projections that consume them
        (ops.ln_fold_weights): (qkv w', qkv col_aff, fc1 w', fc1 col_aff).  Rebuilt whenever a
        parameter it derives from is rewritten (weight loads bump the tensors' versions)."""
        src = (self.ln1_w, self.ln1_b, self.qkv_w, self.qkv_b, self.ln2_w, self.ln2_b, self.fc1_w, self.fc1_b)
        key = tuple((p.data_ptr(), p._version) for p in src)
        if getattr(self, "_lnf_key", None) != key:
            with torch.no_grad():
                qw, qa = ops.ln_fold_weights(self.qkv_w, self.qkv_b, self.ln1_w, self.ln1_b)
                fw, fa = ops.ln_fold_weights(self.fc1_w, self.fc1_b, self.ln2_w, self.ln2_b)
            self._lnf_cache = (qw, qa, fw, fa)
            self._lnf_key = key
        return self._lnf_cache

    def mx_weights(self) -> dict:
        """W8A8 form for the MX tower chain (run_blocks_mx): OCP e4m3 weights with per-output-channel
        scales -- qkv / fc1 with their LayerNorms folded in (:meth:`lnf`), colsum(w') taken over the
        DEQUANTISED fp8 rows the GEMM multiplies with (the fold subtracts mean * colsum exactly) --
        plus out / fc2 as they are.  Cached like :meth:`lnf`."""
        qw, qa, fw, fa = self.lnf()
        key = getattr(self, "_lnf_key", None)
        if getattr(self, "_mx_key", None) != key:
            with torch.no_grad():
                q8, qs = ops.quantize_fp8_rows(qw)
                f8, fs = ops.quantize_fp8_rows(fw)
                qa2, fa2 = qa.clone(), fa.clone()
                qa2[0] = (q8.float() * qs[:, None]).sum(1)
                fa2[0] = (f8.float() * fs[:, None]).sum(1)
                o8, os_ = ops.quantize_fp8_rows(self.out_w)
                c8, cs = ops.quantize_fp8_rows(self.fc2_w)
            self._mx_cache = dict(qkv=(q8, qs, qa2), fc1=(f8, fs, fa2), out=(o8, os_), fc2=(c8, cs))
            self._mx_key = key
        return self._mx_cache

    def tp_shard(self, rank: int, world: int, heads: int, mx: bool = False) -> dict:
        """This rank's slice of the block for tensor-parallel blocks (:func:`run_blocks_tp`):
        column-parallel qkv (the rank's heads of q, k and v) and fc1 (its 1/world of the MLP
        columns), row-parallel out / fc2 (the matching input columns; the biases on rank 0 only).
        GPU: from the LayerNorm-folded weights (:meth:`lnf`) or, ``mx``, their W8A8 form
        (:meth:`mx_weights`, per-output-row scales: a column slice keeps its rows' scales).
        Cached per (rank, world, form) until a source weight changes."""
        gpu = self.qkv_w.is_cuda
        src_key = getattr(self, "_lnf_key", None) if gpu else None
        if gpu:
            self.lnf()
            src_key = self._lnf_key
        key = (rank, world, heads, mx, gpu, src_key,
               tuple((p.data_ptr(), p._version) for p in (self.qkv_w, self.out_w, self.fc1_w, self.fc2_w)))
        cache = getattr(self, "_tp_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        W = self.qkv_w.shape[1]
        mlp = self.fc1_w.shape[0]
        assert heads % world == 0 and mlp % world == 0, "TP tower: heads / MLP width not divisible"
        wr, mr = W // world, mlp // world
        rows = torch.cat([torch.arange(j * W + rank * wr, j * W + (rank + 1) * wr) for j in range(3)]).to(self.qkv_w.device)
        fcr = slice(rank * mr, (rank + 1) * mr)
        d: dict = {}
        with torch.no_grad():
            if gpu:
                qw, qa, fw, fa = self.lnf()
                if mx:
                    m = self.mx_weights()
                    d["qkv"] = (m["qkv"][0].index_select(0, rows).contiguous(), m["qkv"][1][rows].contiguous(),
                                m["qkv"][2][:, rows].contiguous())
                    d["fc1"] = (m["fc1"][0][fcr].contiguous(), m["fc1"][1][fcr].contiguous(),
                                m["fc1"][2][:, fcr].contiguous())
                    d["out"] = (m["out"][0][:, rank * wr:(rank + 1) * wr].contiguous(), m["out"][1])
                    d["fc2"] = (m["fc2"][0][:, fcr].contiguous(), m["fc2"][1])
                else:
                    d["qkv"] = (qw.index_select(0, rows).contiguous(), qa[:, rows].contiguous())
                    d["fc1"] = (fw[fcr].contiguous(), fa[:, fcr].contiguous())
            else:
                d["qkv"] = (self.qkv_w.index_select(0, rows.cpu()).contiguous(), self.qkv_b[rows.cpu()].contiguous())
                d["fc1"] = (self.fc1_w[fcr].contiguous(), self.fc1_b[fcr].contiguous())
            if not (gpu and mx):
                d["out_w"] = self.out_w[:, rank * wr:(rank + 1) * wr].contiguous()
                d["fc2_w"] = self.fc2_w[:, fcr].contiguous()
        d["out_b"] = self.out_b if rank == 0 else None
        d["fc2_b"] = self.fc2_b if rank == 0 else None
        self._tp_cache = (key, d)
        return d

    def random_init(self, gen: torch.Generator, layers: int):
        w = self.qkv_w.shape[1]
        attn_std = w ** -0.5
        proj_std = (w ** -0.5) * ((2 * layers) ** -0.5)
        fc_std = (2 * w) ** -0.5
        for p, s in ((self.qkv_w, attn_std), (self.out_w, proj_std), (self.fc1_w, fc_std), (self.fc2_w, proj_std)):
            p.data.copy_(torch.randn(p.shape, generator=gen) * s)


def _block_steps(x: torch.Tensor, blocks, B: int, S: int, heads: int, act: str, eps: float,
                 causal: bool = False, kv_len: Optional[torch.Tensor] = None, tile: int = -1,
                 res_tile: Optional[int] = None):
    """Pre-LN blocks over the flat residual stream x [B*S, W] (updated in place), one
    ``yield`` per block so several micro-batches can be issued layer-interleaved."""
    T, W = x.shape
    D = W // heads
    o = torch.empty_like(x)
    # GPU: both LayerNorms are folded into qkv / fc1 (ops.linear_lnf): a row-statistics pass writes
    # 8 bytes per row instead of a normalised copy of x, and the GEMMs read the residual stream
    fold = x.is_cuda and _LN_FOLD
    if fold:
        st = torch.empty((T, 2), device=x.device, dtype=torch.float32)
    else:
        h = torch.empty_like(x)
    # the out-proj / fc2 residual is added in the GEMM epilogue (the MFMA GEMM adds the prefetched
    # residual rows before its single bf16 rounding); a separate add + LayerNorm pass measured
    # 5837 vs 5951 img/s on ViT-L/14 b512 (profiles/r2_bench_resid_paths_v1.txt)
    rt = tile if res_tile is None else res_tile
    for i, blk in enumerate(blocks):
        if fold:
            qw, qa, fw, fa = blk.lnf()
            ops.ln_row_stats(x, eps, out=st)
            qkv = ops.linear_lnf(x, qw, qa, st, tile=tile)
        else:
            ops.layer_norm(x, blk.ln1_w, blk.ln1_b, eps, out=h)
            qkv = ops.linear(h, blk.qkv_w, blk.qkv_b, tile=tile)
        q5 = qkv.view(B, S, 3, heads, D)
        ops.attention(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], causal=causal, kv_len=kv_len,
                      out=o.view(B, S, heads, D))
        del qkv, q5
        ops.linear(o, blk.out_w, blk.out_b, residual=x, out=x, tile=rt)
        if fold:
            ops.ln_row_stats(x, eps, out=st)
            f = ops.linear_lnf(x, fw, fa, st, act=act, tile=tile)
        else:
            ops.layer_norm(x, blk.ln2_w, blk.ln2_b, eps, out=h)
            f = ops.linear(h, blk.fc1_w, blk.fc1_b, act=act, tile=tile)
        ops.linear(f, blk.fc2_w, blk.fc2_b, residual=x, out=x, tile=rt)
        del f
        yield i


def run_blocks_mx(x: torch.Tensor, blocks, B: int, S: int, heads: int, act: str, eps: float) -> torch.Tensor:
    """W8A8 pre-LN blocks (GPU, width and MLP width % 128 == 0, head dim 64 / 128), every GEMM
    operand an MX fp8 tensor produced by the kernel before it -- 7 launches per block:

      LN stats + MX copy of x  ->  qkv gemm_mx (LN folded)  ->  attention (MX O)
      ->  out gemm_mx (+ bias + residual)  ->  LN stats + MX copy  ->  fc1 gemm_mx (LN folded + act,
      MX output only)  ->  fc2 gemm_mx (+ bias + residual)

    against 8 for the bf16 blocks (two row-stat passes, four bf16 GEMMs, attention and fc2's split-K
    reduce), at half the K-step bytes per GEMM.  Weights: _Block.mx_weights."""
    T, W = x.shape
    D = W // heads
    dev = x.device
    f8, u8 = torch.float8_e4m3fn, torch.uint8
    mlp = blocks[0].fc1_w.shape[0]
    st = torch.empty((T, 2), device=dev, dtype=torch.float32)
    x8 = torch.empty((T, W), device=dev, dtype=f8)
    xs = torch.empty((W // 128, T, 4), device=dev, dtype=u8)
    a8 = torch.empty((T, W), device=dev, dtype=f8)
    as_ = torch.empty((W // 128, T, 4), device=dev, dtype=u8)
    g8 = torch.empty((T, mlp), device=dev, dtype=f8)
    gs = torch.empty((mlp // 128, T, 4), device=dev, dtype=u8)
    qkv = torch.empty((T, 3 * W), device=dev, dtype=x.dtype)
    for blk in blocks:
        w = blk.mx_weights()
        ops.ln_row_stats(x, eps, out=st, q_out=(x8, xs))
        ops.linear_mx(x8, xs, w["qkv"][0], w["qkv"][1], out=qkv, row_aff=st, col_aff=w["qkv"][2])
        q5 = qkv.view(B, S, 3, heads, D)
        ops.attention_mx(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], q_out=(a8, as_))
        ops.linear_mx(a8, as_, w["out"][0], w["out"][1], bias=blk.out_b, residual=x, out=x)
        ops.ln_row_stats(x, eps, out=st, q_out=(x8, xs))
        ops.linear_mx(x8, xs, w["fc1"][0], w["fc1"][1], row_aff=st, col_aff=w["fc1"][2], act=act, q_out=(g8, gs),
                      write_out=False)
        ops.linear_mx(g8, gs, w["fc2"][0], w["fc2"][1], bias=blk.fc2_b, residual=x, out=x)
    return x


def run_blocks_tp(x: torch.Tensor, blocks, B: int, S: int, heads: int, act: str, eps: float, rank: int,
                  world: int, all_reduce, mx: bool = False) -> torch.Tensor:
    """Tensor-parallel pre-LN blocks (Megatron split): every rank holds the whole residual stream
    x [B*S, W] and runs its heads of attention and its 1/world of the MLP; the row-parallel out /
    fc2 partials are summed by ``all_reduce`` (in place; the IPC one- / two-shot kernels under a TP
    group) -- 2 all-reduces per block.  A single image's tower then runs on every GPU of the TP group
    instead of on rank 0 alone, and the features need no broadcast (VLM.build_prefill).  ``mx``: the
    W8A8 MX chain of :func:`run_blocks_mx` on the shards (GPU; W / world a multiple of 128)."""
    T, W = x.shape
    hr = heads // world
    D = W // heads
    dev = x.device
    gpu = x.is_cuda
    if gpu:
        st = torch.empty((T, 2), device=dev, dtype=torch.float32)
    else:
        h = torch.empty_like(x)
    o = torch.empty((B, S, hr, D), device=dev, dtype=x.dtype)
    if mx:
        f8, u8 = torch.float8_e4m3fn, torch.uint8
        mlp_r = blocks[0].fc1_w.shape[0] // world
        x8 = torch.empty((T, W), device=dev, dtype=f8)
        xs = torch.empty((W // 128, T, 4), device=dev, dtype=u8)
        a8 = torch.empty((T, hr * D), device=dev, dtype=f8)
        as_ = torch.empty((hr * D // 128, T, 4), device=dev, dtype=u8)
        g8 = torch.empty((T, mlp_r), device=dev, dtype=f8)
        gs = torch.empty((mlp_r // 128, T, 4), device=dev, dtype=u8)
    for blk in blocks:
        d = blk.tp_shard(rank, world, heads, mx=mx)
        if mx:
            ops.ln_row_stats(x, eps, out=st, q_out=(x8, xs))
            qkv = ops.linear_mx(x8, xs, d["qkv"][0], d["qkv"][1], row_aff=st, col_aff=d["qkv"][2])
            q5 = qkv.view(B, S, 3, hr, D)
            ops.attention_mx(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], q_out=(a8, as_))
            part = ops.linear_mx(a8, as_, d["out"][0], d["out"][1], bias=d["out_b"])
        else:
            if gpu:
                ops.ln_row_stats(x, eps, out=st)
                qkv = ops.linear_lnf(x, d["qkv"][0], d["qkv"][1], st)
            else:
                ops.layer_norm(x, blk.ln1_w, blk.ln1_b, eps, out=h)
                qkv = ops.linear(h, d["qkv"][0], d["qkv"][1])
            q5 = qkv.view(B, S, 3, hr, D)
            ops.attention(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], out=o)
            part = ops.linear(o.view(T, hr * D), d["out_w"], d["out_b"])
        x.add_(all_reduce(part))
        if mx:
            ops.ln_row_stats(x, eps, out=st, q_out=(x8, xs))
            ops.linear_mx(x8, xs, d["fc1"][0], d["fc1"][1], row_aff=st, col_aff=d["fc1"][2], act=act,
                          q_out=(g8, gs), write_out=False)
            part = ops.linear_mx(g8, gs, d["fc2"][0], d["fc2"][1], bias=d["fc2_b"])
        else:
            if gpu:
                ops.ln_row_stats(x, eps, out=st)
                f = ops.linear_lnf(x, d["fc1"][0], d["fc1"][1], st, act=act)
            else:
                ops.layer_norm(x, blk.ln2_w, blk.ln2_b, eps, out=h)
                f = ops.linear(h, d["fc1"][0], d["fc1"][1], act=act)
            part = ops.linear(f, d["fc2_w"], d["fc2_b"])
        x.add_(all_reduce(part))
        del qkv, part
    return x


def tp_blocks_ok(x: torch.Tensor, blocks, heads: int, world: int, mx: bool) -> bool:
    """Whether :func:`run_blocks_tp` can split these blocks ``world`` ways."""
    if not blocks:
        return False
    W = x.shape[1]
    mlp = blocks[0].fc1_w.shape[0]
    if heads % world or mlp % world or (W // world) % 64 or (mlp // world) % 64:
        return False
    return not mx or (x.is_cuda and (W // world) % 128 == 0 and (mlp // world) % 128 == 0 and W // heads in (64, 128))


def mx_blocks_ok(x: torch.Tensor, blocks, heads: int) -> bool:
    W = x.shape[1]
    return (x.is_cuda and len(blocks) > 0 and W % 128 == 0 and blocks[0].fc1_w.shape[0] % 128 == 0
            and W // heads in (64, 128))


def run_blocks(x: torch.Tensor, blocks, B: int, S: int, heads: int, act: str, eps: float,
               causal: bool = False, kv_len: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Run pre-LN blocks over the flat residual stream x [B*S, W] (updated in place)."""
    for _ in _block_steps(x, blocks, B, S, heads, act, eps, causal, kv_len):
        pass
    return x


# Micro-batched tower (large image batches on the GPU): the batch is cut into LUMEN_VIT_MICRO
# row ranges, each issued on its own HIP stream, layer-interleaved.  A 256x256-tile GEMM over
# M = B*257 rows ends on a nearly empty round of tiles (ViT-L/14 b512: 514 row tiles); with two
# streams the other micro-batch's kernels fill those CUs, so the GEMMs run without the split-K
# tail pass (tile code 1609: ping-pong 256x256, non-persistent, no tail split) and attention /
# LayerNorm of one half overlap GEMM tails of the other.
_VIT_MICRO = int(os.environ.get("LUMEN_VIT_MICRO", "2"))
# (r5's per-bucket hipGraph replay of serving-sized batches lost its serving A/B, 2,897 vs 3,052 img/s
# eager -- the small-batch tower is GPU-bound and the graph's static buffers serialise the engine's two
# batch loops, profiles/r5_clip_graph_serve_v1.txt -- and was removed in r6)
log = logging.getLogger(__name__)
_LN_FOLD = True   # GPU blocks: LayerNorms folded into qkv / fc1 (see _block_steps)
# (r5's LayerNorm partials from the residual GEMMs -- no gain: the row-statistics pass already hides behind
# the other stream's GEMMs, 6248 vs 6251-6268 img/s, profiles/r5_gemm_pp_ds_v1.txt -- were removed in r6)
# ping-pong 256x256, 2 phases per K-tile + priority, no tail split (r2: group_m 2 = 1629 vs 1609 / 1689:
# 6209-6222 vs 6203-6204 / 6129-6130 img/s, profiles/r2_vit_micro_streams_v1.txt); r5: the direct-store
# epilogue (1849: 6287-6340 vs 1629 6225-6227 img/s same box, the persistent forms lose in the 2-stream
# tower), group_m 3 (1839: 6388.6 / 6390.6 vs 1849 6336.6 / 6354.6 and 1629 6383.4 / 6380.4 on a later box),
# profiles/r5_gemm_pp_ds_v1.txt
_VIT_MICRO_TILE = int(os.environ.get("LUMEN_VIT_TILE", "1839"))
_VIT_MICRO_RES_TILE = _VIT_MICRO_TILE
# text tower (B x 77 rows): micro-batched with the auto tile choice once it has this many rows per
# half (b512 x 77: 50.4-50.6k -> 56.2-56.4k texts/s, profiles/r2_vit_micro_streams_v1.txt)
_TEXT_MICRO_MIN_ROWS = 16384
# per micro-batch rows: from 65536 rows (every GEMM >= 512 tiles of 256x256) on the fixed ping-pong tiles, below
# that (serving-sized batches) on the auto tile choice (128x128 LDS-DMA tiles): ViT-L/14 at 40 images 3,784 vs
# 3,116 img/s on one stream, at 64 images 4,127 vs 4,080 (profiles/r5_clip_graph_serve_v1.txt)
_VIT_MICRO_MIN_ROWS = int(os.environ.get("LUMEN_VIT_MICRO_MIN_ROWS", "4096"))
_VIT_MICRO_PP_ROWS = 65536
_MICRO_STREAMS: dict = {}


def _micro_streams(dev: torch.device, n: int):
    key = (dev.index, n)
    if key not in _MICRO_STREAMS:
        _MICRO_STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return _MICRO_STREAMS[key]


def run_blocks_micro(x: torch.Tensor, blocks, B: int, S: int, heads: int, act: str, eps: float,
                     causal: bool = False, min_rows: Optional[int] = None, tile: Optional[int] = None,
                     res_tile: Optional[int] = None, streams: Optional[list] = None) -> torch.Tensor:
    """run_blocks over micro-batches on separate streams (falls back to run_blocks when the
    batch is too small to split or x is on the CPU).  ``streams``: the micro-batch streams to use
    (a graph capture passes its own private ones: the shared module-level streams may at the same
    time carry another thread's eager tower, whose kernels would join the capture -- ADVICE r5)."""
    n = len(streams) if streams else _VIT_MICRO
    min_rows = _VIT_MICRO_MIN_ROWS if min_rows is None else min_rows
    if not x.is_cuda or n <= 1 or B < n or (B // n) * S < min_rows:
        return run_blocks(x, blocks, B, S, heads, act, eps, causal=causal)
    small = (B // n) * S < _VIT_MICRO_PP_ROWS
    tile = (-1 if small else _VIT_MICRO_TILE) if tile is None else tile
    res_tile = (-1 if small else _VIT_MICRO_RES_TILE) if res_tile is None else res_tile
    cur = torch.cuda.current_stream(x.device)
    if _LN_FOLD:
        # the LN-folded weights are built lazily and cached on the block: build them HERE, on the caller's
        # stream that every micro-batch stream waits for -- built inside the generators, the first
        # micro-batch's stream would compute them while the second's GEMMs already read the cache
        for blk in blocks:
            blk.lnf()
    streams = streams or _micro_streams(x.device, n)
    bounds = [B * i // n for i in range(n + 1)]
    gens = []
    for i, st in enumerate(streams):
        st.wait_stream(cur)
        b0, b1 = bounds[i], bounds[i + 1]
        with torch.cuda.stream(st):
            gens.append(_block_steps(x[b0 * S:b1 * S], blocks, b1 - b0, S, heads, act, eps, causal=causal,
                                     tile=tile, res_tile=res_tile))
    live = list(zip(gens, streams))
    while live:
        nxt = []
        for g, st in live:
            with torch.cuda.stream(st):
                if next(g, None) is not None:
                    nxt.append((g, st))
        live = nxt
    for st in streams:             # join: x (allocated on cur) is only freed after this point on cur
        cur.wait_stream(st)
    return x


class VisionTower(nn.Module):
    def __init__(self, cfg: VisionConfig, embed_dim: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.embed_dim = embed_dim
        kw = dict(dtype=dtype, device=device)
        p = cfg.patch_size
        self.grid = cfg.image_size // p
        self.num_patches = self.grid * self.grid
        self.seq = self.num_patches + 1
        self.kdim = 3 * p * p
        self.kpad = _pad64(self.kdim)
        W = cfg.width
        self.patch_w = nn.Parameter(torch.zeros(W, self.kpad, **kw), requires_grad=False)
        self.class_emb = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.pos_emb = nn.Parameter(torch.zeros(self.seq, W, **kw), requires_grad=False)
        self.ln_pre_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.ln_pre_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.blocks = nn.ModuleList([_Block(W, int(W * cfg.mlp_ratio), dtype, device) for _ in range(cfg.layers)])
        self.ln_post_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.ln_post_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.proj_w = nn.Parameter(torch.zeros(embed_dim, W, **kw), requires_grad=False)  # [E, W]

    def random_init(self, gen: torch.Generator):
        W = self.cfg.width
        s = W ** -0.5
        w = torch.randn(W, self.kdim, generator=gen) * (self.kdim ** -0.5)
        self.patch_w.data.zero_()
        self.patch_w.data[:, : self.kdim] = w.to(self.patch_w.dtype)
        self.class_emb.data.copy_(torch.randn(W, generator=gen) * s)
        self.pos_emb.data.copy_(torch.randn(self.seq, W, generator=gen) * 0.01)
        for b in self.blocks:
            b.random_init(gen, self.cfg.layers)
        self.proj_w.data.copy_(torch.randn(self.embed_dim, W, generator=gen) * s)

    @torch.no_grad()
    def forward_patches(self, patches: torch.Tensor, B: int) -> torch.Tensor:
        """patches [B*P, kpad] (bf16) -> L2-normalised fp32 embeddings [B, E]."""
        return self._forward_patches(patches, B)

    def _forward_patches(self, patches: torch.Tensor, B: int) -> torch.Tensor:
        cfg = self.cfg
        S, P, W = self.seq, self.num_patches, cfg.width
        dev, dt = patches.device, self.patch_w.dtype
        x = torch.empty((B * S, W), device=dev, dtype=dt)
        # patch GEMM: row m = b*P + p -> token row b*S + 1 + p, + pos_emb[1 + p]
        ops.linear(patches, self.patch_w, table=self.pos_emb, table_period=P, table_offset=1, out=x,
                   out_group=P, out_group_stride=S, out_row_offset=1)
        ops.cls_fill(x, self.class_emb, self.pos_emb, S)
        ops.layer_norm(x, self.ln_pre_w, self.ln_pre_b, cfg.ln_eps, out=x)
        run_blocks_micro(x, self.blocks, B, S, cfg.heads, cfg.act, cfg.ln_eps)
        cls_rows = torch.arange(B, device=dev, dtype=torch.long) * S
        pooled = ops.layer_norm(x, self.ln_post_w, self.ln_post_b, cfg.ln_eps, row_idx=cls_rows)
        emb = ops.linear(pooled, self.proj_w, out_dtype=torch.float32)
        return ops.l2_normalize_(emb)

    @torch.no_grad()
    def forward_features(self, patches: torch.Tensor, B: int, layer: int = -2, drop_cls: bool = True,
                         tp: Optional[tuple] = None) -> torch.Tensor:
        """Hidden states after block ``layer`` (LLaVA ``mm_vision_select_layer``; -1 = last,
        -2 = penultimate) -> [B, P(+1), W] bf16 patch features (CLS dropped).  ``tp`` = (rank, world,
        all_reduce): the blocks run tensor-parallel over the group (:func:`run_blocks_tp`); every rank
        passes the same patches and gets the full features."""
        cfg = self.cfg
        S, P, W = self.seq, self.num_patches, cfg.width
        x = torch.empty((B * S, W), device=patches.device, dtype=self.patch_w.dtype)
        ops.linear(patches, self.patch_w, table=self.pos_emb, table_period=P, table_offset=1, out=x,
                   out_group=P, out_group_stride=S, out_row_offset=1)
        ops.cls_fill(x, self.class_emb, self.pos_emb, S)
        ops.layer_norm(x, self.ln_pre_w, self.ln_pre_b, cfg.ln_eps, out=x)
        n = len(self.blocks) + layer + 1 if layer < 0 else layer
        mx = getattr(self, "w8a8", False) and mx_blocks_ok(x, self.blocks[:n], cfg.heads)
        if tp is not None and tp[1] > 1:
            run_blocks_tp(x, self.blocks[:n], B, S, cfg.heads, cfg.act, cfg.ln_eps, tp[0], tp[1], tp[2],
                          mx=mx and tp_blocks_ok(x, self.blocks[:n], cfg.heads, tp[1], True))
        elif mx:
            run_blocks_mx(x, self.blocks[:n], B, S, cfg.heads, cfg.act, cfg.ln_eps)
        else:
            run_blocks(x, self.blocks[:n], B, S, cfg.heads, cfg.act, cfg.ln_eps)
        x = x.view(B, S, W)
        return x[:, 1:] if drop_cls else x

    def preprocess(self, images, mean, std, filter: str = "pil_bicubic", center_crop: bool = False,
                   src: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 HWC images -> patch rows [B*P, kpad]: squash resize (the reference's ONNX
        runtime) or shortest-side resize + centre crop (its torch / open_clip runtime).  ``src``:
        the images already uploaded back to back (``images`` then only carry the shapes)."""
        s = self.cfg.image_size
        return ops.image_prep(images, (s, s), mean=mean, std=std, filter=filter, layout="patches",
                              patch=self.cfg.patch_size, kpad=self.kpad, out_dtype=self.patch_w.dtype,
                              device=self.patch_w.device, center_crop=center_crop, src=src)

    def preprocess_nchw_to_patches(self, pix: torch.Tensor) -> torch.Tensor:
        """Already-normalised NCHW float pixels -> patch rows (used for parity tests)."""
        B = pix.shape[0]
        p, g = self.cfg.patch_size, self.grid
        x = pix.reshape(B, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5).reshape(B * g * g, self.kdim)
        out = torch.zeros((B * g * g, self.kpad), device=pix.device, dtype=self.patch_w.dtype)
        out[:, : self.kdim] = x.to(out.dtype)
        return out


class TextTower(nn.Module):
    """OpenAI-style causal text transformer with EOT pooling."""

    def __init__(self, cfg: TextConfig, embed_dim: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.embed_dim = embed_dim
        kw = dict(dtype=dtype, device=device)
        W = cfg.width
        self.token_emb = nn.Parameter(torch.zeros(cfg.vocab_size, W, **kw), requires_grad=False)
        self.pos_emb = nn.Parameter(torch.zeros(cfg.context_length, W, **kw), requires_grad=False)
        self.blocks = nn.ModuleList([_Block(W, int(W * cfg.mlp_ratio), dtype, device) for _ in range(cfg.layers)])
        self.ln_final_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.ln_final_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.proj_w = nn.Parameter(torch.zeros(embed_dim, W, **kw), requires_grad=False)

    def random_init(self, gen: torch.Generator):
        W = self.cfg.width
        self.token_emb.data.copy_(torch.randn(self.token_emb.shape, generator=gen) * 0.02)
        self.pos_emb.data.copy_(torch.randn(self.pos_emb.shape, generator=gen) * 0.01)
        for b in self.blocks:
            b.random_init(gen, self.cfg.layers)
        self.proj_w.data.copy_(torch.randn(self.embed_dim, W, generator=gen) * W ** -0.5)

    @torch.no_grad()
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, ctx] int64 -> L2-normalised fp32 embeddings [B, E]."""
        cfg = self.cfg
        B, S = ids.shape
        dev = self.token_emb.device
        ids = ids.to(dev)
        x = ops.embed(ids, self.token_emb, self.pos_emb[:S]).view(B * S, cfg.width)
        run_blocks_micro(x, self.blocks, B, S, cfg.heads, cfg.act, cfg.ln_eps, causal=True,
                         min_rows=_TEXT_MICRO_MIN_ROWS, tile=-1, res_tile=-1)
        if cfg.eot_token_id is None:
            eot = ids.argmax(dim=-1)
        else:
            eot = (ids == cfg.eot_token_id).int().argmax(dim=-1)
        rows = torch.arange(B, device=dev) * S + eot
        pooled = ops.layer_norm(x, self.ln_final_w, self.ln_final_b, cfg.ln_eps, row_idx=rows.long())
        emb = ops.linear(pooled, self.proj_w, out_dtype=torch.float32)
        return ops.l2_normalize_(emb)


class _BertBlock(nn.Module):
    def __init__(self, c: BertConfig, dtype, device):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        W, I = c.width, c.intermediate
        self.qkv_w = nn.Parameter(torch.empty(3 * W, W, **kw), requires_grad=False)
        self.qkv_b = nn.Parameter(torch.zeros(3 * W, **kw), requires_grad=False)
        self.out_w = nn.Parameter(torch.empty(W, W, **kw), requires_grad=False)
        self.out_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.ln1_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.ln1_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.fc1_w = nn.Parameter(torch.empty(I, W, **kw), requires_grad=False)
        self.fc1_b = nn.Parameter(torch.zeros(I, **kw), requires_grad=False)
        self.fc2_w = nn.Parameter(torch.empty(W, I, **kw), requires_grad=False)
        self.fc2_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.ln2_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.ln2_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)


class BertTextTower(nn.Module):
    """Chinese-CLIP text encoder: BERT embeddings (word + position + token-type 0, LN),
    post-LN blocks, [CLS] hidden state -> text_projection -> L2 normalise.

    Reference: the CN-CLIP ``text.*.onnx`` graphs / ``ChineseCLIPModel`` manual CLS pooling
    (packages/lumen-clip/src/lumen_clip/backends/torch_backend.py:340-393).  Per block on
    the GPU: QKV GEMM -> padded attention (per-sequence key length = non-pad tokens) ->
    out-proj GEMM with the residual fused -> LayerNorm -> fc1 GEMM + GELU -> fc2 GEMM with
    the residual fused -> LayerNorm.  Token type 0 is folded into the position table."""

    def __init__(self, cfg: BertConfig, embed_dim: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.embed_dim = embed_dim
        kw = dict(dtype=dtype, device=device)
        W = cfg.width
        self.token_emb = nn.Parameter(torch.zeros(cfg.vocab_size, W, **kw), requires_grad=False)
        self.pos_emb = nn.Parameter(torch.zeros(cfg.max_position, W, **kw), requires_grad=False)  # + type[0]
        self.emb_ln_w = nn.Parameter(torch.ones(W, **kw), requires_grad=False)
        self.emb_ln_b = nn.Parameter(torch.zeros(W, **kw), requires_grad=False)
        self.blocks = nn.ModuleList([_BertBlock(cfg, dtype, device) for _ in range(cfg.layers)])
        self.proj_w = nn.Parameter(torch.zeros(embed_dim, W, **kw), requires_grad=False)

    def random_init(self, gen: torch.Generator):
        W, I = self.cfg.width, self.cfg.intermediate
        self.token_emb.data.copy_(torch.randn(self.token_emb.shape, generator=gen) * 0.02)
        self.pos_emb.data.copy_(torch.randn(self.pos_emb.shape, generator=gen) * 0.02)
        for b in self.blocks:
            for p, fan in ((b.qkv_w, W), (b.out_w, W), (b.fc1_w, W), (b.fc2_w, I)):
                p.data.copy_(torch.randn(p.shape, generator=gen) * fan ** -0.5)
        self.proj_w.data.copy_(torch.randn(self.embed_dim, W, generator=gen) * W ** -0.5)

    @torch.no_grad()
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, ctx] int64 (right-padded with pad_token_id) -> L2-normalised fp32 [B, E]."""
        c = self.cfg
        B, S = ids.shape
        dev = self.token_emb.device
        ids = ids.to(dev)
        W, Hh = c.width, c.heads
        D = W // Hh
        kv_len = (ids != c.pad_token_id).sum(dim=1).clamp_min(1).to(torch.int32)
        x = ops.embed(ids, self.token_emb, self.pos_emb[:S]).view(B * S, W)
        ops.layer_norm(x, self.emb_ln_w, self.emb_ln_b, c.ln_eps, out=x)
        o = torch.empty_like(x)
        for blk in self.blocks:
            qkv = ops.linear(x, blk.qkv_w, blk.qkv_b)
            q5 = qkv.view(B, S, 3, Hh, D)
            ops.attention(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv_len=kv_len, out=o.view(B, S, Hh, D))
            del qkv, q5
            ops.linear(o, blk.out_w, blk.out_b, residual=x, out=x)          # x + attn
            ops.layer_norm(x, blk.ln1_w, blk.ln1_b, c.ln_eps, out=x)        # post-LN
            f = ops.linear(x, blk.fc1_w, blk.fc1_b, act=c.act)
            ops.linear(f, blk.fc2_w, blk.fc2_b, residual=x, out=x)
            ops.layer_norm(x, blk.ln2_w, blk.ln2_b, c.ln_eps, out=x)
            del f
        cls = x.view(B, S, W)[:, 0]
        emb = ops.linear(cls.contiguous(), self.proj_w, out_dtype=torch.float32)
        return ops.l2_normalize_(emb)


class CLIPModel(nn.Module):
    def __init__(self, cfg: CLIPConfig, dtype=torch.bfloat16, device=None, with_text: bool = True):
        super().__init__()
        self.cfg = cfg
        self.center_crop = False   # preprocessor: see encode_image_uint8
        if cfg.vision_arch == "fastvit":
            self.visual = FastViTTower(cfg.fastvit, cfg.embed_dim, dtype, device)
        else:
            self.visual = VisionTower(cfg.vision, cfg.embed_dim, dtype, device)
        if not with_text:
            self.text = None
        elif cfg.text_arch == "bert":
            self.text = BertTextTower(cfg.bert, cfg.embed_dim, dtype, device)
        else:
            self.text = TextTower(cfg.text, cfg.embed_dim, dtype, device)
        self.logit_scale = cfg.logit_scale

    @staticmethod
    def random(cfg: CLIPConfig | str, seed: int = 0, dtype=torch.bfloat16, device=None, with_text=True):
        if isinstance(cfg, str):
            cfg = PRESETS[cfg]
        m = CLIPModel(cfg, dtype=dtype, device="cpu", with_text=with_text)
        g = torch.Generator().manual_seed(seed)
        m.visual.random_init(g)
        if m.text is not None:
            m.text.random_init(g)
        return m.to(device) if device is not None else m

    # ---- public API (mirrors the reference backend contract: unit-norm fp32 vectors)
    @torch.no_grad()
    def encode_image_uint8(self, images, src: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 HWC images -> unit fp32 embeddings.  ``self.center_crop`` picks the
        preprocessor: False = squash resize (reference ONNX runtime, onnxrt_backend.py:410-431),
        True = shortest side + centre crop (reference torch runtime, torch_backend.py:201-204).
        ``src``: the images already on the device, back to back in one flat uint8 tensor
        (utils.jpeg.decode_batch_to_device); ``images`` then only give the (H, W) shapes."""
        crop = self.center_crop
        if src is not None:
            images = [torch.empty((h, w, 3), dtype=torch.uint8, device="meta") for h, w in images]
        if self.cfg.vision_arch == "fastvit":
            assert src is None, "FastViT preprocessing takes host images"
            x = self.visual.preprocess(images, self.cfg.image_mean, self.cfg.image_std, center_crop=crop)
            return self.visual.forward_embed(x)
        patches = self.visual.preprocess(images, self.cfg.image_mean, self.cfg.image_std, center_crop=crop, src=src)
        B = patches.shape[0] // self.visual.num_patches
        return self.visual.forward_patches(patches, B)

    @torch.no_grad()
    def encode_text_ids(self, ids: torch.Tensor) -> torch.Tensor:
        assert self.text is not None
        return self.text(ids)

    # ---- weight ingestion
    def load_state_dict_any(self, sd: dict) -> None:
        """Load OpenCLIP / OpenAI (``visual.*``), HF ``CLIPModel`` or HF ``ChineseCLIPModel`` naming."""
        if self.cfg.text_arch == "bert" and any(k.startswith("text_model.encoder.layer.") for k in sd):
            _load_bert_text(self.text, sd) if self.text is not None else None
            sd = {k: v for k, v in sd.items() if not k.startswith("text_model.") and k != "text_projection.weight"}
        if any(k.startswith("vision_model.") for k in sd):
            sd = _hf_to_openclip(sd, self.cfg)
        if self.cfg.vision_arch == "fastvit":     # open_clip TimmModel: visual.trunk.<timm FastVit names>
            self.visual.load_timm(sd, prefix="visual.trunk.")
        _load_openclip(self, sd)


def _cp(dst: torch.Tensor, src: torch.Tensor):
    if tuple(dst.shape) != tuple(src.shape):
        raise ValueError(f"shape mismatch {tuple(dst.shape)} vs {tuple(src.shape)}")
    dst.data.copy_(src.to(dst.dtype))


def _load_blocks(blocks, sd, prefix):
    for i, b in enumerate(blocks):
        p = f"{prefix}.resblocks.{i}."
        _cp(b.ln1_w, sd[p + "ln_1.weight"]); _cp(b.ln1_b, sd[p + "ln_1.bias"])
        _cp(b.qkv_w, sd[p + "attn.in_proj_weight"]); _cp(b.qkv_b, sd[p + "attn.in_proj_bias"])
        _cp(b.out_w, sd[p + "attn.out_proj.weight"]); _cp(b.out_b, sd[p + "attn.out_proj.bias"])
        _cp(b.ln2_w, sd[p + "ln_2.weight"]); _cp(b.ln2_b, sd[p + "ln_2.bias"])
        _cp(b.fc1_w, sd[p + "mlp.c_fc.weight"]); _cp(b.fc1_b, sd[p + "mlp.c_fc.bias"])
        _cp(b.fc2_w, sd[p + "mlp.c_proj.weight"]); _cp(b.fc2_b, sd[p + "mlp.c_proj.bias"])


def _load_openclip(m: CLIPModel, sd: dict) -> None:
    v = m.visual
    if isinstance(v, VisionTower):
        conv = sd["visual.conv1.weight"]
        v.patch_w.data.zero_()
        v.patch_w.data[:, : v.kdim] = conv.reshape(conv.shape[0], -1).to(v.patch_w.dtype)
        _cp(v.class_emb, sd["visual.class_embedding"])
        _cp(v.pos_emb, sd["visual.positional_embedding"])
        _cp(v.ln_pre_w, sd["visual.ln_pre.weight"]); _cp(v.ln_pre_b, sd["visual.ln_pre.bias"])
        _load_blocks(v.blocks, sd, "visual.transformer")
        _cp(v.ln_post_w, sd["visual.ln_post.weight"]); _cp(v.ln_post_b, sd["visual.ln_post.bias"])
        _cp(v.proj_w, sd["visual.proj"].t())
    if m.text is not None and "token_embedding.weight" in sd:
        t = m.text
        _cp(t.token_emb, sd["token_embedding.weight"])
        _cp(t.pos_emb, sd["positional_embedding"])
        _load_blocks(t.blocks, sd, "transformer")
        _cp(t.ln_final_w, sd["ln_final.weight"]); _cp(t.ln_final_b, sd["ln_final.bias"])
        _cp(t.proj_w, sd["text_projection"].t())
    if "logit_scale" in sd:
        m.logit_scale = float(sd["logit_scale"])


def export_openclip_state_dict(m: CLIPModel) -> dict:
    """Inverse of the OpenCLIP loader (used to write synthetic model directories)."""
    sd = {}
    v = m.visual
    if isinstance(v, FastViTTower):
        sd.update(v.export_timm(prefix="visual.trunk."))
    else:
        W, p = v.cfg.width, v.cfg.patch_size
        sd["visual.conv1.weight"] = v.patch_w[:, : v.kdim].reshape(W, 3, p, p)
        sd["visual.class_embedding"] = v.class_emb
        sd["visual.positional_embedding"] = v.pos_emb
        sd["visual.ln_pre.weight"], sd["visual.ln_pre.bias"] = v.ln_pre_w, v.ln_pre_b
        sd["visual.ln_post.weight"], sd["visual.ln_post.bias"] = v.ln_post_w, v.ln_post_b
        sd["visual.proj"] = v.proj_w.t()

    def blocks(bl, prefix):
        for i, b in enumerate(bl):
            q = f"{prefix}.resblocks.{i}."
            sd[q + "ln_1.weight"], sd[q + "ln_1.bias"] = b.ln1_w, b.ln1_b
            sd[q + "attn.in_proj_weight"], sd[q + "attn.in_proj_bias"] = b.qkv_w, b.qkv_b
            sd[q + "attn.out_proj.weight"], sd[q + "attn.out_proj.bias"] = b.out_w, b.out_b
            sd[q + "ln_2.weight"], sd[q + "ln_2.bias"] = b.ln2_w, b.ln2_b
            sd[q + "mlp.c_fc.weight"], sd[q + "mlp.c_fc.bias"] = b.fc1_w, b.fc1_b
            sd[q + "mlp.c_proj.weight"], sd[q + "mlp.c_proj.bias"] = b.fc2_w, b.fc2_b

    if isinstance(v, VisionTower):
        blocks(v.blocks, "visual.transformer")
    if m.text is not None:
        t = m.text
        sd["token_embedding.weight"] = t.token_emb
        sd["positional_embedding"] = t.pos_emb
        blocks(t.blocks, "transformer")
        sd["ln_final.weight"], sd["ln_final.bias"] = t.ln_final_w, t.ln_final_b
        sd["text_projection"] = t.proj_w.t()
    sd["logit_scale"] = torch.tensor(m.logit_scale)
    return {k: val.detach().contiguous().cpu() for k, val in sd.items()}


def _load_bert_text(t: BertTextTower, sd: dict) -> None:
    """HF ChineseCLIP / BERT text weights (``text_model.*`` + ``text_projection.weight``)."""
    p = "text_model."
    _cp(t.token_emb, sd[p + "embeddings.word_embeddings.weight"])
    pos = sd[p + "embeddings.position_embeddings.weight"].float() + sd[p + "embeddings.token_type_embeddings.weight"][0].float()
    _cp(t.pos_emb, pos)
    _cp(t.emb_ln_w, sd[p + "embeddings.LayerNorm.weight"]); _cp(t.emb_ln_b, sd[p + "embeddings.LayerNorm.bias"])
    for i, b in enumerate(t.blocks):
        q = f"{p}encoder.layer.{i}."
        a = q + "attention.self."
        _cp(b.qkv_w, torch.cat([sd[a + x + ".weight"] for x in ("query", "key", "value")]))
        _cp(b.qkv_b, torch.cat([sd[a + x + ".bias"] for x in ("query", "key", "value")]))
        _cp(b.out_w, sd[q + "attention.output.dense.weight"]); _cp(b.out_b, sd[q + "attention.output.dense.bias"])
        _cp(b.ln1_w, sd[q + "attention.output.LayerNorm.weight"]); _cp(b.ln1_b, sd[q + "attention.output.LayerNorm.bias"])
        _cp(b.fc1_w, sd[q + "intermediate.dense.weight"]); _cp(b.fc1_b, sd[q + "intermediate.dense.bias"])
        _cp(b.fc2_w, sd[q + "output.dense.weight"]); _cp(b.fc2_b, sd[q + "output.dense.bias"])
        _cp(b.ln2_w, sd[q + "output.LayerNorm.weight"]); _cp(b.ln2_b, sd[q + "output.LayerNorm.bias"])
    _cp(t.proj_w, sd["text_projection.weight"])


def export_chinese_clip_state_dict(m: "CLIPModel") -> dict:
    """HF ``ChineseCLIPModel`` naming (synthetic CN-CLIP model directories)."""
    sd = {}
    v = m.visual
    W, p = v.cfg.width, v.cfg.patch_size
    vm = "vision_model."
    sd[vm + "embeddings.patch_embedding.weight"] = v.patch_w[:, : v.kdim].reshape(W, 3, p, p)
    sd[vm + "embeddings.class_embedding"] = v.class_emb
    sd[vm + "embeddings.position_embedding.weight"] = v.pos_emb
    sd[vm + "pre_layrnorm.weight"], sd[vm + "pre_layrnorm.bias"] = v.ln_pre_w, v.ln_pre_b
    sd[vm + "post_layernorm.weight"], sd[vm + "post_layernorm.bias"] = v.ln_post_w, v.ln_post_b
    sd["visual_projection.weight"] = v.proj_w
    for i, b in enumerate(v.blocks):
        q = f"{vm}encoder.layers.{i}."
        for x, (w_, b_) in zip("qkv", zip(torch.chunk(b.qkv_w, 3), torch.chunk(b.qkv_b, 3))):
            sd[q + f"self_attn.{x}_proj.weight"], sd[q + f"self_attn.{x}_proj.bias"] = w_, b_
        sd[q + "self_attn.out_proj.weight"], sd[q + "self_attn.out_proj.bias"] = b.out_w, b.out_b
        sd[q + "layer_norm1.weight"], sd[q + "layer_norm1.bias"] = b.ln1_w, b.ln1_b
        sd[q + "layer_norm2.weight"], sd[q + "layer_norm2.bias"] = b.ln2_w, b.ln2_b
        sd[q + "mlp.fc1.weight"], sd[q + "mlp.fc1.bias"] = b.fc1_w, b.fc1_b
        sd[q + "mlp.fc2.weight"], sd[q + "mlp.fc2.bias"] = b.fc2_w, b.fc2_b
    t = m.text
    tp = "text_model."
    sd[tp + "embeddings.word_embeddings.weight"] = t.token_emb
    sd[tp + "embeddings.position_embeddings.weight"] = t.pos_emb
    sd[tp + "embeddings.token_type_embeddings.weight"] = torch.zeros(t.cfg.type_vocab, t.cfg.width, dtype=t.pos_emb.dtype)
    sd[tp + "embeddings.LayerNorm.weight"], sd[tp + "embeddings.LayerNorm.bias"] = t.emb_ln_w, t.emb_ln_b
    for i, b in enumerate(t.blocks):
        q = f"{tp}encoder.layer.{i}."
        for x, (w_, b_) in zip(("query", "key", "value"), zip(torch.chunk(b.qkv_w, 3), torch.chunk(b.qkv_b, 3))):
            sd[q + f"attention.self.{x}.weight"], sd[q + f"attention.self.{x}.bias"] = w_, b_
        sd[q + "attention.output.dense.weight"], sd[q + "attention.output.dense.bias"] = b.out_w, b.out_b
        sd[q + "attention.output.LayerNorm.weight"], sd[q + "attention.output.LayerNorm.bias"] = b.ln1_w, b.ln1_b
        sd[q + "intermediate.dense.weight"], sd[q + "intermediate.dense.bias"] = b.fc1_w, b.fc1_b
        sd[q + "output.dense.weight"], sd[q + "output.dense.bias"] = b.fc2_w, b.fc2_b
        sd[q + "output.LayerNorm.weight"], sd[q + "output.LayerNorm.bias"] = b.ln2_w, b.ln2_b
    sd["text_projection.weight"] = t.proj_w
    sd["logit_scale"] = torch.tensor(m.logit_scale)
    return {k: val.detach().contiguous().cpu() for k, val in sd.items()}


def _hf_to_openclip(sd: dict, cfg: CLIPConfig) -> dict:
    """Rename HF transformers CLIPModel weights to the OpenCLIP layout."""
    out = {}
    vm, tm = "vision_model.", "text_model."
    out["visual.conv1.weight"] = sd[vm + "embeddings.patch_embedding.weight"]
    out["visual.class_embedding"] = sd[vm + "embeddings.class_embedding"]
    out["visual.positional_embedding"] = sd[vm + "embeddings.position_embedding.weight"]
    out["visual.ln_pre.weight"] = sd[vm + "pre_layrnorm.weight"]
    out["visual.ln_pre.bias"] = sd[vm + "pre_layrnorm.bias"]
    out["visual.ln_post.weight"] = sd[vm + "post_layernorm.weight"]
    out["visual.ln_post.bias"] = sd[vm + "post_layernorm.bias"]
    out["visual.proj"] = sd["visual_projection.weight"].t()

    def blocks(src_prefix, dst_prefix, n):
        for i in range(n):
            s = f"{src_prefix}encoder.layers.{i}."
            d = f"{dst_prefix}.resblocks.{i}."
            out[d + "ln_1.weight"] = sd[s + "layer_norm1.weight"]
            out[d + "ln_1.bias"] = sd[s + "layer_norm1.bias"]
            out[d + "ln_2.weight"] = sd[s + "layer_norm2.weight"]
            out[d + "ln_2.bias"] = sd[s + "layer_norm2.bias"]
            out[d + "attn.in_proj_weight"] = torch.cat([sd[s + f"self_attn.{x}_proj.weight"] for x in "qkv"])
            out[d + "attn.in_proj_bias"] = torch.cat([sd[s + f"self_attn.{x}_proj.bias"] for x in "qkv"])
            out[d + "attn.out_proj.weight"] = sd[s + "self_attn.out_proj.weight"]
            out[d + "attn.out_proj.bias"] = sd[s + "self_attn.out_proj.bias"]
            out[d + "mlp.c_fc.weight"] = sd[s + "mlp.fc1.weight"]
            out[d + "mlp.c_fc.bias"] = sd[s + "mlp.fc1.bias"]
            out[d + "mlp.c_proj.weight"] = sd[s + "mlp.fc2.weight"]
            out[d + "mlp.c_proj.bias"] = sd[s + "mlp.fc2.bias"]

    blocks(vm, "visual.transformer", cfg.vision.layers)
    if tm + "embeddings.token_embedding.weight" in sd:
        out["token_embedding.weight"] = sd[tm + "embeddings.token_embedding.weight"]
        out["positional_embedding"] = sd[tm + "embeddings.position_embedding.weight"]
        out["ln_final.weight"] = sd[tm + "final_layer_norm.weight"]
        out["ln_final.bias"] = sd[tm + "final_layer_norm.bias"]
        out["text_projection"] = sd["text_projection.weight"].t()
        blocks(tm, "transformer", cfg.text.layers)
    if "logit_scale" in sd:
        out["logit_scale"] = sd["logit_scale"]
    return out
