"""Llama / Qwen2 decoder for the VLM, tensor-parallel over RCCL.

Reference: the FastVLM decoder ONNX graph (Qwen2-0.5B) driven by
packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:161-533; the north star
adds Llama-3-8B (LLaVA-style) at TP=8.  Per layer (every op one gfx950 kernel):

  RMSNorm (fused residual add)  ->  QKV GEMM (+bias, Qwen2)  ->  RoPE + paged-KV write
  ->  attention (prefill: flash kernel reading the rotated QKV in place, causal;
      decode: paged flash-decoding)  ->  o_proj GEMM  ->  RMSNorm  ->  gate|up GEMM with
  the SwiGLU epilogue  ->  down GEMM

Tensor parallelism (Megatron): QKV and gate|up are column-parallel (whole heads /
whole 8-column GLU groups per rank), o_proj and down are row-parallel followed by
an all-reduce (RCCL); with TP the residual add is fused into the next RMSNorm
(``norm(add=partial, resid_out=x)``) instead of the GEMM epilogue.  Embedding and
lm_head are vocab-parallel (masked lookup + all-reduce; local top-k + all-gather of
the candidates for sampling).  Weights can be loaded from HF Qwen2/Llama state dicts
(sharded at load) or random-initialised per rank directly on the device.
"""
from __future__ import annotations


import math
import os
from dataclasses import asdict, dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch
from torch import nn

from .. import ops
from ..ops import llm as lops

# Every projection runs on the hand-written kernels: bf16 prefill on the MFMA GEMMs (128x128
# LDS-DMA pipeline at a few hundred tokens), fp8 prefill W8A8 on the fp8 matrix cores
# (ops.linear_f8, csrc/gemm_f8.hip, per-token scales from the fused RMSNorm+quant kernel),
# decode on the skinny split-K kernels.  The r1 hipBLASLt prefill path is gone: FastVLM-0.5B
# TTFT measured 12.25-12.72 ms without it vs 12.60-12.76 ms with it (same box, r2).
# W8A8 prefill from this many tokens up (decode batches stay on the weight-only skinny kernels)
_F8_MIN_ROWS = 33
# GPU: RMSNorm gammas folded into qkv / gate|up / lm_head (LLM.fold_norms); decode norms become
# rstd row scales in the skinny GEMM epilogues (ops.linear_dec)
_FUSED_DECODE_NORM = True
# decode: RoPE + current-token KV-cache write inside the paged attention kernel (no rope_kv launch)
_FUSED_DECODE_ROPE = True
# TP prefill from this many rows up: the rows run as two halves whose row-parallel all-reduces go
# to a communication stream, so half A's all-reduce overlaps half B's GEMMs (624-token
# LLaVA prompts at TP 8: 64 x 5 MB all-reduces on the time-to-first-token path)
_TP_OVERLAP_MIN_ROWS = 256
# (r4's fused MX prefill chain -- block-scaled activations from the epilogues, 6 launches per
# layer -- lost its A/B to this per-token chain, 13.12 vs 12.79 ms TTFT, profiles/r4_mx_chain_ab_v1.txt,
# and was removed in r5; the MX W8A8 chain stays for the ViT tower, models/clip.py:run_blocks_mx)


@dataclass
class LLMConfig:
    vocab_size: int = 151936
    hidden_size: int = 896
    num_layers: int = 24
    num_heads: int = 14
    num_kv_heads: int = 2
    head_dim: int = 64
    intermediate_size: int = 4864
    rope_theta: float = 1000000.0
    rms_eps: float = 1e-6
    max_position: int = 32768
    tie_word_embeddings: bool = True
    qkv_bias: bool = True
    rope_scaling: Optional[dict] = None
    bos_token_id: int = 151643
    eos_token_id: int = 151645

    @staticmethod
    def from_dict(d: dict) -> "LLMConfig":
        keys = LLMConfig.__dataclass_fields__.keys()
        return LLMConfig(**{k: v for k, v in d.items() if k in keys})

    @staticmethod
    def from_hf(c: dict) -> "LLMConfig":
        H = c["num_attention_heads"]
        hd = c.get("head_dim") or c["hidden_size"] // H
        mt = c.get("model_type", "llama")
        return LLMConfig(vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], num_layers=c["num_hidden_layers"],
                         num_heads=H, num_kv_heads=c.get("num_key_value_heads", H), head_dim=hd,
                         intermediate_size=c["intermediate_size"], rope_theta=c.get("rope_theta", 10000.0),
                         rms_eps=c.get("rms_norm_eps", 1e-6), max_position=c.get("max_position_embeddings", 4096),
                         tie_word_embeddings=c.get("tie_word_embeddings", False),
                         qkv_bias=c.get("attention_bias", mt == "qwen2"), rope_scaling=c.get("rope_scaling"),
                         bos_token_id=c.get("bos_token_id") or 0,
                         eos_token_id=(c.get("eos_token_id")[0] if isinstance(c.get("eos_token_id"), list)
                                       else c.get("eos_token_id") or 0))

    def to_dict(self):
        return asdict(self)


LLM_PRESETS = {
    "qwen2-0.5b": LLMConfig(),
    "llama3-8b": LLMConfig(vocab_size=128256, hidden_size=4096, num_layers=32, num_heads=32, num_kv_heads=8,
                           head_dim=128, intermediate_size=14336, rope_theta=500000.0, rms_eps=1e-5,
                           max_position=8192, tie_word_embeddings=False, qkv_bias=False, bos_token_id=128000,
                           eos_token_id=128009),
    "vicuna-7b": LLMConfig(vocab_size=32000, hidden_size=4096, num_layers=32, num_heads=32, num_kv_heads=32,
                           head_dim=128, intermediate_size=11008, rope_theta=10000.0, rms_eps=1e-5,
                           max_position=4096, tie_word_embeddings=False, qkv_bias=False, bos_token_id=1,
                           eos_token_id=2),
    "tiny": LLMConfig(vocab_size=512, hidden_size=128, num_layers=2, num_heads=4, num_kv_heads=2, head_dim=32,
                      intermediate_size=256, max_position=2048, bos_token_id=1, eos_token_id=2),
    # TP = 4 / 8 test shapes: 8 query heads over 8 KV heads (one of each per rank at TP = 8) and over
    # 2 KV heads (GQA: every KV head replicated on TP / 2 ranks, the kv_rep > 1 load path)
    "tiny-h8": LLMConfig(vocab_size=512, hidden_size=256, num_layers=2, num_heads=8, num_kv_heads=8, head_dim=32,
                         intermediate_size=512, max_position=2048, bos_token_id=1, eos_token_id=2),
    "tiny-gqa8": LLMConfig(vocab_size=512, hidden_size=256, num_layers=2, num_heads=8, num_kv_heads=2, head_dim=32,
                           intermediate_size=512, max_position=2048, bos_token_id=1, eos_token_id=2),
}


@dataclass
class TPInfo:
    rank: int = 0
    world: int = 1
    group: object = None

    @property
    def enabled(self) -> bool:
        return self.world > 1


class DecoderLayer(nn.Module):
    def __init__(self, cfg: LLMConfig, tp: TPInfo, dtype, device):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        Hd, D = cfg.hidden_size, cfg.head_dim
        self.H = cfg.num_heads // tp.world
        self.Hkv = max(cfg.num_kv_heads // tp.world, 1)
        self.I = cfg.intermediate_size // tp.world
        self.ln1 = nn.Parameter(torch.ones(Hd, **kw), requires_grad=False)
        self.ln2 = nn.Parameter(torch.ones(Hd, **kw), requires_grad=False)
        self.qkv_w = nn.Parameter(torch.zeros((self.H + 2 * self.Hkv) * D, Hd, **kw), requires_grad=False)
        self.qkv_b = nn.Parameter(torch.zeros((self.H + 2 * self.Hkv) * D, dtype=torch.float32, device=device),
                                  requires_grad=False) if cfg.qkv_bias else None
        self.o_w = nn.Parameter(torch.zeros(Hd, self.H * D, **kw), requires_grad=False)
        self.gu_w = nn.Parameter(torch.zeros(2 * self.I, Hd, **kw), requires_grad=False)
        self.down_w = nn.Parameter(torch.zeros(Hd, self.I, **kw), requires_grad=False)


class LLM(nn.Module):
    def __init__(self, cfg: LLMConfig, tp: Optional[TPInfo] = None, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.tp = tp or TPInfo()
        w = self.tp.world
        assert cfg.num_heads % w == 0 and (cfg.num_kv_heads % w == 0 or w % cfg.num_kv_heads == 0), "TP heads"
        assert cfg.intermediate_size % (8 * w) == 0 and cfg.vocab_size % w == 0, "TP shapes"
        self.Vl = cfg.vocab_size // w
        self.v0 = self.tp.rank * self.Vl
        kw = dict(dtype=dtype, device=device)
        self.embed = nn.Parameter(torch.zeros(self.Vl, cfg.hidden_size, **kw), requires_grad=False)
        self.layers = nn.ModuleList([DecoderLayer(cfg, self.tp, dtype, device) for _ in range(cfg.num_layers)])
        self.norm = nn.Parameter(torch.ones(cfg.hidden_size, **kw), requires_grad=False)
        self.lm_head = None if cfg.tie_word_embeddings else nn.Parameter(torch.zeros(self.Vl, cfg.hidden_size, **kw),
                                                                         requires_grad=False)
        self.register_buffer("cos_sin", lops.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                                          cfg.rope_scaling).to(device), persistent=False)
        self.H, self.Hkv = self.layers[0].H, self.layers[0].Hkv
        self.comm = None   # parallel.Communicator for the TP group (IPC one-shot all-reduce + RCCL); None = RCCL
        self.weight_dtype = "bf16"
        self.norm_folded = False     # RMSNorm gammas folded into the consuming projections (fold_norms)
        self._ssq = None             # decode: per-(row, 16-column tile) sums of squares of the residual stream

    # ------------------------------------------------------------------ weights
    @torch.no_grad()
    def random_init(self, seed: int = 0):
        """Per-rank random shards generated on the model's device (coherent full model)."""
        dev = self.embed.device
        g = torch.Generator(device=dev).manual_seed(seed * 1000 + self.tp.rank)
        Hd = self.cfg.hidden_size
        L = self.cfg.num_layers

        def rnd(p, std):
            p.copy_((torch.randn(p.shape, generator=g, device=dev, dtype=torch.float32) * std).to(p.dtype))

        self.norm_folded = False
        rnd(self.embed, 0.02)
        if self.lm_head is not None:
            rnd(self.lm_head, 0.02)
        for l in self.layers:
            rnd(l.qkv_w, Hd ** -0.5)
            rnd(l.o_w, (Hd ** -0.5) / math.sqrt(2 * L))
            rnd(l.gu_w, Hd ** -0.5)
            rnd(l.down_w, (l.I * self.tp.world) ** -0.5 / math.sqrt(2 * L))
            if l.qkv_b is not None:
                rnd(l.qkv_b, 0.02)

    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict, prefix: str = "model.") -> None:
        """HF Qwen2 / Llama weights (``model.layers.N.self_attn.q_proj.weight`` ...), sharded for this rank."""
        cfg, r, w = self.cfg, self.tp.rank, self.tp.world
        D = cfg.head_dim

        def get(k):
            return sd[k].to(torch.float32)

        def rows(t, n, i):   # i-th of n equal row shards
            s = t.shape[0] // n
            return t[i * s:(i + 1) * s]

        self.norm_folded = False
        self.embed.copy_(rows(get(prefix + "embed_tokens.weight"), w, r).to(self.embed.dtype))
        if self.lm_head is not None:
            self.lm_head.copy_(rows(get("lm_head.weight"), w, r).to(self.lm_head.dtype))
        self.norm.copy_(get(prefix + "norm.weight").to(self.norm.dtype))
        kv_rep = w // cfg.num_kv_heads if w > cfg.num_kv_heads else 1
        for i, l in enumerate(self.layers):
            p = f"{prefix}layers.{i}."
            q = rows(get(p + "self_attn.q_proj.weight"), w, r)
            kvi = r // kv_rep
            kvn = max(w // kv_rep, 1)
            k = rows(get(p + "self_attn.k_proj.weight"), kvn, kvi)
            v = rows(get(p + "self_attn.v_proj.weight"), kvn, kvi)
            l.qkv_w.copy_(torch.cat([q, k, v], 0).to(l.qkv_w.dtype))
            if l.qkv_b is not None:
                bq = rows(get(p + "self_attn.q_proj.bias"), w, r)
                bk = rows(get(p + "self_attn.k_proj.bias"), kvn, kvi)
                bv = rows(get(p + "self_attn.v_proj.bias"), kvn, kvi)
                l.qkv_b.copy_(torch.cat([bq, bk, bv], 0))
            o = get(p + "self_attn.o_proj.weight")
            l.o_w.copy_(o[:, r * l.H * D:(r + 1) * l.H * D].to(l.o_w.dtype))
            gate = rows(get(p + "mlp.gate_proj.weight"), w, r)
            up = rows(get(p + "mlp.up_proj.weight"), w, r)
            l.gu_w.copy_(ops.glu_interleave(gate, up).to(l.gu_w.dtype))
            dn = get(p + "mlp.down_proj.weight")
            l.down_w.copy_(dn[:, r * l.I:(r + 1) * l.I].to(l.down_w.dtype))
            l.ln1.copy_(get(p + "input_layernorm.weight").to(l.ln1.dtype))
            l.ln2.copy_(get(p + "post_attention_layernorm.weight").to(l.ln2.dtype))

    @torch.no_grad()
    def fold_norms(self) -> None:
        """Fold every RMSNorm gamma into the projection that consumes it -- W' = W * gamma[k]
        for qkv (ln1), gate|up (ln2) and an untied lm_head (final norm) -- and set the gammas
        to 1.  rms_norm(x, g) . W^T = rstd(x) * (x . W'^T), so the decode GEMMs run on the raw
        residual stream and apply rstd in their epilogue (ops.linear_dec): no norm launch and
        no normalised copy of x per token.  fp8 weights are dequantised, folded and
        requantised per row.  Weight loads reset the flag."""
        if self.norm_folded:
            return

        def fold(obj, wname, gamma):
            w = getattr(obj, wname)
            sc = getattr(obj, wname[:-2] + "_s" if wname.endswith("_w") else wname + "_s", None)
            g = gamma.float()[None, :]
            for r0 in range(0, w.shape[0], 8192):            # bounded fp32 temporaries
                blk = w[r0:r0 + 8192].float()
                if w.dtype == torch.float8_e4m3fn:
                    blk = blk * sc[r0:r0 + 8192].float()[:, None] * g
                    w8, s8 = ops.quantize_fp8_rows(blk)
                    w[r0:r0 + 8192].copy_(w8)
                    sc[r0:r0 + 8192].copy_(s8)
                else:
                    w[r0:r0 + 8192].copy_((blk * g).to(w.dtype))

        for l in self.layers:
            fold(l, "qkv_w", l.ln1)
            l.ln1.fill_(1)
            fold(l, "gu_w", l.ln2)
            l.ln2.fill_(1)
        if self.lm_head is not None:
            fold(self, "lm_head", self.norm)
            self.norm.fill_(1)
        self.norm_folded = True

    def _ssq_buf(self, dev) -> torch.Tensor:
        if self._ssq is None or self._ssq.device != dev:
            self._ssq = torch.zeros((32, self.cfg.hidden_size // 16), device=dev, dtype=torch.float32)
        return self._ssq

    def _maybe_fold(self, x: torch.Tensor) -> None:
        # never inside a graph capture: the in-place weight rewrite would be replayed every step
        # (the engine warms up eagerly before capturing, so the fold has happened by then)
        if x.is_cuda and _FUSED_DECODE_NORM and not self.norm_folded and \
                not torch.cuda.is_current_stream_capturing():
            self.fold_norms()
            self._ssq_buf(x.device)

    @torch.no_grad()
    def quantize_fp8(self, lm_head: bool = True) -> None:
        """fp8 decoder: QKV / o / gate|up / down (and an untied lm_head) become OCP e4m3fn
        with per-output-row fp32 scales (``<name>_s`` buffers).  Decode GEMMs (<= 32 rows)
        are HBM-bound on weights and stream the fp8 weights into bf16 MFMAs (half the bytes
        per token); prefill quantises the activations per token and runs fp8 x fp8 on the
        block-scaled matrix cores (:meth:`_f8_ok`).  Accumulation and epilogues are fp32."""
        if self.weight_dtype == "fp8":
            return
        for l in self.layers:
            for name in ("qkv", "o", "gu", "down"):
                w8, sc = ops.quantize_fp8_rows(getattr(l, name + "_w"))
                setattr(l, name + "_w", nn.Parameter(w8, requires_grad=False))
                l.register_buffer(name + "_s", sc, persistent=False)
        if lm_head and self.lm_head is not None:
            w8, sc = ops.quantize_fp8_rows(self.lm_head)
            self.lm_head = nn.Parameter(w8, requires_grad=False)
            self.register_buffer("lm_head_s", sc, persistent=False)
        self.weight_dtype = "fp8"

    @staticmethod
    def _lin(x, l, name, bias=None, residual=None, out=None, glu=False):
        w = getattr(l, name + "_w")
        return ops.linear(x, w, bias=bias, residual=residual, out=out, glu=glu,
                          w_scale=getattr(l, name + "_s", None))

    def _f8_ok(self, T: int) -> bool:
        """W8A8 prefill: fp8 weights, enough rows, every projection K a multiple of 128."""
        if self.weight_dtype != "fp8" or T < _F8_MIN_ROWS:
            return False
        l = self.layers[0]
        return all(getattr(l, n + "_w").shape[1] % 128 == 0 for n in ("qkv", "o", "gu", "down"))

    @staticmethod
    def _lin8(x8, xs, l, name, bias=None, residual=None, out=None, glu=False):
        return ops.linear_f8(x8, xs, getattr(l, name + "_w"), getattr(l, name + "_s"), bias=bias, residual=residual,
                             out=out, glu=glu)

    # ------------------------------------------------------------------ collectives
    def _all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp.enabled:
            if self.comm is not None:
                return self.comm.all_reduce(t)
            import torch.distributed as dist

            dist.all_reduce(t, group=self.tp.group)
        return t

    def _comm_stream(self, dev: torch.device):
        """The TP group's communication stream (private: graph-safe, never PyTorch's pool)."""
        cs = getattr(self, "_cstream", None)
        if cs is None or cs.device != dev:
            cs = self._cstream = ops.private_stream(dev)
        return cs

    def _all_reduce_async(self, t: torch.Tensor):
        """Start the all-reduce of ``t`` (in place) on the communication stream once the work issued
        so far on the current stream (t's producer) is done; returns the event to wait for before
        reading ``t`` (None: it completed synchronously, e.g. on the CPU)."""
        if not t.is_cuda:
            self._all_reduce(t)
            return None
        cur = torch.cuda.current_stream(t.device)
        cs = self._comm_stream(t.device)
        cs.wait_stream(cur)
        with torch.cuda.stream(cs):
            self._all_reduce(t)
        ev = torch.cuda.Event()
        ev.record(cs)
        t.record_stream(cs)
        return ev

    @staticmethod
    def _wait(ev) -> None:
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    # ------------------------------------------------------------------ pieces
    def embed_tokens(self, ids: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ids [T] -> [T, hidden] (vocab-parallel: masked local lookup + all-reduce)."""
        e = ops.embed(ids.reshape(1, -1), self.embed, id_offset=self.v0,
                      out=out.view(1, -1, self.cfg.hidden_size) if out is not None else None)
        e = e.view(-1, self.cfg.hidden_size)
        return self._all_reduce(e)

    def _layers(self, x: torch.Tensor, pos: torch.Tensor, slots: Optional[torch.Tensor], kv, attn_fn) -> torch.Tensor:
        """x [T, hidden] residual stream (updated in place); returns x."""
        if self._f8_ok(x.shape[0]):
            return self._layers_f8(x, pos, slots, kv, attn_fn)
        cfg = self.cfg
        D = cfg.head_dim
        eps = cfg.rms_eps
        T = x.shape[0]
        h = torch.empty_like(x)
        tp = self.tp.enabled
        # decode rows with folded norms: every RMSNorm is an rstd row scale in the epilogue of the
        # skinny GEMM that consumes it, fed by the sums of squares the producing GEMM's epilogue
        # wrote (TP keeps the norm kernel: it also adds the all-reduced row-parallel partial)
        if x.is_cuda and T <= 32 and not tp and self.norm_folded:
            return self._layers_dec(x, pos, slots, kv, attn_fn)
        if tp and T >= _TP_OVERLAP_MIN_ROWS:
            return self._layers_tp_overlap(x, pos, slots, kv, attn_fn, f8=False)
        pending: Optional[torch.Tensor] = None   # TP: row-parallel partial to add before the next norm
        for i, l in enumerate(self.layers):
            if pending is None:
                ops.rms_norm(x, l.ln1, eps, out=h)
            else:
                ops.rms_norm(x, l.ln1, eps, add=self._all_reduce(pending), resid_out=x, out=h)
            qkv = self._lin(h, l, "qkv", bias=l.qkv_b)
            kc, vc = (kv.k[i], kv.v[i]) if kv is not None else (None, None)
            if not getattr(attn_fn, "fuses_rope", False):
                lops.rope_kv(qkv, pos, self.cos_sin, l.H, l.Hkv, D, slots, kc, vc)
            att = attn_fn(qkv, l, kc, vc)                            # [T, H*D]
            if tp:
                part = self._lin(att, l, "o")
                ops.rms_norm(x, l.ln2, eps, add=self._all_reduce(part), resid_out=x, out=h)
            else:
                self._lin(att, l, "o", residual=x, out=x)
                ops.rms_norm(x, l.ln2, eps, out=h)
            g = self._lin(h, l, "gu", glu=True)
            if tp:
                pending = self._lin(g, l, "down")
            else:
                self._lin(g, l, "down", residual=x, out=x)
            del qkv, att, g
        if pending is not None:
            x.add_(self._all_reduce(pending))
        return x

    def _layers_dec(self, x, pos, slots, kv, attn_fn):
        """Decode layer stack (<= 32 rows, norms folded): 4 GEMM launches per layer and no norm
        kernel -- o / down write the residual stream plus its per-tile sums of squares
        (``ssq``), qkv / gate|up scale their rows by the rstd those give (ops.linear_dec)."""
        D, eps = self.cfg.head_dim, self.cfg.rms_eps
        ssq = self._ssq_buf(x.device)
        for i, l in enumerate(self.layers):
            # layer 0 reads the embeddings (no producer GEMM): rstd from x itself
            qkv = ops.linear_dec(x, l.qkv_w, getattr(l, "qkv_s", None), bias=l.qkv_b, norm_eps=eps,
                                 ssq_in=ssq if i > 0 else None)
            kc, vc = (kv.k[i], kv.v[i]) if kv is not None else (None, None)
            if not getattr(attn_fn, "fuses_rope", False):      # decode attention rotates + caches itself
                lops.rope_kv(qkv, pos, self.cos_sin, l.H, l.Hkv, D, slots, kc, vc)
            att = attn_fn(qkv, l, kc, vc)
            ops.linear_dec(att, l.o_w, getattr(l, "o_s", None), residual=x, out=x, ssq_out=ssq)
            g = ops.linear_dec(x, l.gu_w, getattr(l, "gu_s", None), glu=True, norm_eps=eps, ssq_in=ssq)
            ops.linear_dec(g, l.down_w, getattr(l, "down_s", None), residual=x, out=x, ssq_out=ssq)
            del qkv, att, g
        return x

    def _layers_f8(self, x, pos, slots, kv, attn_fn):
        """W8A8 layer stack: every projection input is quantised per token by the kernel that
        produces it (RMSNorm+quant for qkv / gate|up, a row-quant pass for o / down) and the
        GEMMs run fp8 x fp8 (csrc/gemm_f8.hip).  Same TP structure as :meth:`_layers`."""
        cfg = self.cfg
        D, eps, T = cfg.head_dim, cfg.rms_eps, x.shape[0]
        dev = x.device
        h8 = torch.empty((T, x.shape[1]), device=dev, dtype=torch.float8_e4m3fn)
        hs = torch.empty((T,), device=dev, dtype=torch.float32)
        tp = self.tp.enabled
        if tp and T >= _TP_OVERLAP_MIN_ROWS:
            return self._layers_tp_overlap(x, pos, slots, kv, attn_fn, f8=True)
        pending: Optional[torch.Tensor] = None
        for i, l in enumerate(self.layers):
            add = self._all_reduce(pending) if pending is not None else None
            ops.rms_norm_quant_fp8(x, l.ln1, eps, add=add, resid_out=x if add is not None else None, out=h8, scale=hs)
            qkv = self._lin8(h8, hs, l, "qkv", bias=l.qkv_b)
            kc, vc = (kv.k[i], kv.v[i]) if kv is not None else (None, None)
            lops.rope_kv(qkv, pos, self.cos_sin, l.H, l.Hkv, D, slots, kc, vc)
            att = attn_fn(qkv, l, kc, vc)                            # [T, H*D] bf16
            a8, as_ = ops.quant_rows_fp8(att)
            if tp:
                part = self._lin8(a8, as_, l, "o")
                ops.rms_norm_quant_fp8(x, l.ln2, eps, add=self._all_reduce(part), resid_out=x, out=h8, scale=hs)
            else:
                self._lin8(a8, as_, l, "o", residual=x, out=x)
                ops.rms_norm_quant_fp8(x, l.ln2, eps, out=h8, scale=hs)
            g = self._lin8(h8, hs, l, "gu", glu=True)
            g8, gs = ops.quant_rows_fp8(g)
            if tp:
                pending = self._lin8(g8, gs, l, "down")
            else:
                self._lin8(g8, gs, l, "down", residual=x, out=x)
            del qkv, att, a8, g, g8
        if pending is not None:
            x.add_(self._all_reduce(pending))
        return x

    def _layers_tp_overlap(self, x, pos, slots, kv, attn_fn, f8: bool):
        """TP prefill with the row-parallel all-reduces off the critical path.  The rows run as two
        halves A / B through every projection; each half's o / down partial is all-reduced on the
        communication stream (:meth:`_all_reduce_async`) while the compute stream carries on with
        the other half:

            o(A) -> AR(o A) | o(B) -> AR(o B) | norm(A) gu(A) down(A) -> AR(down A) | norm(B) ...

        so AR(o A) hides under o(B), AR(o B) under A's MLP, AR(down A) under B's MLP and AR(down B)
        under the next layer's A norm + qkv.  RoPE and attention run over all rows at once (every
        query needs the keys of both halves).  Same arithmetic as :meth:`_layers` / :meth:`_layers_f8`
        row for row (the reductions are per row), so TP results do not depend on the split."""
        cfg = self.cfg
        D, eps, T = cfg.head_dim, cfg.rms_eps, x.shape[0]
        dev = x.device
        # split on a 64-row boundary (GEMM row tiles), the halves as equal as that allows
        t0 = max(64, min(T - 64, (T // 2 + 32) // 64 * 64))
        halves = ((0, t0), (t0, T))
        if f8:
            h8 = torch.empty((T, x.shape[1]), device=dev, dtype=torch.float8_e4m3fn)
            hs = torch.empty((T,), device=dev, dtype=torch.float32)
        else:
            h = torch.empty_like(x)
        pend = [None, None]      # per half: row-parallel partial still to be added to x
        evs = [None, None]       # per half: its all-reduce's completion event

        def norm(i_half, gamma):
            a, b = halves[i_half]
            add = pend[i_half]
            if add is not None:
                self._wait(evs[i_half])
            xs = x[a:b]
            kw = dict(add=add, resid_out=xs) if add is not None else {}
            if f8:
                ops.rms_norm_quant_fp8(xs, gamma, eps, out=h8[a:b], scale=hs[a:b], **kw)
            else:
                ops.rms_norm(xs, gamma, eps, out=h[a:b], **kw)
            pend[i_half] = None

        def lin(i_half, l, name, inp, inp_s=None, **kw):
            a, b = halves[i_half]
            if f8:
                return self._lin8(inp[a:b], inp_s[a:b], l, name, **kw)
            return self._lin(inp[a:b], l, name, **kw)

        for i, l in enumerate(self.layers):
            nq = (l.H + 2 * l.Hkv) * D
            qkv = torch.empty((T, nq), device=dev, dtype=x.dtype)
            for c, (a, b) in enumerate(halves):
                norm(c, l.ln1)
                lin(c, l, "qkv", h8 if f8 else h, hs if f8 else None, bias=l.qkv_b, out=qkv[a:b])
            kc, vc = (kv.k[i], kv.v[i]) if kv is not None else (None, None)
            if not getattr(attn_fn, "fuses_rope", False):
                lops.rope_kv(qkv, pos, self.cos_sin, l.H, l.Hkv, D, slots, kc, vc)
            att = attn_fn(qkv, l, kc, vc)                            # [T, H*D]
            if f8:
                a8, as_ = ops.quant_rows_fp8(att)
            for c in range(2):
                pend[c] = lin(c, l, "o", a8 if f8 else att, as_ if f8 else None)
                evs[c] = self._all_reduce_async(pend[c])
            for c in range(2):
                norm(c, l.ln2)
                a, b = halves[c]
                g = lin(c, l, "gu", h8 if f8 else h, hs if f8 else None, glu=True)
                if f8:
                    g8, gs = ops.quant_rows_fp8(g)
                    pend[c] = self._lin8(g8, gs, l, "down")
                else:
                    pend[c] = self._lin(g, l, "down")
                evs[c] = self._all_reduce_async(pend[c])
            del qkv, att
        for c, (a, b) in enumerate(halves):
            self._wait(evs[c])
            x[a:b].add_(pend[c])
        return x

    def logits(self, x_rows: torch.Tensor, ssq: Optional[torch.Tensor] = None) -> torch.Tensor:
        """final norm + lm_head of rows [B, hidden] -> local-vocab fp32 logits [B, V/tp].
        With folded norms (untied head, <= 32 rows) the norm is the lm_head GEMM's rstd row
        scale; ``ssq``: the last down projection's sums of squares of these rows (decode)."""
        w = self.lm_head if self.lm_head is not None else self.embed
        ws = getattr(self, "lm_head_s", None)
        if self.norm_folded and self.lm_head is not None and x_rows.is_cuda and x_rows.shape[0] <= 32:
            return ops.linear_dec(x_rows, w, ws, norm_eps=self.cfg.rms_eps, ssq_in=ssq, out_dtype=torch.float32)
        h = ops.rms_norm(x_rows, self.norm, self.cfg.rms_eps)
        return ops.linear(h, w, out_dtype=torch.float32, w_scale=ws)

    # ------------------------------------------------------------------ forward passes
    @torch.no_grad()
    def prefill(self, x: torch.Tensor, kv=None, slots: Optional[torch.Tensor] = None, start_pos: int = 0,
                prefix_blocks: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One sequence: input embeddings x [T, hidden] (modified in place) at positions
        start_pos.., k/v written to ``slots``; returns last-token logits [1, V/tp] fp32.

        Chunked prefill (``start_pos`` > 0): ``prefix_blocks`` (int64, the sequence's KV
        blocks covering [0, start_pos + T)) — the chunk's queries attend the cached prefix
        plus themselves (causal, last query aligned with the last key).  K/V of the prefix
        are gathered from the paged cache (K [blk, Hkv, 64, D]; V stored transposed)."""
        self._maybe_fold(x)
        T = x.shape[0]
        pos = torch.arange(start_pos, start_pos + T, device=x.device, dtype=torch.int32)
        D = self.cfg.head_dim
        S = start_pos + T

        def attn(qkv, l, kc, vc):
            q5 = qkv.view(1, T, l.H + 2 * l.Hkv, D)
            if start_pos > 0:
                assert prefix_blocks is not None and kc is not None, "chunked prefill needs the KV cache"
                kb = kc.index_select(0, prefix_blocks)                       # [nb, Hkv, 64, D]
                vb = vc.index_select(0, prefix_blocks)                       # [nb, Hkv, D, 64]
                if kb.dtype != qkv.dtype:                                     # fp8 cache -> bf16
                    kb, vb = kb.to(qkv.dtype), vb.to(qkv.dtype)
                k_all = kb.permute(0, 2, 1, 3).reshape(1, -1, l.Hkv, D)[:, :S]
                v_all = vb.permute(0, 3, 1, 2).reshape(1, -1, l.Hkv, D)[:, :S].contiguous()
            else:
                k_all, v_all = q5[:, :, l.H:l.H + l.Hkv], q5[:, :, l.H + l.Hkv:]
            o = ops.attention(q5[:, :, :l.H], k_all, v_all, causal=True)
            return o.view(T, l.H * D)

        self._layers(x, pos, slots, kv, attn)
        return self.logits(x[T - 1:T])

    @torch.no_grad()
    def decode(self, ids: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor, kv, block_table: torch.Tensor,
               ctx_len: torch.Tensor, workspace: Optional[dict] = None) -> torch.Tensor:
        """B sequences, one new token each -> logits [B, V/tp] fp32."""
        x = self.embed_tokens(ids)
        self._maybe_fold(x)

        fuse = _FUSED_DECODE_ROPE and x.is_cuda and self.cfg.head_dim in (64, 128) and \
            self.norm_folded and x.shape[0] <= 32 and not self.tp.enabled and kv is not None

        def attn(qkv, l, kc, vc):
            return lops.paged_decode(qkv, kc, vc, block_table, ctx_len, l.H, l.Hkv, workspace=workspace,
                                     rope=(pos, self.cos_sin, slots) if fuse else None)

        attn.fuses_rope = fuse     # read by _layers_dec: no separate rope_kv launch
        self._layers(x, pos, slots, kv, attn)
        dec = self.norm_folded and x.is_cuda and x.shape[0] <= 32 and not self.tp.enabled
        return self.logits(x, ssq=self._ssq if dec else None)
