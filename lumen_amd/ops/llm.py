"""Decoder-LLM ops: RoPE tables, fused RoPE + paged KV write, paged decode attention,
repetition penalty, candidate sampling.

GPU tensors run the HIP kernels of csrc/llm.hip; CPU tensors run fp32 references with
the same semantics (cache layouts in csrc/llm.h: k [NB, Hkv, 64, D], v [NB, Hkv, D, 64]).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence

import numpy as np
import torch

from .._native import hip_ops
from ..utils.h2d import h2d

KV_BLOCK = 64


def rope_cos_sin(max_pos: int, head_dim: int, theta: float = 10000.0, scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, D/2, 2] fp32 (cos, sin) with HF inv_freq (+ Llama-3 frequency scaling)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2 / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        f = float(scaling.get("factor", 8.0))
        lo, hi = float(scaling.get("low_freq_factor", 1.0)), float(scaling.get("high_freq_factor", 4.0))
        old = float(scaling.get("original_max_position_embeddings", 8192))
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > old / lo, inv / f, inv)
        mid = (wl <= old / lo) & (wl >= old / hi)
        scaled = torch.where(mid, (1 - smooth) * inv / f + smooth * inv, scaled)
        inv = scaled
    elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
        inv = inv / float(scaling.get("factor", 1.0))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()


def _rot_ref(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    """x [T, n, D] fp32, cs [T, D/2, 2] -> rotate-half RoPE."""
    half = x.shape[-1] // 2
    c, s = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor, H: int, Hkv: int, D: int,
            slots: Optional[torch.Tensor] = None, k_cache: Optional[torch.Tensor] = None,
            v_cache: Optional[torch.Tensor] = None) -> None:
    """Rotate q and k heads of qkv [T, (H + 2Hkv) D] in place; with ``slots`` also write k / v
    of every token into the paged cache (slot = block * 64 + offset, < 0 skipped)."""
    T = qkv.shape[0]
    if qkv.is_cuda:
        hip_ops().rope_kv(qkv, pos.to(torch.int32).contiguous(), cos_sin,
                          slots.to(torch.long).contiguous() if slots is not None else None,
                          k_cache if k_cache is not None else qkv, v_cache if v_cache is not None else qkv,
                          int(H), int(Hkv), int(D))
        return
    if T == 0:
        return
    cs = cos_sin[pos.long()]
    nq = (H + Hkv) * D
    x = qkv[:, :nq].float().view(T, H + Hkv, D)
    xr = _rot_ref(x, cs).to(qkv.dtype)
    qkv[:, :nq] = xr.view(T, nq)
    if slots is not None:
        v = qkv[:, nq:nq + Hkv * D].view(T, Hkv, D)
        for t in range(T):
            sl = int(slots[t])
            if sl < 0:
                continue
            blk, off = sl // KV_BLOCK, sl % KV_BLOCK
            kt, vt = xr[t, H:].float(), v[t].float()
            if k_cache.dtype == torch.float8_e4m3fn:      # the GPU writers saturate to +-448
                kt, vt = kt.clamp(-448, 448), vt.clamp(-448, 448)
            k_cache[blk, :, off, :] = kt.to(k_cache.dtype)
            v_cache[blk, :, :, off] = vt.to(v_cache.dtype)


_DECODE_WAVES = 4             # waves (= 64-token blocks) per paged-decode workgroup (csrc/llm.hip PD_NW)
_DECODE_MAX_SPLITS = 32        # the in-launch split combine merges at most 32 splits per kv head


_DECODE_FEW = 4                # <= this many sequences: one-wave workgroups, one block per split


def decode_splits(B: int, Hkv: int, max_blocks: int, target_wg: Optional[int] = None) -> tuple[int, int]:
    """(nsplit, min blocks_per_split) of the paged decode kernel.

    A split is one workgroup of 4 waves, one 64-token block per wave.  Batched decode (B > 4):
    splits of >= 4 blocks, so a context of <= 256 tokens is one workgroup per kv head with no
    cross-workgroup combine; longer contexts use up to 32 splits merged in-launch, and past 8k
    tokens the waves loop over several blocks.  A few sequences (B <= 4): the same launch with
    no minimum, so each sequence's blocks spread over all launched splits.  The kernel sizes the
    splits from each sequence's ctx_len on the device (blocks per split = max(min,
    ceil(blocks / nsplit)))."""
    nsplit = max(1, min(-(-max_blocks // _DECODE_WAVES), _DECODE_MAX_SPLITS))
    if B <= _DECODE_FEW:
        # one block per wave, but the context spread over every launched split: 650 tokens on an
        # 8-split launch run as 6 splits x 2 blocks, 9.8 us vs 10.7 us as 3 x 4 and 20.4 us as 32
        # one-wave splits, whose single-wave combine is latency-serial (r3_decode_attn_splits_v1.txt)
        return nsplit, 1
    bps = -(-max_blocks // nsplit)
    return -(-max_blocks // bps), bps


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_table: torch.Tensor,
                 ctx_len: torch.Tensor, H: int, Hkv: int, scale: Optional[float] = None,
                 out: Optional[torch.Tensor] = None, workspace: Optional[dict] = None,
                 rope: Optional[tuple] = None, prefetch: Sequence[torch.Tensor] = (),
                 splits: Optional[tuple] = None) -> torch.Tensor:
    """Single-token attention of q [B, H*D] (rows may be views) over each sequence's cached
    context (ctx_len tokens, including the current token).

    ``rope = (pos [B] int32, cos_sin, slots [B] int64)``: q is the *unrotated* packed QKV row
    and the kernel applies RoPE to q in registers and writes the current token's rotated k and
    its v to ``slots`` itself (what :func:`rope_kv` would do; one launch per layer fewer).
    ``prefetch``: up to two tensors (the next GEMMs' weights) that extra workgroups of the same
    launch read once into the Infinity Cache while the attention occupies only a few CUs.
    Head dims 64 / 128 on the GPU."""
    B = q.shape[0]
    D = k_cache.shape[3]
    if rope is not None and not (q.is_cuda and D in (64, 128)):
        pos, cos_sin, slots = rope
        q = q.clone()
        rope_kv(q, pos, cos_sin, H, Hkv, D, slots, k_cache, v_cache)
        rope = None
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if out is None:
        out = torch.empty((B, H * D), device=q.device, dtype=q.dtype)
    if q.is_cuda:
        mb = block_table.shape[1]
        nsplit, bps = splits if splits is not None else decode_splits(B, Hkv, mb)   # splits: benchmarks
        po = pm = None
        if nsplit > 1:
            need = B * H * nsplit
            ws = workspace if workspace is not None else {}
            po = ws.get("o")
            if po is None or po.numel() < need * D:
                po = torch.empty(need * D, device=q.device, dtype=torch.float32)
                ws["o"] = po
            pm = ws.get("ml")
            if pm is None or pm.numel() < need * 2:
                pm = torch.empty(need * 2, device=q.device, dtype=torch.float32)
                ws["ml"] = pm
        rp = (None, None, None) if rope is None else \
            (rope[0].to(torch.int32).contiguous(), rope[1], rope[2].to(torch.long).contiguous())
        pf = list(prefetch)[:2] + [None, None]
        hip_ops().paged_decode(q, k_cache, v_cache, block_table, ctx_len, out, int(H), int(Hkv), float(scale),
                               int(nsplit), int(bps), po, pm, *rp, pf[0], pf[1])
        return out
    G = H // Hkv
    for b in range(B):
        L = int(ctx_len[b])
        nb = -(-L // KV_BLOCK)
        blocks = block_table[b, :nb].long()
        k = k_cache[blocks].float().permute(1, 0, 2, 3).reshape(Hkv, nb * KV_BLOCK, D)[:, :L]
        v = v_cache[blocks].float().permute(1, 0, 3, 2).reshape(Hkv, nb * KV_BLOCK, D)[:, :L]
        qb = q[b, :H * D].float().view(Hkv, G, D)
        s = torch.einsum("hgd,htd->hgt", qb, k) * scale
        p = torch.softmax(s, -1)
        o = torch.einsum("hgt,htd->hgd", p, v)
        out[b, :H * D] = o.reshape(H * D).to(out.dtype)
    return out


def rep_penalty_(logits: torch.Tensor, token_ids: Sequence[Sequence[int]], penalty: Sequence[float]) -> torch.Tensor:
    """logits[b, t] /= p (if > 0) or *= p for every distinct previously seen token t."""
    B = logits.shape[0]
    uniq = [sorted(set(int(t) for t in ids)) for ids in token_ids]
    maxn = max((len(u) for u in uniq), default=0)
    if maxn == 0:
        return logits
    ids = np.full((B, maxn), -1, np.int32)
    for b, u in enumerate(uniq):
        ids[b, :len(u)] = u
    if logits.is_cuda:
        hip_ops().rep_penalty_(logits, h2d(ids, logits.device), h2d(list(penalty), logits.device, torch.float32))
        return logits
    for b, u in enumerate(uniq):
        if not u:
            continue
        idx = torch.tensor(u)
        v = logits[b, idx]
        logits[b, idx] = torch.where(v > 0, v / penalty[b], v * penalty[b])
    return logits


def sample_from_candidates(vals: np.ndarray, idx: np.ndarray, lse: float, temperature: float, top_p: float,
                           rng: np.random.Generator) -> int:
    """Nucleus sampling from the top-k candidates of one row.

    ``vals`` are logits/temperature sorted descending, ``lse`` the log-sum-exp over the
    full vocabulary of the same scaled logits, so ``exp(vals - lse)`` are exact
    probabilities.  The nucleus is the smallest prefix with mass >= top_p; when the
    top-k mass is below top_p the whole candidate set is used (documented truncation)."""
    p = np.exp(vals.astype(np.float64) - lse)
    c = np.cumsum(p)
    n = int(np.searchsorted(c, top_p * c[-1] if c[-1] < top_p else top_p) + 1)
    n = max(1, min(n, len(p)))
    q = p[:n] / p[:n].sum()
    return int(idx[int(rng.choice(n, p=q))])
