"""Device-resident label banks for zero-shot classification (K12-K14).

The bank ([N, D] unit vectors, from ``datasets.<name>.embeddings`` .npy or computed
from prompts) lives in HBM as bf16 — a 10^6 x 768 TreeOfLife bank is 1.5 GB, a
rounding error against 288 GB.  A query batch is scored with the MFMA GEMM
(fp32 out) and reduced by the fused row top-k / log-sum-exp kernel, so the
softmax probabilities of the winners come out without a second pass over N.

Sharding (K13): the bank is split N/world rows per GPU and every shard
returns its local top-k (score, global index) plus its log-sum-exp; the candidates
are merged into the global top-k and the LSEs into the global softmax normaliser.
Two transports for the merge:

* SPMD ranks in a process group (``group=``): RCCL all-gather
  (``torch.distributed.all_gather_into_tensor``) — every rank gets the result;
* a serving worker pool (``shard=(rank, world)``, no group): each worker holds its
  shard (sliced from the memory-mapped .npy, never the whole bank) and answers
  :meth:`topk_local`; the service process merges with :meth:`merge_host`
  (B x k candidates per worker — bytes, not the bank).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .. import ops


def orient_bank(emb, n_labels: int, dim: Optional[int] = None):
    """A bank stored (D, N) instead of (N, D) is transposed (reference bioclip_model.py:286-309)."""
    if n_labels and emb.shape[0] != n_labels and emb.shape[1] == n_labels and (dim is None or emb.shape[0] == dim):
        return emb.T
    return emb


class LabelBank:
    def __init__(self, embeddings, device: torch.device, normalize: bool = True, group=None,
                 shard: Optional[tuple] = None):
        """embeddings: the whole bank [N, D] (array or memmap).  ``group``: shard over the
        ranks of a process group (RCCL merge); ``shard=(rank, world)``: keep only this
        rank's rows, merged by the caller (:meth:`merge_host`)."""
        self.n_total, self.dim = int(embeddings.shape[0]), int(embeddings.shape[1])
        self.group = group
        self.rank, self.world = 0, 1
        if group is not None:
            import torch.distributed as dist

            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        elif shard is not None:
            self.rank, self.world = int(shard[0]), int(shard[1])
        per = math.ceil(self.n_total / self.world)
        self.offset = min(self.rank * per, self.n_total)
        emb = torch.from_numpy(np.array(embeddings[self.offset: self.offset + per], dtype=np.float32, copy=True))
        if emb.dim() != 2:
            raise ValueError(f"label bank must be 2-D, got {tuple(emb.shape)}")
        if normalize:
            emb = emb / emb.norm(dim=1, keepdim=True).clamp_min(1e-12)
        self.n_local = emb.shape[0]
        self.device = device
        dt = torch.bfloat16 if device.type == "cuda" else torch.float32
        if device.type == "cuda" and self.n_local % 16:
            # the score GEMM tiles N in 16s: zero rows pad the bank, their scores are cut off
            # before the top-k (ImageNet's 1000 classes, a shard's remainder)
            emb = torch.cat([emb, emb.new_zeros(16 - self.n_local % 16, emb.shape[1])])
        self.bank = emb.to(device=device, dtype=dt).contiguous()

    @torch.no_grad()
    def _local(self, queries, k: int, scale: float, softmax: bool):
        q = torch.from_numpy(np.array(queries, dtype=np.float32, copy=True)).to(self.device)
        if q.dim() == 1:
            q = q[None]
        kl = min(k, self.n_local) if self.n_local > 0 else 0
        if kl > 0:
            s = ops.bank_scores(q, self.bank)
            if s.shape[1] != self.n_local:
                s = s[:, :self.n_local].contiguous()
            v, i, lse = ops.row_topk(s, kl, scale=scale, with_lse=softmax, index_offset=self.offset)
        else:
            B = q.shape[0]
            v = torch.full((B, 0), float("-inf"), device=self.device)
            i = torch.zeros((B, 0), dtype=torch.int32, device=self.device)
            lse = torch.full((B,), float("-inf"), device=self.device) if softmax else None
        return v, i, lse

    def topk_local(self, queries, k: int, scale: float = 1.0, softmax: bool = False):
        """This shard's candidates: (raw scores [B, kl], global indices [B, kl], lse [B] | None)."""
        v, i, lse = self._local(queries, min(k, self.n_total), scale, softmax)
        return (v.float().cpu().numpy(), i.long().cpu().numpy(),
                lse.float().cpu().numpy() if lse is not None else None)

    @staticmethod
    def merge_host(parts, k: int, scale: float = 1.0, softmax: bool = False):
        """Merge per-shard :meth:`topk_local` results -> (scores [B, k], indices [B, k]);
        ties broken by the lower global index (the unsharded kernel's order)."""
        v = np.concatenate([p[0] for p in parts], axis=1)
        i = np.concatenate([p[1] for p in parts], axis=1)
        k = min(k, v.shape[1])
        order = np.lexsort((i, -v), axis=1)[:, :k] if v.shape[0] else np.zeros((0, k), np.int64)
        tv = np.take_along_axis(v, order, 1)
        ti = np.take_along_axis(i, order, 1)
        if softmax:
            lse = np.logaddexp.reduce(np.stack([p[2] for p in parts]), axis=0)
            tv = np.exp(tv * scale - lse[:, None])
        return tv.astype(np.float32), ti.astype(np.int64)

    @torch.no_grad()
    def topk(self, queries, k: int, scale: float = 1.0, softmax: bool = False):
        """queries [B, D] (unit) -> (scores [B, k] np.float32, indices [B, k] np.int64).

        softmax=False: raw cosine scores (BioCLIP); softmax=True: probabilities of
        softmax(scale * cos) over the whole bank (CLIP ImageNet classify).
        """
        if self.group is None and self.world > 1:
            raise RuntimeError("a pool shard answers topk_local(); merge with LabelBank.merge_host")
        k = min(k, self.n_total)
        v, i, lse = self._local(queries, k, scale, softmax)
        if self.world > 1:
            v, i, lse = self._merge(v, i, lse, k)
        v = v.float()
        if softmax:
            v = torch.exp(v * scale - lse[:, None])
        return v.cpu().numpy(), i.long().cpu().numpy()

    def _merge(self, v, i, lse, k):
        import torch.distributed as dist

        B, kl = v.shape
        pad = k - kl
        if pad > 0:
            v = torch.cat([v, torch.full((B, pad), float("-inf"), device=v.device)], 1)
            i = torch.cat([i, torch.full((B, pad), -1, dtype=i.dtype, device=i.device)], 1)
        # [world*B, k] outputs (rank-major): the layout both RCCL and gloo accept
        gv = torch.empty((self.world * B, k), device=v.device, dtype=v.dtype)
        gi = torch.empty((self.world * B, k), device=i.device, dtype=i.dtype)
        dist.all_gather_into_tensor(gv, v.contiguous(), group=self.group)
        dist.all_gather_into_tensor(gi, i.contiguous(), group=self.group)
        cv = gv.view(self.world, B, k).permute(1, 0, 2).reshape(B, self.world * k)
        ci = gi.view(self.world, B, k).permute(1, 0, 2).reshape(B, self.world * k)
        tv, pos = torch.topk(cv, k, dim=1)
        ti = torch.gather(ci, 1, pos)
        if lse is not None:
            g = torch.empty((self.world * B,), device=lse.device, dtype=lse.dtype)
            dist.all_gather_into_tensor(g, lse.contiguous(), group=self.group)
            lse = torch.logsumexp(g.view(self.world, B), dim=0)
        return tv, ti, lse


class PoolShardedBank:
    """Client side of a bank sharded over a serving worker pool (one shard per GPU worker,
    built by the worker from its own memory-mapped copy of the bank): broadcast the queries,
    merge the per-shard candidates on the host.  Same ``topk`` contract as :class:`LabelBank`."""

    def __init__(self, pool, n_total: int, kind: str = "bank_topk"):
        self.pool = pool
        self.n_total = int(n_total)
        self.kind = kind

    def topk(self, queries, k: int, scale: float = 1.0, softmax: bool = False):
        q = np.asarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None]
        k = min(k, self.n_total)
        parts = [r[0] for r in self.pool.broadcast(self.kind, [(q, k, float(scale), bool(softmax))])]
        return LabelBank.merge_host(parts, k, scale, softmax)
