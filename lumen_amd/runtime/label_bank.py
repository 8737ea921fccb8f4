"""Device-resident label banks for zero-shot classification (K12-K14).

The bank ([N, D] unit vectors, from ``datasets.<name>.embeddings`` .npy or computed
from prompts) lives in HBM as bf16 — a 10^6 x 768 TreeOfLife bank is 1.5 GB, a
rounding error against 288 GB.  A query batch is scored with the MFMA GEMM
(fp32 out) and reduced by the fused row top-k / log-sum-exp kernel, so the
softmax probabilities of the winners come out without a second pass over N.

With a process group (DP workers, one per GPU) the bank is sharded N/world per
GPU; each rank computes its local top-k and the (score, index) candidates are
merged with an RCCL all-gather (``torch.distributed.all_gather_into_tensor``),
plus a log-sum-exp all-reduce for global softmax normalisation.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .. import ops


class LabelBank:
    def __init__(self, embeddings, device: torch.device, normalize: bool = True, group=None):
        emb = torch.from_numpy(np.array(embeddings, dtype=np.float32, copy=True))
        if emb.dim() != 2:
            raise ValueError(f"label bank must be 2-D, got {tuple(emb.shape)}")
        if normalize:
            emb = emb / emb.norm(dim=1, keepdim=True).clamp_min(1e-12)
        self.n_total, self.dim = emb.shape
        self.group = group
        self.rank, self.world = 0, 1
        if group is not None:
            import torch.distributed as dist

            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        per = math.ceil(self.n_total / self.world)
        self.offset = self.rank * per
        shard = emb[self.offset: self.offset + per]
        self.n_local = shard.shape[0]
        self.device = device
        dt = torch.bfloat16 if device.type == "cuda" else torch.float32
        self.bank = shard.to(device=device, dtype=dt).contiguous()

    @torch.no_grad()
    def topk(self, queries, k: int, scale: float = 1.0, softmax: bool = False):
        """queries [B, D] (unit) -> (scores [B, k] np.float32, indices [B, k] np.int64).

        softmax=False: raw cosine scores (BioCLIP); softmax=True: probabilities of
        softmax(scale * cos) over the whole bank (CLIP ImageNet classify).
        """
        q = torch.from_numpy(np.array(queries, dtype=np.float32, copy=True)).to(self.device)
        if q.dim() == 1:
            q = q[None]
        k = min(k, self.n_total)
        kl = min(k, self.n_local) if self.n_local > 0 else 0
        if kl > 0:
            s = ops.bank_scores(q, self.bank)
            v, i, lse = ops.row_topk(s, kl, scale=scale, with_lse=softmax, index_offset=self.offset)
        else:
            B = q.shape[0]
            v = torch.full((B, 0), float("-inf"), device=self.device)
            i = torch.zeros((B, 0), dtype=torch.int32, device=self.device)
            lse = torch.full((B,), float("-inf"), device=self.device) if softmax else None
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
        gv = torch.empty((self.world, B, k), device=v.device, dtype=v.dtype)
        gi = torch.empty((self.world, B, k), device=i.device, dtype=i.dtype)
        dist.all_gather_into_tensor(gv, v.contiguous(), group=self.group)
        dist.all_gather_into_tensor(gi, i.contiguous(), group=self.group)
        cv = gv.permute(1, 0, 2).reshape(B, self.world * k)
        ci = gi.permute(1, 0, 2).reshape(B, self.world * k)
        tv, pos = torch.topk(cv, k, dim=1)
        ti = torch.gather(ci, 1, pos)
        if lse is not None:
            g = torch.empty((self.world, B), device=lse.device, dtype=lse.dtype)
            dist.all_gather_into_tensor(g, lse.contiguous(), group=self.group)
            lse = torch.logsumexp(g, dim=0)
        return tv, ti, lse
