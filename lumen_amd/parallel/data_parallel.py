"""SPMD image-batch data parallelism (one process per GPU, RCCL all-gather).

Used by batch jobs launched with torchrun (``tools/build_label_bank.py``: the
BioCLIP / CLIP label-bank precompute): every rank encodes its
contiguous shard of the global batch on its own GPU, then one RCCL
``all_gather_into_tensor`` over xGMI assembles the [global_batch, D] result on
every rank.  For online serving behind one gRPC endpoint the equivalent is
:class:`~lumen_amd.parallel.worker_pool.GPUWorkerPool`.

Sizing for 288 GB HBM: a ViT-L/14 bf16 tower is 0.6 GB of weights and ~0.6 MB
of activations per image per live layer, so per-GPU batches of 512-2048 images
fit with room to spare; bigger shards mean fewer, larger all-gathers.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from .comm import Communicator


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous near-equal split of n items: [start, stop) of ``rank``."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


class DataParallelRunner:
    """``run(global_items)``: apply ``fn`` to this rank's shard, all-gather the rows.

    ``fn(local_items) -> Tensor [n_local, ...]`` runs on this rank's device; the
    result is [len(global_items), ...] on every rank, in global order."""

    def __init__(self, fn: Callable, comm: Optional[Communicator] = None):
        self.fn = fn
        self.comm = comm or Communicator(ipc=False)

    def local_slice(self, n: int) -> slice:
        a, b = shard_range(n, self.comm.rank, self.comm.world)
        return slice(a, b)

    def run(self, global_items) -> torch.Tensor:
        local = global_items[self.local_slice(len(global_items))]
        out = self.fn(local)
        return self.comm.all_gather_rows(out)
