"""Collectives for the MI355X build: RCCL for bulk traffic, IPC one-shot for latency.

xGMI on an 8 x MI355X node is a full mesh of point-to-point links (7 per GPU,
~153 GB/s each), not a switch.  Two regimes follow:

* **Latency-bound** (TP decode: one [B, hidden] bf16 row block per layer, 8 KB
  at B = 1): a ring all-reduce pays 2(n-1) link hops of launch + sync latency.
  :class:`CustomAllReduce` instead writes each rank's partial into its own
  IPC-mapped uncached buffer, exchanges one flag per peer, and every rank reads
  all 7 peers concurrently and reduces locally — one hop, all links busy
  (``csrc/comm.hip``).  It is hipGraph-capturable (device-side epochs).
* **Bandwidth-bound** (prefill all-reduces of MBs, DP result gathers, label-bank
  candidate merges): RCCL through ``torch.distributed`` ("nccl" backend).

:class:`Communicator` picks per call: the IPC path when the group lives on
distinct GPUs of one node, the tensor is bf16/fp32 and at most ``max_bytes``;
RCCL (or gloo on CPU) otherwise.  The selection threshold is the size where a
one-shot read of (n-1) x bytes over 7 links stops beating RCCL's ring.
"""
from __future__ import annotations

import logging
import os
from typing import Optional, Sequence

import torch

log = logging.getLogger("lumen.comm")

DEFAULT_IPC_MAX_BYTES = int(os.environ.get("LUMEN_IPC_AR_MAX_BYTES", str(512 * 1024)))
# two-shot IPC all-reduce (reduce-scatter + all-gather reading every peer at once): messages above the
# one-shot limit and up to this many bytes, in groups of >= 4 ranks, where it moves 2 (n-1)/n of the
# message per rank instead of the ring's 2 (n-1)/n in 2 (n-1) serial hops -- the TP prefill
# all-reduces (624 x 4096 bf16 = 5 MB per layer at Llama-3-8B)
TWO_SHOT_MAX_BYTES = int(os.environ.get("LUMEN_IPC_AR2_MAX_BYTES", str(16 << 20)))
TWO_SHOT_MIN_WORLD = int(os.environ.get("LUMEN_IPC_AR2_MIN_WORLD", "4"))
# without RCCL (gloo groups: several TP ranks sharing one GPU in tests) every message the IPC
# kernel cannot take is staged through the host; cover prefill-sized all-reduces there too
GLOO_IPC_MAX_BYTES = 32 << 20


class TPGroupUnavailable(RuntimeError):
    """A tensor-parallel peer stopped answering (the IPC all-reduce gave up waiting for it):
    the group's results are invalid and the service reports UNAVAILABLE."""


def _group_ranks(group) -> tuple[int, int]:
    import torch.distributed as dist

    return dist.get_rank(group), dist.get_world_size(group)


class CustomAllReduce:
    """IPC one-shot all-reduce over one process group (every member on its own GPU,
    or — for single-GPU testing — several processes sharing one GPU).

    Construction is collective over ``group``: each rank allocates one uncached
    buffer (16 KiB control + 2 x ``max_bytes`` data), exports its hipIpc handle,
    all-gathers the handles and maps every peer's buffer."""

    def __init__(self, group=None, device: Optional[torch.device] = None, max_bytes: int = DEFAULT_IPC_MAX_BYTES):
        import torch.distributed as dist

        from .._native import hip_ops

        self.ops = hip_ops()
        self.group = group
        self.rank, self.world = _group_ranks(group)
        if self.world > 8:
            raise ValueError("CustomAllReduce supports at most 8 ranks (one xGMI node)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = (int(max_bytes) + 15) // 16 * 16
        with torch.cuda.device(self.device):
            self.own = int(self.ops.ar_alloc(self.max_bytes))
            handle = self.ops.ar_handle(self.own)
        handles: list = [None] * self.world
        dist.all_gather_object(handles, handle.numpy().tobytes(), group=group)
        self.bases: list[int] = []
        self._opened: list[int] = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    self.bases.append(self.own)
                else:
                    p = int(self.ops.ar_open(torch.frombuffer(bytearray(h), dtype=torch.uint8)))
                    self.bases.append(p)
                    self._opened.append(p)
        dist.barrier(group=group)
        self.closed = False

    def eligible(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (not self.closed and t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and nbytes % 16 == 0 and 0 < nbytes <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None, two_shot: bool = False) -> torch.Tensor:
        """Sum over the group; in place unless ``out`` is given.  ``two_shot``: the reduce-scatter +
        all-gather form (bandwidth-bound messages); every rank must pass the same value."""
        out = t if out is None else out
        self.ops.custom_all_reduce(t, out, self.bases, self.rank, self.max_bytes, bool(two_shot))
        return out

    def error(self) -> bool:
        """True if any call so far gave up waiting for a peer (synchronises)."""
        return bool(self.ops.ar_error(self.own))

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.ops.ar_close(p)
        self.ops.ar_free(self.own)


class Communicator:
    """Per-group collective front-end (all-reduce / all-gather / broadcast).

    ``ipc``: None = auto (enable the IPC all-reduce for a multi-rank group of GPU
    processes when the native library is present), True = require, False = RCCL only.
    """

    def __init__(self, group=None, device: Optional[torch.device] = None, ipc: Optional[bool] = None,
                 ipc_max_bytes: int = DEFAULT_IPC_MAX_BYTES, two_shot_max_bytes: int = TWO_SHOT_MAX_BYTES):
        import torch.distributed as dist

        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.rank, self.world = _group_ranks(group) if self.enabled else (0, 1)
        self.device = device
        self.custom: Optional[CustomAllReduce] = None
        self.stats = {"ipc_calls": 0, "rccl_calls": 0, "ipc_bytes": 0, "rccl_bytes": 0, "ipc2_calls": 0}
        self.one_shot_max = ipc_max_bytes
        if ipc is None:
            ipc = os.environ.get("LUMEN_IPC_ALLREDUCE", "1") == "1"
            ipc = ipc and self.world > 1 and device is not None and device.type == "cuda"
        if ipc and self.world > 1:
            cap = ipc_max_bytes
            if self.enabled and dist.get_backend(group) != "nccl":
                cap = max(cap, GLOO_IPC_MAX_BYTES)     # (above the one-shot limit: two-shot)
            if self.world >= TWO_SHOT_MIN_WORLD:
                cap = max(cap, two_shot_max_bytes)
            try:
                self.custom = CustomAllReduce(group, device, cap)
            except Exception as e:  # noqa: BLE001 - fall back to RCCL, loudly
                log.warning("IPC all-reduce unavailable (%s); using RCCL for every all-reduce", e)
                self.custom = None

    # ---------------------------------------------------------------- all-reduce
    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group (no-op for a group of one)."""
        if self.world <= 1:
            return t
        nbytes = t.numel() * t.element_size()
        if self.custom is not None and self.custom.eligible(t):
            self.stats["ipc_calls"] += 1
            self.stats["ipc_bytes"] += nbytes
            two = nbytes > self.one_shot_max      # room above it: groups of >= TWO_SHOT_MIN_WORLD / gloo groups
            self.stats["ipc2_calls"] += int(two)
            return self.custom.all_reduce(t, two_shot=two)
        import torch.distributed as dist

        self.stats["rccl_calls"] += 1
        self.stats["rccl_bytes"] += nbytes
        dist.all_reduce(t, group=self.group)
        return t

    # ---------------------------------------------------------------- gathers
    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate [n_r, ...] row blocks of every rank (n_r may differ) -> [sum n_r, ...]."""
        if self.world <= 1:
            return t
        import torch.distributed as dist

        n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.int64)
        ns = torch.empty(self.world, device=t.device, dtype=torch.int64)
        dist.all_gather_into_tensor(ns, n, group=self.group)
        sizes = [int(x) for x in ns.tolist()]
        mx = max(sizes)
        if t.shape[0] < mx:
            pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
            t = torch.cat([t, pad], 0)
        buf = torch.empty((self.world * mx,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(buf, t.contiguous(), group=self.group)
        if all(s == mx for s in sizes):
            return buf
        return torch.cat([buf[r * mx: r * mx + s] for r, s in enumerate(sizes)], 0)

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """Equal-size gather into a preallocated [world * n, ...] tensor (RCCL)."""
        if self.world <= 1:
            out.copy_(t)
            return out
        import torch.distributed as dist

        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def broadcast_object(self, obj=None, src: int = 0):
        if self.world <= 1:
            return obj
        import torch.distributed as dist

        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    def barrier(self) -> None:
        if self.world > 1:
            import torch.distributed as dist

            dist.barrier(group=self.group)

    def check(self) -> None:
        """Raise :class:`TPGroupUnavailable` if an IPC all-reduce gave up on a peer (synchronises:
        call it at points that already wait for the device, e.g. after a step's token D2H)."""
        if self.custom is not None and self.custom.error():
            raise TPGroupUnavailable("tensor-parallel peer not responding (IPC all-reduce timed out)")

    def error_into(self, out: torch.Tensor) -> None:
        """Enqueue the IPC all-reduce error word into ``out[0]`` (int32, device; capturable), so a
        step's result copy carries it; zero when the IPC path is off."""
        if self.custom is not None:
            self.custom.ops.ar_error_into(self.custom.own, out)
        else:
            out[:1].zero_()

    def close(self) -> None:
        if self.custom is not None:
            self.custom.close()
            self.custom = None


class BucketedAllGather:
    """Coalesce many small per-rank tensors into ONE all-gather per flush.

    DP serving produces one small result per request (a 768-d embedding is 3 KB);
    gathering each separately is pure latency.  Tensors are packed into a flat
    byte bucket (``bucket_bytes``, sized for xGMI: large enough that the ring is
    bandwidth-bound, ~4 MB), gathered once, and unpacked per rank."""

    def __init__(self, comm: Communicator, bucket_bytes: int = 4 << 20):
        self.comm = comm
        self.bucket_bytes = bucket_bytes
        self._items: list[torch.Tensor] = []
        self._bytes = 0

    def add(self, t: torch.Tensor) -> None:
        self._items.append(t.contiguous())
        self._bytes += t.numel() * t.element_size()

    @property
    def full(self) -> bool:
        return self._bytes >= self.bucket_bytes

    def flush(self) -> list[list[torch.Tensor]]:
        """-> per rank, the list of tensors that rank added (same shapes/dtypes on every rank)."""
        items, self._items, self._bytes = self._items, [], 0
        if not items:
            return [[] for _ in range(self.comm.world)]
        flat = torch.cat([x.reshape(-1).view(torch.uint8) for x in items])
        pad = (-flat.numel()) % 16
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
        buf = torch.empty(self.comm.world * flat.numel(), dtype=torch.uint8, device=flat.device)
        self.comm.all_gather_into(buf, flat)
        out = []
        step = flat.numel()
        for r in range(self.comm.world):
            chunk = buf[r * step:(r + 1) * step]
            off = 0
            per = []
            for x in items:
                nb = x.numel() * x.element_size()
                per.append(chunk[off:off + nb].view(x.dtype).view(x.shape))
                off += nb
            out.append(per)
        return out


def ring_all_reduce_time_model(nbytes: int, world: int, link_gbps: float = 153.0, hop_us: float = 5.0) -> dict:
    """Link-time cost model behind the IPC path (microseconds; latency terms dominate).

    ring: 2(n-1) dependent steps of nbytes/n over one link each, each paying a hop;
    one-shot: every rank reads (n-1) x nbytes over its n-1 links in parallel + one
    flag exchange.  For the 8 KB-per-row decode messages the ring is ~7x slower
    purely from hop latency.  The model ignores what bounds one-shot for large
    messages — staging through uncached memory and (n-1)x HBM read amplification —
    which is why :data:`DEFAULT_IPC_MAX_BYTES` (512 KB) caps the IPC path and RCCL
    carries everything bigger."""
    n = max(world, 1)
    link = link_gbps * 1e3  # bytes per microsecond
    ring = 2 * (n - 1) * (nbytes / n / link + hop_us)
    one_shot = nbytes / link + 2 * hop_us
    return {"ring_us": ring, "one_shot_us": one_shot}
