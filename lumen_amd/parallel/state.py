"""Process-group bootstrap: one process per GPU, RCCL over xGMI, TP x DP layout.

The reference has no distributed runtime at all ("no parallelism and
no collective communication anywhere"); this module is the MI355X build's
first-class replacement.  Launch contract is torchrun's: RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT in the environment (use 127.0.0.1 as the
master address on a single node).  The backend is ``nccl`` (= RCCL on ROCm) when
the process owns a GPU and ``gloo`` otherwise, so every path here also runs in
CPU tests.

Layout: ranks are split into ``world / tp`` tensor-parallel groups of consecutive
ranks ([0..tp), [tp..2tp), ...) — on an 8-GPU MI355X node every GPU pair has its
own xGMI link, so consecutive grouping costs nothing — and ``tp`` data-parallel
groups of ranks with equal TP rank.  Image services (CLIP / face / OCR) run with
tp = 1 (pure DP = 8); the VLM decoder runs tp = 8 (or 4 x dp 2).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch

_STATE: Optional["ParallelState"] = None


@dataclass
class ParallelState:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"
    tp_size: int = 1
    tp_rank: int = 0
    tp_group: object = None
    tp_ranks: tuple = (0,)
    dp_size: int = 1
    dp_rank: int = 0
    dp_group: object = None
    dp_ranks: tuple = (0,)
    owns_pg: bool = False

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def tp_info(self):
        """The decoder's TP descriptor (``models.llm.TPInfo``) for this rank."""
        from ..models.llm import TPInfo

        return TPInfo(rank=self.tp_rank, world=self.tp_size, group=self.tp_group if self.tp_size > 1 else None)


def env_world() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torchrun-style environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def _pick_backend(device: torch.device) -> str:
    """RCCL on GPUs, gloo on CPU; ``LUMEN_DIST_BACKEND`` overrides (e.g. gloo for several ranks
    sharing one GPU in tests: RCCL refuses two ranks on the same device)."""
    env = os.environ.get("LUMEN_DIST_BACKEND")
    if env:
        return env
    return "nccl" if device.type == "cuda" else "gloo"


def init_distributed(tp_size: int = 1, backend: Optional[str] = None, device: Optional[torch.device] = None,
                     timeout_s: float = 600.0, rank: Optional[int] = None, world: Optional[int] = None,
                     init_method: Optional[str] = None) -> ParallelState:
    """Initialise the default process group (if needed) and the TP / DP sub-groups.

    ``timeout_s`` bounds every collective (the RCCL watchdog turns a lost rank into
    an exception instead of a hang — SURVEY §5.3 failure detection)."""
    global _STATE
    import torch.distributed as dist

    er, ew, el = env_world()
    rank = er if rank is None else rank
    world = ew if world is None else world
    local = el if world == ew else rank
    if device is None:
        if torch.cuda.is_available():
            device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
        else:
            device = torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world % tp_size != 0:
        raise ValueError(f"world size {world} is not a multiple of tp_size {tp_size}")
    st = ParallelState(rank=rank, world=world, local_rank=local, device=device, tp_size=tp_size)
    if world > 1:
        backend = backend or _pick_backend(device)
        owns = False
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if init_method:
                kw["init_method"] = init_method
            if backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
            owns = True
        st.backend = dist.get_backend()
        st.owns_pg = owns
        # every rank must create every group, in the same order
        for g in range(world // tp_size):
            ranks = tuple(range(g * tp_size, (g + 1) * tp_size))
            pg = dist.new_group(list(ranks)) if tp_size > 1 else None
            if rank in ranks:
                st.tp_group, st.tp_ranks, st.tp_rank = pg, ranks, ranks.index(rank)
        dp = world // tp_size
        for t in range(tp_size):
            ranks = tuple(range(t, world, tp_size))
            if tp_size == 1:
                pg = dist.group.WORLD          # pure DP: reuse the default communicator
            else:
                pg = dist.new_group(list(ranks)) if dp > 1 else None
            if rank in ranks:
                st.dp_group, st.dp_ranks, st.dp_rank = pg, ranks, ranks.index(rank)
        st.dp_size = dp
    _STATE = st
    return st


def get_state() -> ParallelState:
    """Current state (a single-process state if :func:`init_distributed` was never called)."""
    global _STATE
    if _STATE is None:
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        _STATE = ParallelState(device=dev)
    return _STATE


def destroy() -> None:
    global _STATE
    import torch.distributed as dist

    st = _STATE
    _STATE = None
    if st is not None and st.owns_pg and dist.is_initialized():
        dist.destroy_process_group()
