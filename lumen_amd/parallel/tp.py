"""Tensor-parallel serving group for the VLM decoder.

The gRPC service process is TP rank 0 (the *leader*): it owns the continuous-
batching engine, tokenizer and sampling, and broadcasts every engine step.
Ranks 1..N-1 (*followers*) are child processes started here with the torchrun
environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 /
MASTER_PORT); each builds the same model with its weight shard on its own GPU
and replays the leader's steps (:func:`lumen_amd.runtime.engine.follower_loop`),
so every rank issues the same kernels and the same collectives.  Column-/row-
parallel layers all-reduce through :class:`~lumen_amd.parallel.comm.Communicator`
(IPC one-shot for decode-size messages, RCCL for prefill-size ones).

Followers are started as child processes (``subprocess``), never by exec-ing a
process that already touched the GPU.  A monitor thread watches them: if one
dies the group is marked failed and the leader's requests fail with
``ERROR_CODE_UNAVAILABLE`` instead of hanging in a collective (the collective
timeout of :func:`~lumen_amd.parallel.state.init_distributed` is the backstop).
"""
from __future__ import annotations

import json
import logging
import os
import socket
import subprocess
import sys
import threading
import time
from typing import Optional, Sequence

import torch

from .state import ParallelState, destroy, init_distributed

log = logging.getLogger("lumen.tp")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TPServingGroup:
    """Leader side: spawn follower ranks, join the process group as rank 0."""

    def __init__(self, world: int, worker_spec: dict, devices: Optional[Sequence[str]] = None,
                 port: Optional[int] = None, timeout_s: float = 600.0, worker_module: str = "lumen_amd.parallel.tp_worker"):
        if world < 2:
            raise ValueError("a TP serving group needs at least 2 ranks")
        self.world = world
        self.port = port or free_port()
        if devices is None:
            n = torch.cuda.device_count() if torch.cuda.is_available() else 0
            devices = [f"cuda:{r % n}" for r in range(world)] if n else ["cpu"] * world
        self.devices = list(devices)
        self.failed: Optional[str] = None
        self.procs: list[subprocess.Popen] = []
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        for r in range(1, world):
            env = dict(os.environ)
            env.update(RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.port),
                       LOCAL_RANK=str(r), LUMEN_TP_DEVICE=self.devices[r],
                       PYTHONPATH=root + os.pathsep + env.get("PYTHONPATH", ""))
            spec = dict(worker_spec, device=self.devices[r], timeout_s=timeout_s)
            self.procs.append(subprocess.Popen([sys.executable, "-m", worker_module, json.dumps(spec)], env=env))
        dev = torch.device(self.devices[0])
        self.state: ParallelState = init_distributed(tp_size=world, rank=0, world=world, device=dev,
                                                     timeout_s=timeout_s,
                                                     init_method=f"tcp://127.0.0.1:{self.port}")
        self._stop = threading.Event()
        self._mon = threading.Thread(target=self._watch, name="lumen-tp-monitor", daemon=True)
        self._mon.start()

    def _watch(self) -> None:
        while not self._stop.wait(0.5):
            for r, p in enumerate(self.procs, start=1):
                rc = p.poll()
                if rc is not None and not self._stop.is_set():
                    self.failed = f"TP rank {r} exited with code {rc}"
                    log.error(self.failed)
                    return

    def close(self, timeout: float = 30.0) -> None:
        """Call after the engine sent its stop message to the followers."""
        self._stop.set()
        t0 = time.time()
        for p in self.procs:
            try:
                p.wait(timeout=max(0.1, timeout - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(timeout=10)
        destroy()
