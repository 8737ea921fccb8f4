"""Parallel runtime for MI355X nodes: process groups, collectives, DP and TP.

* :mod:`.state`          — torchrun-style bootstrap, TP x DP process groups (RCCL / gloo)
* :mod:`.comm`           — :class:`Communicator` (IPC one-shot all-reduce for small
                           messages, RCCL for bulk), bucketed all-gather
* :mod:`.data_parallel`  — SPMD image-batch DP (shard + RCCL all-gather)
* :mod:`.worker_pool`    — multi-process GPU worker pool for DP serving, heartbeats,
                           respawn on failure
* :mod:`.tp`             — tensor-parallel serving group (leader + follower ranks)

The reference (EdwinZhanCN/Lumen) has no parallelism or collectives;
everything here is new, designed for 8 x MI355X over point-to-point xGMI.
"""
from .comm import BucketedAllGather, Communicator, CustomAllReduce  # noqa: F401
from .data_parallel import DataParallelRunner, shard_range  # noqa: F401
from .state import ParallelState, destroy, get_state, init_distributed  # noqa: F401
from .worker_pool import GPUWorkerPool, WorkerLostError, WorkerTaskError, default_devices  # noqa: F401
