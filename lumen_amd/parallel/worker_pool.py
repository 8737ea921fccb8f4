"""Multi-process GPU worker pool: image-batch data parallelism for serving.

The reference runs every model in the gRPC server process, batch 1, on one
device (SURVEY §2.5 DP row).  Here a service with ``LUMEN_DP_SIZE = N`` owns N
worker processes, one per GPU (each its own HIP context, caching allocator and
stream — no GIL or allocator contention between GPUs).  The service's dynamic
batcher runs several dispatcher threads (``concurrency``), each handing a whole merged
batch to :meth:`GPUWorkerPool.submit` (least in-flight worker), so every GPU has up to
two batches queued: host decode / transfer of the next batch overlaps the current one.
:meth:`GPUWorkerPool.run` (split one batch into per-worker shards) stays for SPMD-style
callers.  Payloads move through per-worker shared-memory rings created by the pool
(``shm_slots`` x ``shm_slot_bytes`` each way), never pickled through the pipe:

* inputs that are a list of ``bytes`` (compressed images): the pool packs the batch into
  the next free input slot (a semaphore counts free slots, the worker releases a slot once
  it has copied the batch out) and sends only the offsets;
* results that are a list of equally shaped numpy rows (embeddings): the worker writes the
  stacked array into the next free result slot, the pool copies it out and releases it.

Anything else (token ids, small results, a batch larger than a slot) travels pickled.
Each spawn of a worker gets a new generation number and fresh rings; ring descriptors
carry the generation, so a message a dead worker left queued is dropped instead of
reading (or releasing a slot of) a ring that no longer exists.

Failure detection: every worker sends a heartbeat each
``heartbeat_s``; the monitor thread declares a worker lost when its process exits
or its heartbeat is older than ``dead_after_s``, fails that worker's in-flight
shards with :class:`WorkerLostError` (the services map it to
``ERROR_CODE_UNAVAILABLE``) and respawns it.  ``LUMEN_FAULT_KILL_WORKER=w:n``
makes worker w exit hard after n tasks (fault-injection tests).

Workers are started with the ``spawn`` context (a fresh interpreter started as a
child process, never an exec of a GPU-initialised process) and pinned to their
device before the factory builds the model.
"""
from __future__ import annotations

import importlib
import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time
import traceback
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Optional, Sequence

log = logging.getLogger("lumen.workers")


class WorkerLostError(RuntimeError):
    """A worker process died (or stopped heart-beating) with work in flight."""


class WorkerTaskError(RuntimeError):
    """The worker's batch function raised; carries the remote traceback."""


_SHM_MIN_BYTES = 64 * 1024      # smaller results are cheaper to pickle


def _resolve(path: str) -> Callable:
    mod, _, attr = path.partition(":")
    return getattr(importlib.import_module(mod), attr)


def _fault_plan(wid: int) -> Optional[int]:
    spec = os.environ.get("LUMEN_FAULT_KILL_WORKER", "")
    if not spec:
        return None
    w, _, n = spec.partition(":")
    return int(n or 0) if int(w) == wid else None


def _as_rows(res):
    """A result that is a list of equally shaped numpy arrays -> one stacked array, else None."""
    try:
        import numpy as np
    except ImportError:  # pragma: no cover
        return None
    if not isinstance(res, list) or not res or not all(isinstance(r, np.ndarray) for r in res):
        return None
    r0 = res[0]
    if r0.dtype.hasobject or any(r.shape != r0.shape or r.dtype != r0.dtype for r in res):
        return None
    return np.stack(res)


class _ShmRing:
    """Worker side of a ring: slot k of ``nslots`` at offset k * slot_bytes."""

    def __init__(self, name: str, nslots: int, slot_bytes: int, free_sem, gen: int):
        from multiprocessing import shared_memory

        self.shm = shared_memory.SharedMemory(name=name)
        self.nslots, self.slot_bytes, self.free, self.gen = nslots, slot_bytes, free_sem, gen
        self.next = 0

    def put(self, arr):
        import numpy as np

        if arr.nbytes > self.slot_bytes:
            return None
        self.free.acquire()
        slot = self.next
        self.next = (self.next + 1) % self.nslots
        dst = np.ndarray(arr.shape, arr.dtype, buffer=self.shm.buf, offset=slot * self.slot_bytes)
        dst[...] = arr
        return self.gen, slot, arr.shape, arr.dtype.str

    def take(self, desc) -> list:
        """Input ring: copy the batch of ``bytes`` items out of its slot, then free the slot."""
        _gen, slot, ends = desc
        base = slot * self.slot_bytes
        buf = self.shm.buf
        out, a = [], 0
        for b in ends:
            out.append(bytes(buf[base + a:base + b]))
            a = b
        self.free.release()
        return out


def _as_blobs(items) -> Optional[list]:
    """Cumulative end offsets when ``items`` is a non-empty list of bytes-like objects."""
    if not isinstance(items, list) or not items or not all(isinstance(x, (bytes, bytearray, memoryview)) for x in items):
        return None
    ends, t = [], 0
    for x in items:
        t += len(x)
        ends.append(t)
    return ends


def _worker_main(wid: int, device: str, factory: str, kwargs: dict, inq, outq, heartbeat_s: float,
                 shm: Optional[tuple] = None, shm_in: Optional[tuple] = None) -> None:
    """Child process body: pin device, build the batch fn, serve tasks until None."""
    ring = in_ring = None
    try:
        if device.startswith("cuda"):
            import torch

            torch.cuda.set_device(torch.device(device))
        fac = _resolve(factory)
        kw = dict(kwargs)
        pool_world = int(kw.pop("_pool_world", 1))
        import inspect

        params = inspect.signature(fac).parameters
        if "rank" in params and "rank" not in kw:      # sharded workers (e.g. a label-bank shard)
            kw["rank"] = wid
        if "world" in params and "world" not in kw:
            kw["world"] = pool_world
        fn = fac(device, **kw)
        if shm is not None:
            ring = _ShmRing(*shm)
        if shm_in is not None:
            in_ring = _ShmRing(*shm_in)
    except BaseException:  # noqa: BLE001
        outq.put(("fatal", wid, None, traceback.format_exc()))
        return
    outq.put(("ready", wid, None, os.getpid()))
    kill_after = _fault_plan(wid)
    done = 0
    alive = threading.Event()

    def beat():   # heart-beats keep flowing while a long batch runs
        while not alive.wait(heartbeat_s):
            outq.put(("hb", wid, None, time.time()))

    threading.Thread(target=beat, name="lumen-worker-hb", daemon=True).start()
    while True:
        msg = inq.get()
        if msg is None:
            alive.set()
            break
        tid, kind, items, in_desc = msg
        if kill_after is not None and done >= kill_after:
            os._exit(17)
        try:
            if in_desc is not None:
                items = in_ring.take(in_desc)
            res = fn(kind, items)
            arr = _as_rows(res) if ring is not None else None
            desc = ring.put(arr) if arr is not None and arr.nbytes >= _SHM_MIN_BYTES else None
            if desc is not None:
                outq.put(("okshm", wid, tid, desc))
            else:
                outq.put(("ok", wid, tid, res))
        except BaseException:  # noqa: BLE001
            outq.put(("err", wid, tid, traceback.format_exc()))
        done += 1


@dataclass
class _Worker:
    wid: int
    device: str
    proc: Any = None
    inq: Any = None
    ready: bool = False
    pid: int = 0
    last_hb: float = 0.0
    inflight: dict = field(default_factory=dict)   # tid -> (Future, submit time)
    restarts: int = 0
    shm: Any = None          # SharedMemory of the result ring (owned by the pool)
    shm_free: Any = None     # semaphore: free slots of the result ring
    shm_in: Any = None       # SharedMemory of the input ring (owned by the pool)
    shm_in_free: Any = None  # semaphore: free slots of the input ring
    in_next: int = 0         # next input slot the pool fills
    in_lock: Any = field(default_factory=threading.Lock)   # orders slot fill + enqueue per worker
    gen: int = 0             # spawn generation (tags ring descriptors)


class GPUWorkerPool:
    """N worker processes, one per device, running ``factory(device, **kwargs)``'s
    batch function ``fn(kind, items) -> list``."""

    def __init__(self, factory: str, devices: Sequence[str], kwargs: Optional[dict] = None, heartbeat_s: float = 1.0,
                 dead_after_s: float = 30.0, respawn: bool = True, start_timeout_s: float = 600.0,
                 task_timeout_s: Optional[float] = None, shm_slots: int = 4, shm_slot_bytes: int = 8 << 20):
        self.factory = factory
        self.shm_slots = int(shm_slots)
        self.shm_slot_bytes = int(shm_slot_bytes)
        self.kwargs = dict(kwargs or {})
        self.heartbeat_s = heartbeat_s
        self.dead_after_s = dead_after_s
        self.respawn = respawn
        self.task_timeout_s = task_timeout_s   # a batch running longer => the worker is hung: kill + respawn
        self._ctx = mp.get_context("spawn")
        self._outq = self._ctx.Queue()
        self._lock = threading.Lock()
        self._tid = itertools.count(1)
        self._stop = threading.Event()
        self.workers = [_Worker(wid=i, device=d) for i, d in enumerate(devices)]
        self.stats = {"tasks": 0, "items": 0, "lost": 0, "restarts": 0, "shm_results": 0, "shm_inputs": 0,
                      "stale_dropped": 0}
        self._gen = itertools.count(1)
        self._fatal: Optional[str] = None
        for w in self.workers:
            self._start(w)
        self._collector = threading.Thread(target=self._collect, name="lumen-pool-collect", daemon=True)
        self._collector.start()
        self._monitor = threading.Thread(target=self._watch, name="lumen-pool-monitor", daemon=True)
        self._monitor.start()
        self.wait_ready(start_timeout_s)

    # ------------------------------------------------------------------ lifecycle
    def _start(self, w: _Worker) -> None:
        """(Re)spawn worker w with fresh rings; the caller holds ``self._lock`` on a restart."""
        w.inq = self._ctx.Queue()
        w.ready = False
        w.last_hb = time.time()
        w.gen = next(self._gen)
        w.in_next = 0
        kwargs = dict(self.kwargs)
        kwargs.setdefault("_pool_world", len(self.workers))
        self._free_shm(w)
        shm = shm_in = None
        if self.shm_slots > 0:
            from multiprocessing import shared_memory

            try:
                w.shm = shared_memory.SharedMemory(create=True, size=self.shm_slots * self.shm_slot_bytes)
                w.shm_free = self._ctx.Semaphore(self.shm_slots)
                shm = (w.shm.name, self.shm_slots, self.shm_slot_bytes, w.shm_free, w.gen)
                w.shm_in = shared_memory.SharedMemory(create=True, size=self.shm_slots * self.shm_slot_bytes)
                w.shm_in_free = self._ctx.Semaphore(self.shm_slots)
                shm_in = (w.shm_in.name, self.shm_slots, self.shm_slot_bytes, w.shm_in_free, w.gen)
            except OSError as e:   # no /dev/shm space: payloads travel pickled
                log.warning("worker %d: no shared-memory rings (%s)", w.wid, e)
                self._free_shm(w)
                shm = shm_in = None
        w.proc = self._ctx.Process(target=_worker_main, name=f"lumen-worker-{w.wid}",
                                   args=(w.wid, w.device, self.factory, kwargs, w.inq, self._outq,
                                         self.heartbeat_s, shm, shm_in), daemon=True)
        w.proc.start()

    @staticmethod
    def _free_shm(w: _Worker) -> None:
        for name in ("shm", "shm_in"):
            seg = getattr(w, name)
            if seg is not None:
                try:
                    seg.close()
                except Exception:  # noqa: BLE001 - e.g. BufferError with views alive; still unlink
                    pass
                try:
                    seg.unlink()
                except Exception:  # noqa: BLE001
                    pass
        w.shm = w.shm_free = w.shm_in = w.shm_in_free = None

    def wait_ready(self, timeout: float) -> None:
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self._fatal:
                self.close()
                raise RuntimeError(f"worker failed to start:\n{self._fatal}")
            if all(w.ready for w in self.workers):
                return
            time.sleep(0.05)
        raise TimeoutError("GPU workers did not become ready")

    def close(self) -> None:
        if self._stop.is_set():
            return
        self._stop.set()
        for w in self.workers:
            try:
                w.inq.put(None)
            except Exception:  # noqa: BLE001
                pass
        self._monitor.join(timeout=5)
        for w in self.workers:
            proc = w.proc
            if proc is not None:
                proc.join(timeout=10)
                if proc.is_alive():
                    proc.kill()
                    proc.join(timeout=5)
        with self._lock:
            for w in self.workers:
                for fut, _ in w.inflight.values():
                    if not fut.done():
                        fut.set_exception(WorkerLostError("pool closed"))
                w.inflight.clear()
        self._collector.join(timeout=2)
        for w in self.workers:
            with w.in_lock:
                self._free_shm(w)

    @property
    def size(self) -> int:
        return len(self.workers)

    def live(self) -> list[_Worker]:
        return [w for w in self.workers if w.ready and w.proc is not None and w.proc.is_alive()]

    # ------------------------------------------------------------------ submit
    def submit(self, kind: str, items: list, worker: Optional[int] = None) -> Future:
        """One task on one worker (least in-flight unless ``worker`` is given)."""
        fut: Future = Future()
        with self._lock:
            cands = self.live()
            if not cands:
                fut.set_exception(WorkerLostError("no live GPU worker"))
                return fut
            w = self.workers[worker] if worker is not None else min(cands, key=lambda x: len(x.inflight))
            tid = next(self._tid)
            w.inflight[tid] = (fut, time.time())
            self.stats["tasks"] += 1
            self.stats["items"] += len(items)
            gen, seg, free, inq = w.gen, w.shm_in, w.shm_in_free, w.inq
        ends = _as_blobs(items) if seg is not None else None
        if ends is None or ends[-1] > self.shm_slot_bytes:
            inq.put((tid, kind, items, None))
            return fut
        # input ring: wait for a free slot OUTSIDE the pool lock (back-pressure on this caller
        # only); the per-worker lock keeps slot order == queue order, which the worker relies on
        with w.in_lock:
            while not free.acquire(timeout=0.5):
                if self._stop.is_set() or w.gen != gen:   # worker respawned: its ring is gone
                    return fut                            # (the future was failed by the monitor)
            if w.gen != gen:
                return fut
            slot = w.in_next
            w.in_next = (slot + 1) % self.shm_slots
            base, a = slot * self.shm_slot_bytes, 0
            buf = seg.buf
            for x, b in zip(items, ends):
                buf[base + a:base + b] = x
                a = b
            inq.put((tid, kind, None, (gen, slot, ends)))
        with self._lock:
            self.stats["shm_inputs"] += 1
        return fut

    def broadcast(self, kind: str, items: list, timeout: Optional[float] = None) -> list:
        """The same task on EVERY worker (in worker order) — sharded state such as a
        label-bank shard per GPU; fails if a worker is not live (its shard is missing)."""
        futs = [self.submit(kind, list(items), worker=w.wid) for w in self.workers]
        return [f.result(timeout) for f in futs]

    def run(self, kind: str, items: Sequence, timeout: Optional[float] = None) -> list:
        """Split ``items`` into one contiguous shard per live worker; ordered results."""
        items = list(items)
        if not items:
            return []
        n = max(1, min(len(self.live()) or 1, len(items)))
        per = -(-len(items) // n)
        futs = [self.submit(kind, items[i:i + per]) for i in range(0, len(items), per)]
        out: list = []
        for f in futs:
            out.extend(f.result(timeout))
        return out

    # ------------------------------------------------------------------ background threads
    def _collect(self) -> None:
        while not self._stop.is_set():
            try:
                kind, wid, tid, payload = self._outq.get(timeout=0.2)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                break
            try:
                self._handle(kind, wid, tid, payload)
            except Exception:  # noqa: BLE001 -- one bad message must not kill the collector
                log.exception("worker pool: dropping message %r from worker %s", kind, wid)

    def _handle(self, kind, wid, tid, payload) -> None:
        w = self.workers[wid]
        with self._lock:
            w.last_hb = time.time()
            if kind == "ready":
                w.ready, w.pid = True, int(payload)
            elif kind == "fatal":
                self._fatal = str(payload)
            elif kind == "okshm":
                if payload[0] != w.gen or w.shm is None:   # from a previous spawn: ring is gone
                    self.stats["stale_dropped"] += 1
                    return
                payload = self._read_shm(w, payload)
                self.stats["shm_results"] += 1
                kind = "ok"
            if kind in ("ok", "err"):
                fut, _ = w.inflight.pop(tid, (None, 0.0))
                if fut is not None and not fut.done():
                    if kind == "ok":
                        fut.set_result(payload)
                    else:
                        fut.set_exception(WorkerTaskError(str(payload)))

    def _read_shm(self, w: _Worker, desc) -> list:
        """Copy a result out of worker w's ring slot and release the slot (messages of one
        worker arrive in order, so slots are consumed in the order the worker filled them)."""
        import numpy as np

        _gen, slot, shape, dt = desc
        arr = np.ndarray(shape, np.dtype(dt), buffer=w.shm.buf, offset=slot * self.shm_slot_bytes).copy()
        w.shm_free.release()
        return list(arr)

    def _watch(self) -> None:
        while not self._stop.wait(self.heartbeat_s / 2):
            now = time.time()
            for w in self.workers:
                if w.proc is None or self._stop.is_set():
                    continue
                dead = not w.proc.is_alive()
                stale = w.ready and now - w.last_hb > self.dead_after_s
                if self.task_timeout_s is not None and w.ready:
                    with self._lock:
                        oldest = min((t for _, t in w.inflight.values()), default=now)
                    stale = stale or now - oldest > self.task_timeout_s
                if not (dead or stale):
                    continue
                with self._lock:
                    lost = [f for f, _ in w.inflight.values()]
                    w.inflight.clear()
                    w.ready = False
                    self.stats["lost"] += 1
                for fut in lost:
                    if not fut.done():
                        fut.set_exception(WorkerLostError(f"GPU worker {w.wid} ({w.device}) lost"))
                log.error("GPU worker %d on %s lost (%s)", w.wid, w.device, "exited" if dead else "no heartbeat")
                if stale and w.proc.is_alive():
                    w.proc.kill()
                w.proc.join(timeout=5)
                if self.respawn and not self._stop.is_set():
                    with self._lock:
                        w.gen = 0      # a submit waiting for an input slot sees the ring retired
                    # the input ring is replaced under its fill lock (no submit mid-copy into it),
                    # and the collector reads w.shm / w.gen under the pool lock
                    with w.in_lock, self._lock:
                        w.restarts += 1
                        self.stats["restarts"] += 1
                        self._start(w)
                else:
                    w.proc = None


def default_devices(n: int) -> list[str]:
    """n device strings: cuda:0..n-1 when GPUs are present, else n CPU workers."""
    try:
        import torch

        cnt = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        cnt = 0
    if cnt:
        return [f"cuda:{i % cnt}" for i in range(n)]
    return ["cpu"] * n


# ---------------------------------------------------------------------- test/bench factories
def echo_factory(device: str, scale: float = 1.0):
    """Worker that returns scale * sum(item) per item (pool plumbing tests)."""
    import numpy as np

    def fn(kind, items):
        if kind == "fail":
            raise ValueError("requested failure")
        if kind == "sleep":
            time.sleep(float(items[0]))
            return [0.0]
        return [float(np.sum(x)) * scale for x in items]

    return fn
