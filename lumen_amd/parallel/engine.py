"""One GPU engine process per device, fed by many serving front-end processes.

The reference serves everything from one process on a 10-thread gRPC pool, batch 1
(``src/lumen/server.py:232-235``).  Round 3 scaled serving by running N full hub replicas per
GPU (N copies of every model, N independent batchers).  Here the serving stack splits in two:

* **front ends** (K processes, ``hub.server.serve(frontends=K)``): gRPC accept, chunk reassembly,
  JPEG decode, tokenisation and the service logic -- the Python-bound work that one
  interpreter lock would serialise -- each running the normal service classes whose backends
  see a :class:`RemotePool` where a GPU worker pool would be;
* **engines** (one process per GPU, :func:`engine_main`): the models, and a batch loop per
  service that pops whatever requests ALL front ends have queued on that service's
  :class:`~lumen_amd.parallel.shm_channel.ShmChannel` (futex wait, then a short linger), runs
  them as one device batch through the service's GPU-worker factory (the same
  ``fn(kind, items)`` the DP worker pool runs) and completes each request slot.

A request slot carries one front-end batch (pickled item list; images arrive decoded), so a
front end pays one channel round trip per batch while the engine merges batches of every
front end.  Engines heart-beat into the channel; the :class:`EngineSet` supervisor respawns a
dead engine, whose restart fails the requests it had taken (front ends see
:class:`~lumen_amd.parallel.worker_pool.WorkerLostError` -> gRPC UNAVAILABLE) while queued ones
wait for the new engine.
"""
from __future__ import annotations

import importlib
import inspect
import logging
import multiprocessing as mp
import os
import pickle
import threading
import time
import traceback
from concurrent.futures import Future, ThreadPoolExecutor
from contextlib import contextmanager
from typing import Optional, Sequence

from .shm_channel import ChannelError, ChannelGroup, ChannelSpec, EngineUnavailable, ShmChannel
from .worker_pool import WorkerLostError, WorkerTaskError

log = logging.getLogger("lumen.engine")

KINDS = ("call",)          # every request is one pickled (kind, items) batch


def _resolve(path: str):
    mod, _, attr = path.partition(":")
    return getattr(importlib.import_module(mod), attr)


# ============================================================================ front-end side
class RemotePool:
    """Stand-in for :class:`~lumen_amd.parallel.worker_pool.GPUWorkerPool` inside a front-end
    process: ``submit(kind, items)`` ships the batch to the least-loaded engine of the service."""

    def __init__(self, group: ChannelGroup, info: Optional[dict] = None, timeout_s: float = 300.0,
                 max_inflight: int = 64):
        self.group = group
        self.info = info or {}
        self.timeout_s = timeout_s
        self._ex = ThreadPoolExecutor(max_workers=max_inflight, thread_name_prefix="lumen-remote")
        self.stats = {"tasks": 0, "items": 0, "split": 0}

    @property
    def size(self) -> int:
        return len(self.group.channels)

    def _call(self, kind: str, items: list) -> list:
        blob = pickle.dumps((kind, items), protocol=pickle.HIGHEST_PROTOCOL)
        ch = self.group.pick()
        if len(blob) > ch.slot_bytes and len(items) > 1:      # split a batch larger than a slot
            self.stats["split"] += 1
            h = len(items) // 2
            return self._call(kind, items[:h]) + self._call(kind, items[h:])
        try:
            res = ch.call("call", blob, timeout=self.timeout_s)
        except EngineUnavailable as e:
            raise WorkerLostError(str(e)) from e
        except ChannelError as e:
            msg = str(e)
            if msg.startswith("engine restarted"):
                raise WorkerLostError(msg) from e
            raise WorkerTaskError(msg) from e
        out = pickle.loads(res)
        if isinstance(out, BaseException):
            raise out
        return out

    def submit(self, kind: str, items: list, worker: Optional[int] = None) -> Future:
        self.stats["tasks"] += 1
        self.stats["items"] += len(items)
        return self._ex.submit(self._call, kind, list(items))

    def run(self, kind: str, items: Sequence, timeout: Optional[float] = None) -> list:
        return self.submit(kind, list(items)).result(timeout)

    def stream(self, kind: str, item):
        """Generator over ONE streaming request (the engine factory lists ``kind`` in its
        ``solo_kinds``): yields every partial object the engine emits as it lands and returns the
        final result (``final = yield from pool.stream(...)``).  Closing it early abandons the
        request on the engine."""
        blob = pickle.dumps((kind, [item]), protocol=pickle.HIGHEST_PROTOCOL)
        ch = self.group.pick()
        self.stats["tasks"] += 1
        self.stats["items"] += 1
        try:
            for tag, val in ch.call_stream("call", blob, timeout=self.timeout_s):
                if tag == "partial":
                    yield pickle.loads(val)
                    continue
                out = pickle.loads(val)
                if isinstance(out, BaseException):
                    raise out
                if isinstance(out[0], BaseException):
                    raise out[0]
                return out[0]
        except EngineUnavailable as e:
            raise WorkerLostError(str(e)) from e
        except ChannelError as e:
            msg = str(e)
            if msg.startswith("engine restarted"):
                raise WorkerLostError(msg) from e
            raise WorkerTaskError(msg) from e

    def broadcast(self, kind: str, items: list, timeout: Optional[float] = None) -> list:
        futs = []
        for ch in self.group.channels:
            g = ChannelGroup([ch])
            futs.append(self._ex.submit(RemotePool(g, self.info, self.timeout_s, 1)._call, kind, list(items)))
        return [f.result(timeout) for f in futs]

    def close(self) -> None:
        self._ex.shutdown(wait=False)

    def prefixed(self, prefix: str) -> "PrefixedRemote":
        """A view of this pool for one model of a multi-model service (SmartCLIP: general CLIP +
        BioCLIP on one engine, :func:`multi_worker`): every kind is sent as ``prefix:kind``."""
        return PrefixedRemote(self, prefix)


class PrefixedRemote:
    """:class:`RemotePool` facade whose task kinds carry a model prefix (see :func:`multi_worker`)."""

    def __init__(self, pool: RemotePool, prefix: str):
        self.pool = pool
        self.prefix = prefix
        self.info = pool.info

    @property
    def size(self) -> int:
        return self.pool.size

    def submit(self, kind: str, items: list, worker: Optional[int] = None) -> Future:
        return self.pool.submit(f"{self.prefix}:{kind}", items, worker)

    def run(self, kind: str, items: Sequence, timeout: Optional[float] = None) -> list:
        return self.pool.run(f"{self.prefix}:{kind}", items, timeout)

    def stream(self, kind: str, item):
        return (yield from self.pool.stream(f"{self.prefix}:{kind}", item))

    def broadcast(self, kind: str, items: list, timeout: Optional[float] = None) -> list:
        return self.pool.broadcast(f"{self.prefix}:{kind}", items, timeout)

    def close(self) -> None:       # the shared pool is closed by its owner
        pass


def is_remote(pool) -> bool:
    return isinstance(pool, (RemotePool, PrefixedRemote))


def _call_factory(path: str, device: str, kwargs: dict, rank: int, world: int):
    fac = _resolve(path)
    kw = dict(kwargs)
    params = inspect.signature(fac).parameters
    if "rank" in params and "rank" not in kw:
        kw["rank"] = rank
    if "world" in params and "world" not in kw:
        kw["world"] = world
    return fac(device, **kw)


def multi_worker(device: str, parts: dict, rank: int = 0, world: int = 1):
    """Engine factory of a multi-model service: ``parts`` = name -> (factory path, kwargs); the
    batch function routes kind ``name:kind`` to that part's function (the front end's backends talk
    to it through :meth:`RemotePool.prefixed`)."""
    fns = {name: _call_factory(path, device, kw, rank, world) for name, (path, kw) in parts.items()}

    def fn(kind, items):
        name, sep, sub = kind.partition(":")
        if not sep or name not in fns:
            raise ValueError(f"multi-model engine: unknown kind {kind!r} (parts {list(fns)})")
        return fns[name](sub, items)

    solo = tuple(f"{name}:{k}" for name, f in fns.items() for k in getattr(f, "solo_kinds", ()))
    if solo:
        def stream(kind, item, emit):
            name, _, sub = kind.partition(":")
            return fns[name].stream(sub, item, emit)

        fn.stream, fn.solo_kinds = stream, solo
    return fn


_REMOTE: dict = {}
_scope = threading.local()


def install_remote(service: str, pool: RemotePool) -> None:
    _REMOTE[service] = pool


@contextmanager
def remote_scope(service: Optional[str]):
    """While building service ``service`` in a front end, backends find its RemotePool."""
    prev = getattr(_scope, "name", None)
    _scope.name = service
    try:
        yield
    finally:
        _scope.name = prev


def current_remote() -> Optional[RemotePool]:
    name = getattr(_scope, "name", None)
    return _REMOTE.get(name) if name is not None else None


# ============================================================================ engine side
_stats_lock = threading.Lock()


def _run_solo(ch: ShmChannel, fn, slot: int, kind: str, items: list, stats: dict) -> None:
    """One slot of a ``solo`` kind on its own thread: ``fn.stream(kind, item, emit)`` per item, each
    ``emit(obj)`` appending a partial record the front end receives at once (False once the front
    end abandoned the request); the slot completes on its own, not with a merged batch."""
    def emit(obj) -> bool:
        return ch.partial(slot, pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)) != -2

    try:
        t0 = time.perf_counter()
        res = []
        for it in items:
            try:
                res.append(fn.stream(kind, it, emit))
            except Exception as e:  # noqa: BLE001 - reported per request
                res.append(e)
        with _stats_lock:
            stats["fn_s"] = stats.get("fn_s", 0.0) + time.perf_counter() - t0
            stats["solo"] = stats.get("solo", 0) + 1
            stats["items"] = stats.get("items", 0) + len(items)
            stats["slots"] = stats.get("slots", 0) + 1
        ch.complete(slot, pickle.dumps(res, protocol=pickle.HIGHEST_PROTOCOL))
    except Exception:  # noqa: BLE001 - e.g. an unpicklable result
        ch.complete(slot, error=traceback.format_exc()[-4000:])


def _serve_channel(ch: ShmChannel, fn, stop: threading.Event, max_items: int, linger_us: int,
                   stats: dict, solo_ex: Optional[ThreadPoolExecutor] = None, device: Optional[str] = None) -> None:
    """Batch loop over one channel: pop queued front-end batches, merge by kind, run, complete.
    Kinds the factory lists in ``fn.solo_kinds`` (a VLM's generations) are not merged: each slot
    runs on ``solo_ex`` and may stream partial results.  On a GPU every batch loop issues on a HIP
    stream of its own: the loops' batches overlap on the device, and one loop's host waits (a D2H
    of detections, an embedding copy) wait for its own kernels only, not for the other loop's."""
    # (r6 A/B through serve_bench, profiles/r6_serve_thread_streams_v1.txt: face 2,437 -> 2,664 img/s,
    # CLIP 3,150 -> 3,220 img/s)
    if device is not None and device.startswith("cuda"):
        import torch

        from ..ops import private_stream

        with torch.cuda.stream(private_stream(torch.device(device))):
            return _serve_channel(ch, fn, stop, max_items, linger_us, stats, solo_ex, None)
    solo = set(getattr(fn, "solo_kinds", ()))
    while not stop.is_set():
        slots = ch.pop_batch(ch.nslots, wait_ms=100, linger_us=linger_us)
        if not slots:
            continue
        groups: dict = {}
        for s in slots:
            try:
                _kind, blob, _meta = ch.request(s)
                kind, items = pickle.loads(bytes(blob))
                if kind == "__stats__":        # engine counters (tests, tools/serve_bench.py)
                    with _stats_lock:
                        snap = dict(stats)
                    ch.complete(s, pickle.dumps([snap]))
                    continue
                if kind in solo and solo_ex is not None:
                    solo_ex.submit(_run_solo, ch, fn, s, kind, items, stats)
                    continue
                groups.setdefault(kind, []).append((s, items))
            except Exception as e:  # noqa: BLE001 - a bad request fails alone
                ch.complete(s, error=f"bad request: {e}")
        for kind, reqs in groups.items():
            fronts = len({ch.tag(s) >> 32 for s, _ in reqs})
            flat = [it for _, items in reqs for it in items]
            try:
                res: list = []
                t0 = time.perf_counter()
                for i in range(0, len(flat), max_items):
                    res.extend(fn(kind, flat[i:i + max_items]))
                with _stats_lock:
                    stats["fn_s"] = stats.get("fn_s", 0.0) + time.perf_counter() - t0
                    stats["batches"] = stats.get("batches", 0) + 1
                    stats["batch_items"] = stats.get("batch_items", 0) + len(flat)
                    stats["items"] = stats.get("items", 0) + len(flat)
                    stats["slots"] = stats.get("slots", 0) + len(reqs)
                    stats["max_frontends_per_batch"] = max(stats.get("max_frontends_per_batch", 0), fronts)
                    if fronts > 1:
                        stats["shared_batches"] = stats.get("shared_batches", 0) + 1
                if len(res) != len(flat):
                    raise RuntimeError(f"engine fn returned {len(res)} results for {len(flat)} items")
            except Exception:  # noqa: BLE001 - the whole merged batch failed
                msg = traceback.format_exc()
                for s, _ in reqs:
                    ch.complete(s, error=msg[-4000:])
                continue
            k = 0
            for s, items in reqs:
                part = res[k:k + len(items)]
                k += len(items)
                try:
                    ch.complete(s, pickle.dumps(part, protocol=pickle.HIGHEST_PROTOCOL))
                except Exception as e:  # noqa: BLE001 - e.g. a result larger than the slot
                    ch.complete(s, error=f"result: {e}")


def engine_main(services: dict, device: str, ready_q, stop_ev, max_items: int = 256, linger_us: int = 1500,
                threads_per_service: int = 2, rank: int = 0, world: int = 1) -> None:
    """Engine process body.  ``services``: name -> (ChannelSpec, factory path, kwargs[, options]).
    Pins the device, builds every service's batch function (factories taking ``rank`` / ``world``
    get this engine's index / the engine count: a label bank is sharded over the engines), then
    serves each channel with ``threads_per_service`` batch loops (one batch's host work overlaps the
    other's GPU work; a service's ``options["threads"]`` overrides it -- a continuous-batching
    service keeps one loop per request in flight)."""
    try:
        if device.startswith("cuda"):
            import torch

            torch.cuda.set_device(torch.device(device))
        chans, fns, nthreads, opts_of = {}, {}, {}, {}
        for name, entry in services.items():
            spec, factory, kwargs = entry[:3]
            opts = entry[3] if len(entry) > 3 else {}
            opts_of[name] = opts
            ch = ShmChannel.attach(spec)
            fns[name] = _call_factory(factory, device, kwargs, rank, world)
            chans[name] = ch
            nthreads[name] = int(opts.get("threads", threads_per_service))
        for ch in chans.values():
            failed = ch.engine_start()
            if failed:
                log.warning("engine on %s: failed %d request(s) left running by a previous engine", device, failed)
            ch.register_host()
    except BaseException:  # noqa: BLE001
        ready_q.put(("fatal", device, traceback.format_exc()))
        return
    stop = threading.Event()
    stats: dict = {}
    ths = []
    solo_exs = []
    for name, ch in chans.items():
        sx = None
        if getattr(fns[name], "solo_kinds", ()):
            # one thread per request in flight (a continuous-batching engine holds many at once)
            sx = ThreadPoolExecutor(max_workers=int(opts_of[name].get("solo_threads", 64)),
                                    thread_name_prefix=f"lumen-solo-{name}")
            solo_exs.append(sx)
        # a solo service's requests never merge, so waiting for more to arrive only delays them
        lg = 0 if sx is not None else linger_us
        for i in range(nthreads[name]):
            t = threading.Thread(target=_serve_channel, args=(ch, fns[name], stop, max_items, lg, stats, sx, device),
                                 name=f"lumen-engine-{name}-{i}", daemon=True)
            t.start()
            ths.append(t)
    ready_q.put(("ready", device, os.getpid()))
    from ..utils.sampler import maybe_start

    stop_sampler = maybe_start(f"engine-{device.replace(':', '')}")   # LUMEN_SAMPLE_DIR
    # stop_ev: a shared byte, polled (an mp.Event's set() blocks on a waiter that died in its wait)
    every = float(os.environ.get("LUMEN_ENGINE_STATS_S", "0") or 0)    # periodic load log (serving benches)
    t_log, last = time.perf_counter(), {}
    while not stop_ev.value:
        for ch in chans.values():
            ch.heartbeat()
        time.sleep(0.25)
        if every > 0 and time.perf_counter() - t_log >= every:
            now = time.perf_counter()
            with _stats_lock:
                cur = dict(stats)
            dt = now - t_log
            db = cur.get("batches", 0) - last.get("batches", 0)
            di = cur.get("batch_items", 0) - last.get("batch_items", 0)
            busy = (cur.get("fn_s", 0.0) - last.get("fn_s", 0.0)) / dt
            log.warning("engine %s: %.0f items/s, %.1f batches/s, %.1f items/batch, batch-fn busy %.2f "
                        "(loops x fraction), shared batches %d", device, di / dt, db / dt, di / max(db, 1), busy,
                        cur.get("shared_batches", 0))
            t_log, last = now, cur
    stop.set()
    for t in ths:
        t.join(timeout=5)
    for sx in solo_exs:
        sx.shutdown(wait=False, cancel_futures=True)
    stop_sampler()


class EngineSet:
    """Launcher side: one channel per (service, engine), one engine process per device,
    supervision (a dead engine is respawned on the same channels)."""

    def __init__(self, services: dict, devices: Sequence[str], nslots: int = 64, slot_bytes: int = 32 << 20,
                 result_bytes: int = 4 << 20, start_timeout_s: float = 900.0, respawn: bool = True,
                 threads_per_service: int = 2, linger_us: int = 1500, max_items: int = 256):
        """``services``: name -> (factory path, kwargs[, options])."""
        self.services = dict(services)
        self.loop_args = (max_items, linger_us, threads_per_service)
        self.devices = list(devices)
        self.respawn = respawn
        self._ctx = mp.get_context("spawn")
        self._ready = self._ctx.Queue()
        self._stop = self._ctx.Value("b", 0, lock=False)
        self.channels: dict = {name: [ShmChannel.create(f"{name}-{i}", KINDS, nslots, slot_bytes, result_bytes)
                                      for i in range(len(self.devices))] for name in self.services}
        self.procs: list = [None] * len(self.devices)
        self.restarts = 0
        for i in range(len(self.devices)):
            self._spawn(i)
        self._wait_ready(len(self.devices), start_timeout_s)
        self._mon_stop = threading.Event()
        self._mon = threading.Thread(target=self._monitor, name="lumen-engine-monitor", daemon=True)
        self._mon.start()

    def _spawn(self, i: int) -> None:
        svc = {name: (self.channels[name][i].spec(), *entry) for name, entry in self.services.items()}
        p = self._ctx.Process(target=engine_main, args=(svc, self.devices[i], self._ready, self._stop, *self.loop_args,
                                                        i, len(self.devices)),
                              name=f"lumen-engine-{i}", daemon=False)
        p.start()
        self.procs[i] = p

    def _wait_ready(self, n: int, timeout: float) -> None:
        t0 = time.time()
        got = 0
        while got < n:
            left = timeout - (time.time() - t0)
            if left <= 0:
                raise TimeoutError("GPU engines did not become ready")
            kind, dev, payload = self._ready.get(timeout=left)
            if kind == "fatal":
                self.close()
                raise RuntimeError(f"engine on {dev} failed to start:\n{payload}")
            got += 1

    def _monitor(self) -> None:
        while not self._mon_stop.wait(1.0):
            for i, p in enumerate(self.procs):
                if p is not None and not p.is_alive() and self.respawn and not self._stop.value:
                    log.error("engine %d on %s exited (%s): respawning", i, self.devices[i], p.exitcode)
                    self.restarts += 1
                    self._spawn(i)
                    try:
                        self._wait_ready(1, 900.0)
                    except Exception:  # noqa: BLE001
                        log.exception("engine %d respawn failed", i)

    def frontend_specs(self) -> dict:
        """name -> [ChannelSpec per engine] for ONE front-end process (fresh fd handles)."""
        return {name: [c.spec() for c in chans] for name, chans in self.channels.items()}

    def close(self) -> None:
        self._stop.value = 1
        if getattr(self, "_mon_stop", None) is not None:
            self._mon_stop.set()
        for p in self.procs:
            if p is not None:
                p.join(timeout=15)
                if p.is_alive():
                    p.kill()
                    p.join(timeout=5)
        for chans in self.channels.values():
            for c in chans:
                c.close()


def attach_frontend(specs: dict, dead_after_s: float = 30.0) -> None:
    """In a front-end process: map every service's channels and install its RemotePool."""
    for name, sl in specs.items():
        chans = [ShmChannel.attach(s) for s in sl]
        install_remote(name, RemotePool(ChannelGroup(chans, dead_after_s)))


def engine_factory_of(service_cls, svc_cfg, cache_dir) -> Optional[tuple]:
    """(factory path, kwargs) when the service class can run on engines, else None."""
    f = getattr(service_cls, "engine_spec", None)
    return f(svc_cfg, cache_dir) if f is not None else None


# a ChannelSpec must be importable where pickled objects are rebuilt
__all__ = ["RemotePool", "PrefixedRemote", "EngineSet", "engine_main", "attach_frontend", "install_remote",
           "remote_scope", "current_remote", "engine_factory_of", "multi_worker", "is_remote", "ChannelSpec"]
