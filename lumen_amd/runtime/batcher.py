"""Dynamic request batcher (one GPU-owning worker thread per batcher).

The reference serves every request as a batch-1 ONNX run on whichever gRPC
thread received it (SURVEY §3.2 "no cross-stream batching").  Here concurrent
requests from all gRPC streams are queued and a single worker thread — the
only thread that launches work on that model's HIP stream — drains up to
``max_batch`` items or waits at most ``max_wait_ms`` after the first item, then
runs one batched call.  Results are delivered through futures, so callers stay
synchronous.  ``concurrency`` > 1 runs that many dispatcher threads on the same
queue, for batch functions that hand work to a multi-GPU worker pool (several
batches in flight, one per dispatcher).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from concurrent.futures import Future
from typing import Any, Callable, Optional, Sequence

from .metrics import StageTimer, batch_size, current_timer, use_timer

log = logging.getLogger("lumen.batcher")


class DynamicBatcher:
    def __init__(self, fn: Callable[[Sequence[Any]], Sequence[Any]], max_batch: int = 64, max_wait_ms: float = 2.0,
                 name: str = "batcher", concurrency: int = 1):
        self.fn = fn
        self.max_batch = max(1, int(max_batch))
        self.max_wait = max_wait_ms / 1000.0
        self.name = name
        self._q: "queue.Queue[tuple[Any, Future]]" = queue.Queue()
        self._stop = threading.Event()
        self.batches = 0
        self.items = 0
        self._count_lock = threading.Lock()
        self._threads = [threading.Thread(target=self._loop, name=f"lumen-{name}-{i}", daemon=True)
                         for i in range(max(1, int(concurrency)))]
        for t in self._threads:
            t.start()

    def submit(self, item: Any) -> Future:
        if self._stop.is_set():
            raise RuntimeError(f"{self.name} is closed")
        fut: Future = Future()
        fut.lumen_t_submit = time.perf_counter()
        self._q.put((item, fut))
        return fut

    @staticmethod
    def _collect(fut: Future, timeout: Optional[float]) -> Any:
        out = fut.result(timeout)
        t = current_timer()
        stats = getattr(fut, "lumen_stats", None)
        if t is not None and stats:
            t.merge(stats)
        return out

    def __call__(self, item: Any, timeout: Optional[float] = None) -> Any:
        return self._collect(self.submit(item), timeout)

    def map(self, items: Sequence[Any], timeout: Optional[float] = None) -> list:
        futs = [self.submit(x) for x in items]
        return [self._collect(f, timeout) for f in futs]

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                first = self._q.get(timeout=0.1)
            except queue.Empty:
                continue
            batch = [first]
            deadline = time.perf_counter() + self.max_wait
            while len(batch) < self.max_batch:
                rem = deadline - time.perf_counter()
                try:
                    batch.append(self._q.get(timeout=max(rem, 0.0)) if rem > 0 else self._q.get_nowait())
                except queue.Empty:
                    break
            items = [b[0] for b in batch]
            t_start = time.perf_counter()
            timer = StageTimer(self.name)
            try:
                with use_timer(timer):
                    outs = self.fn(items)
                stats = dict(timer.finish())
                h = batch_size()
                if h is not None:
                    h.labels(self.name).observe(len(items))
                if len(outs) != len(items):
                    raise RuntimeError(f"{self.name}: batch fn returned {len(outs)} results for {len(items)} items")
                for (_, fut), out in zip(batch, outs):
                    # per request: the batch's stage times, its queue wait and the batch size
                    fut.lumen_stats = dict(stats, queue=(t_start - getattr(fut, "lumen_t_submit", t_start)) * 1000)
                    fut.lumen_batch = len(items)
                    if isinstance(out, BaseException):
                        fut.set_exception(out)
                    else:
                        fut.set_result(out)
            except BaseException as e:  # deliver the failure to every waiter
                log.exception("%s batch failed", self.name)
                for _, fut in batch:
                    if not fut.done():
                        fut.set_exception(e)
            with self._count_lock:
                self.batches += 1
                self.items += len(items)

    def close(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2.0)
        while True:
            try:
                _, fut = self._q.get_nowait()
            except queue.Empty:
                break
            fut.set_exception(RuntimeError(f"{self.name} closed"))
