"""Observability: Prometheus metrics, per-stage timers, ROCTX ranges, fault injection.

SURVEY §5.1/§5.5: the reference only stamps wall-clock latencies into response meta.
Here every service request is counted and timed (``lumen_requests_total``,
``lumen_request_seconds``), the device pipelines time their stages (decode,
preprocess, forward, post-process, serialise) with :class:`StageTimer` — host clocks,
or HIP events when ``LUMEN_GPU_TIMERS=1`` so device time is measured without extra
synchronisation on the hot path — and wrap them in ROCTX ranges (visible in
``rocprofv3 --marker-trace``).  The hub exports the registry on
``LUMEN_METRICS_PORT`` (Prometheus text format); the control plane serves
``/metrics`` for its own process.

Fault injection (for tests): ``LUMEN_FAULT=<site>:<prob>`` makes
:func:`maybe_fault` raise :class:`InjectedFault` at that site with the given
probability (sites: ``infer``, ``batch``, ``engine``).
"""
from __future__ import annotations

import contextlib
import contextvars
import os
import random
import threading
import time
from typing import Optional

try:
    import prometheus_client as prom
except Exception:  # pragma: no cover
    prom = None

_lock = threading.Lock()
_metrics: dict = {}


def _get(kind: str, name: str, doc: str, labels: tuple = (), **kw):
    with _lock:
        m = _metrics.get(name)
        if m is None and prom is not None:
            m = getattr(prom, kind)(name, doc, labels, **kw)
            _metrics[name] = m
        return m


LAT_BUCKETS = (0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1, 2, 5, 10, 30)


def requests_total():
    return _get("Counter", "lumen_requests_total", "gRPC Infer requests", ("service", "task", "status"))


def request_seconds():
    return _get("Histogram", "lumen_request_seconds", "end-to-end request latency", ("service", "task"),
                buckets=LAT_BUCKETS)


def stage_seconds():
    return _get("Histogram", "lumen_stage_seconds", "pipeline stage latency", ("pipeline", "stage"),
                buckets=LAT_BUCKETS)


def batch_size():
    return _get("Histogram", "lumen_batch_size", "dynamic batch sizes", ("batcher",),
                buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512))


def ttft_seconds():
    return _get("Histogram", "lumen_vlm_ttft_seconds", "VLM time to first token", (), buckets=LAT_BUCKETS)


def tokens_total():
    return _get("Counter", "lumen_vlm_tokens_total", "generated tokens", ())


def kv_blocks_used():
    return _get("Gauge", "lumen_kv_blocks_used", "paged KV blocks in use", ())


def observe_request(service: str, task: str, status: str, seconds: float) -> None:
    c, h = requests_total(), request_seconds()
    if c is not None:
        c.labels(service, task or "-", status).inc()
        h.labels(service, task or "-").observe(seconds)


class StageTimer:
    """``with timer.stage("forward"): ...`` -> per-stage milliseconds in ``timer.ms`` and
    the ``lumen_stage_seconds`` histogram; ROCTX range per stage."""

    def __init__(self, pipeline: str, gpu: Optional[bool] = None):
        self.pipeline = pipeline
        self.ms: dict[str, float] = {}
        self.gpu = (os.environ.get("LUMEN_GPU_TIMERS") == "1") if gpu is None else gpu
        self._events: list = []

    @contextlib.contextmanager
    def stage(self, name: str):
        nvtx = _nvtx()
        if nvtx is not None:
            nvtx.range_push(f"{self.pipeline}:{name}")
        if self.gpu:
            import torch

            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._events.append((name, s, e))
                if nvtx is not None:
                    nvtx.range_pop()
            return
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t0
            self.ms[name] = self.ms.get(name, 0.0) + dt * 1000
            h = stage_seconds()
            if h is not None:
                h.labels(self.pipeline, name).observe(dt)
            if nvtx is not None:
                nvtx.range_pop()

    def finish(self) -> dict[str, float]:
        """resolve HIP-event timings (synchronises on the last event only)."""
        if self._events:
            self._events[-1][2].synchronize()
            h = stage_seconds()
            for name, s, e in self._events:
                ms = s.elapsed_time(e)
                self.ms[name] = self.ms.get(name, 0.0) + ms
                if h is not None:
                    h.labels(self.pipeline, name).observe(ms / 1000)
            self._events.clear()
        return self.ms

    def merge(self, ms: dict, prefix: str = "") -> None:
        """Add stage times measured elsewhere (a dynamic batcher's batch) to this timer."""
        for k, v in (ms or {}).items():
            key = prefix + k
            self.ms[key] = self.ms.get(key, 0.0) + float(v)

    def meta(self, prefix: str = "t_") -> dict[str, str]:
        return {f"{prefix}{k}_ms": f"{v:.3f}" for k, v in self.finish().items()}


# The request's timer travels in a context variable: the service installs one per request
# (:func:`use_timer`), the pipelines mark stages with :func:`stage` without plumbing a timer
# argument through every layer, and a dynamic batcher's worker thread runs each batch under
# its own timer whose stage times are merged back into every request of the batch.
_CURRENT: "contextvars.ContextVar[Optional[StageTimer]]" = contextvars.ContextVar("lumen_stage_timer", default=None)


def current_timer() -> Optional[StageTimer]:
    return _CURRENT.get()


@contextlib.contextmanager
def use_timer(t: Optional[StageTimer]):
    tok = _CURRENT.set(t)
    try:
        yield t
    finally:
        _CURRENT.reset(tok)


@contextlib.contextmanager
def stage(name: str):
    """Time a pipeline stage on the current request/batch timer (no-op without one)."""
    t = _CURRENT.get()
    if t is None:
        yield
        return
    with t.stage(name):
        yield


_nvtx_mod = None


def _nvtx():
    global _nvtx_mod
    if os.environ.get("LUMEN_ROCTX", "0") != "1":
        return None
    if _nvtx_mod is None:
        try:
            import torch

            _nvtx_mod = torch.cuda.nvtx
        except Exception:  # pragma: no cover
            _nvtx_mod = False
    return _nvtx_mod or None


def exposition() -> bytes:
    if prom is None:
        return b""
    return prom.generate_latest()


def start_metrics_server(port: Optional[int] = None) -> Optional[int]:
    port = int(port or os.environ.get("LUMEN_METRICS_PORT", "0") or 0)
    if not port or prom is None:
        return None
    prom.start_http_server(port)
    return port


# ----------------------------------------------------------------------------- fault injection
class InjectedFault(RuntimeError):
    pass


def _fault_spec() -> dict[str, float]:
    spec = os.environ.get("LUMEN_FAULT", "")
    out = {}
    for part in spec.split(","):
        if ":" in part:
            k, v = part.split(":", 1)
            try:
                out[k.strip()] = float(v)
            except ValueError:
                pass
    return out


def maybe_fault(site: str) -> None:
    p = _fault_spec().get(site)
    if p and random.random() < p:
        raise InjectedFault(f"injected fault at {site}")
