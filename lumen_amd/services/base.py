"""Service-layer plumbing shared by every gRPC service (L4).

* :class:`TaskRegistry` / :class:`TaskDefinition` — task name -> handler
  ``(payload, mime, meta) -> (bytes, mime, meta)`` plus the ``IOTask``/``Capability``
  builders (reference packages/lumen-clip/src/lumen_clip/registry.py:20-132, copied
  verbatim into face/ocr/vlm there; one implementation here).
* :class:`BaseInferenceService` — the bidirectional ``Infer`` loop with chunk
  reassembly by correlation id (``seq``/``total``), per-request latency meta,
  error mapping to ``InferResponse.error`` (unknown task ->
  ``ERROR_CODE_INVALID_ARGUMENT``, anything else -> ``ERROR_CODE_INTERNAL``), the
  capability RPCs and ``Health``.  Every service implements
  ``get_supported_tasks()`` and ``initialize()`` (the reference hub crashes on
  services lacking the former and never calls the latter — SURVEY §A.6 Q1/Q2).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, Optional

import grpc

from ..proto import ml_service as pb
from ..runtime.metrics import StageTimer, maybe_fault, observe_request, use_timer

log = logging.getLogger("lumen.service")

Handler = Callable[[bytes, str, dict], tuple]

MAX_PAYLOAD = 50 * 1024 * 1024
IMAGE_MIMES = ["image/jpeg", "image/png", "image/webp"]


def now_ms() -> int:
    return int(time.time() * 1000)


@dataclass
class TaskDefinition:
    name: str
    handler: Handler
    description: str
    input_mimes: list = field(default_factory=list)
    output_mime: str = "application/json"
    metadata: dict = field(default_factory=dict)

    def to_io_task(self) -> "pb.IOTask":
        limits = {"max_payload_size": str(MAX_PAYLOAD), "max_concurrency": "1"}
        limits.update({k: str(v) for k, v in self.metadata.items()})
        return pb.IOTask(name=self.name, input_mimes=list(self.input_mimes), output_mimes=[self.output_mime],
                         limits=limits)


class TaskRegistry:
    def __init__(self, service_name: str = "unknown"):
        self._tasks: dict[str, TaskDefinition] = {}
        self._service_name = service_name

    def register_task(self, name: str, handler: Handler, description: str = "", input_mimes=None,
                      output_mime: str = "application/json", metadata: Optional[dict] = None) -> None:
        if name in self._tasks:
            log.warning("task %s already registered, overwriting", name)
        self._tasks[name] = TaskDefinition(name, handler, description, list(input_mimes or []), output_mime,
                                           dict(metadata or {}))

    def set_service_name(self, name: str) -> None:
        self._service_name = name

    def get_handler(self, name: str) -> Handler:
        if name not in self._tasks:
            raise ValueError(f"Task '{name}' not found. Available tasks: {list(self._tasks)}")
        return self._tasks[name].handler

    def get_task_definition(self, name: str) -> TaskDefinition:
        if name not in self._tasks:
            raise ValueError(f"Task '{name}' not found. Available tasks: {list(self._tasks)}")
        return self._tasks[name]

    def list_task_names(self) -> list[str]:
        return list(self._tasks)

    def list_task_definitions(self) -> list[TaskDefinition]:
        return list(self._tasks.values())

    def get_all_tasks(self) -> list:
        return [t.to_io_task() for t in self._tasks.values()]

    def build_capability(self, service_name: str, model_id, runtime: str, precisions: list,
                         extra_metadata: Optional[dict] = None, max_concurrency: int = 1) -> "pb.Capability":
        extra = {k: ("" if v is None else str(v)) for k, v in (extra_metadata or {}).items()}
        model_ids = model_id if isinstance(model_id, list) else [model_id]
        return pb.Capability(service_name=service_name, model_ids=model_ids, runtime=runtime,
                             max_concurrency=max_concurrency, precisions=list(precisions), extra=extra,
                             tasks=self.get_all_tasks(), protocol_version="1.0")


@dataclass
class RuntimeModelInfo:
    """Runtime state of a loaded model (reference runtime_info.py:19-210)."""

    model_name: str
    model_id: str
    runtime: str = "mi355x"
    device: str = "cuda"
    precisions: list = field(default_factory=lambda: ["bf16"])
    embedding_dim: Optional[int] = None
    model_version: str = ""
    load_time: float = 0.0
    supports_classification: bool = False
    backend_info: str = ""
    extra: dict = field(default_factory=dict)

    def to_capability_metadata(self) -> dict[str, str]:
        d = {"device": self.device, "runtime": self.runtime, "model_version": self.model_version,
             "precisions": ",".join(self.precisions), "load_time_s": f"{self.load_time:.3f}"}
        if self.embedding_dim is not None:
            d["embedding_dim"] = str(self.embedding_dim)
        d.update({k: str(v) for k, v in self.extra.items()})
        return d


class BaseInferenceService(pb.InferenceServicer):
    """Shared Infer/GetCapabilities/StreamCapabilities/Health implementation."""

    SERVICE_NAME = "unknown"
    LATENCY_KEY = "lat_ms"            # CLIP: lat_ms; face/VLM: processing_time_ms; OCR: duration_ms
    UNKNOWN_TASK_CODE = pb.ERROR_CODE_INVALID_ARGUMENT
    DEFAULT_TASK: Optional[str] = None

    def __init__(self):
        self.registry = TaskRegistry(self.SERVICE_NAME)
        self.is_initialized = False
        self._init_lock = threading.Lock()

    # ---- lifecycle
    def initialize(self) -> None:
        with self._init_lock:
            if self.is_initialized:
                return
            self._initialize()
            self.is_initialized = True

    def _initialize(self) -> None:  # pragma: no cover - overridden
        pass

    def get_supported_tasks(self) -> list[str]:
        return self.registry.list_task_names()

    def close(self) -> None:
        pass

    def engine_spec(self):
        """(factory path, kwargs) of this service's GPU side for the engine / front-end serving
        topology (parallel/engine.py), or None when the service runs in-process only."""
        return None

    # ---- helpers
    @staticmethod
    def _assemble(cid: str, req, buffers: dict) -> tuple[bytes, bool]:
        if req.total <= 1:
            return bytes(req.payload), True
        buf = buffers.setdefault(cid, bytearray())
        buf.extend(req.payload)
        if req.seq + 1 == req.total:
            data = bytes(buf)
            del buffers[cid]
            return data, True
        return b"", False

    def _request_meta(self, req, context) -> dict[str, str]:
        return dict(req.meta)

    def _error(self, cid: str, code: int, msg: str, detail: str = "") -> "pb.InferResponse":
        return pb.InferResponse(correlation_id=cid, is_final=True, error=pb.Error(code=code, message=msg, detail=detail))

    def handle(self, task: str, payload: bytes, mime: str, meta: dict) -> tuple:
        """Dispatch one assembled request (used by the gRPC loop and in-process callers)."""
        handler = self.registry.get_handler(task)
        return handler(payload, mime, meta)

    # ---- gRPC methods
    # > 0: requests of ONE stream are handled concurrently, up to this many in flight (responses in
    # request order), so a client streaming many images feeds the dynamic batcher whole batches
    # instead of one request per round trip.  Services whose handlers stream (VLM) keep 0.
    PIPELINE = 0
    _pipe_pool = None
    _pipe_lock = threading.Lock()

    def Infer(self, request_iterator: Iterable, context):
        if not self.is_initialized:
            try:
                self.initialize()
            except Exception as e:  # surface as FAILED_PRECONDITION like the reference
                log.exception("initialize failed")
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"Model not initialized: {e}")
        if self.PIPELINE > 1:
            yield from self._infer_pipelined(request_iterator, context)
            return
        buffers: dict[str, bytearray] = {}
        try:
            for req in request_iterator:
                cid = req.correlation_id or f"cid-{now_ms()}"
                t0 = time.perf_counter()
                try:
                    payload, ready = self._assemble(cid, req, buffers)
                    if not ready:
                        continue
                    task = req.task or self.DEFAULT_TASK or ""
                    try:
                        handler = self.registry.get_handler(task)
                    except ValueError as e:
                        yield self._error(cid, self.UNKNOWN_TASK_CODE, str(e))
                        continue
                    meta = self._request_meta(req, context)
                    maybe_fault("infer")
                    timer = StageTimer(self.SERVICE_NAME)
                    with use_timer(timer):
                        out = handler(payload, req.payload_mime, meta)
                    if hasattr(out, "__next__"):  # streaming handler: yields (bytes, mime, meta, is_final)
                        while True:
                            with use_timer(timer):   # the generator body runs on each next()
                                chunk = next(out, None)
                            if chunk is None:
                                break
                            res, mime, extra, final = chunk
                            m = dict(extra or {})
                            if final:
                                m.update(timer.meta())
                            m[self.LATENCY_KEY] = str(int((time.perf_counter() - t0) * 1000))
                            schema = mime.split("schema=")[-1] if (final and "schema=" in mime) else ""
                            yield pb.InferResponse(correlation_id=cid, is_final=final, result=res, result_mime=mime,
                                                   meta=m, result_schema=schema)
                        observe_request(self.SERVICE_NAME, task, "ok", time.perf_counter() - t0)
                        continue
                    res, mime, extra = out
                    m = dict(extra or {})
                    m.update(timer.meta())   # per-stage times: t_<stage>_ms (decode, forward, queue, ...)
                    m[self.LATENCY_KEY] = str(int((time.perf_counter() - t0) * 1000))
                    schema = mime.split("schema=")[-1] if "schema=" in mime else ""
                    observe_request(self.SERVICE_NAME, task, "ok", time.perf_counter() - t0)
                    yield pb.InferResponse(correlation_id=cid, is_final=True, result=res, result_mime=mime, meta=m,
                                           result_schema=schema)
                except Exception as e:
                    log.exception("task %s failed", req.task)
                    code = pb.ERROR_CODE_UNAVAILABLE if _unavailable(e) else pb.ERROR_CODE_INTERNAL
                    observe_request(self.SERVICE_NAME, req.task, "error", time.perf_counter() - t0)
                    yield self._error(cid, code, str(e))
        finally:
            buffers.clear()

    def _one(self, req, cid: str, payload: bytes, context) -> list:
        """One assembled request -> its response messages (pipelined path; non-streaming handlers)."""
        t0 = time.perf_counter()
        try:
            task = req.task or self.DEFAULT_TASK or ""
            try:
                handler = self.registry.get_handler(task)
            except ValueError as e:
                return [self._error(cid, self.UNKNOWN_TASK_CODE, str(e))]
            meta = self._request_meta(req, context)
            maybe_fault("infer")
            timer = StageTimer(self.SERVICE_NAME)
            with use_timer(timer):
                out = handler(payload, req.payload_mime, meta)
                if hasattr(out, "__next__"):      # a streaming handler: run it out here, in order
                    chunks = list(out)
            msgs = []
            if hasattr(out, "__next__"):
                for res, mime, extra, final in chunks:
                    m = dict(extra or {})
                    if final:
                        m.update(timer.meta())
                    m[self.LATENCY_KEY] = str(int((time.perf_counter() - t0) * 1000))
                    schema = mime.split("schema=")[-1] if (final and "schema=" in mime) else ""
                    msgs.append(pb.InferResponse(correlation_id=cid, is_final=final, result=res, result_mime=mime,
                                                 meta=m, result_schema=schema))
            else:
                res, mime, extra = out
                m = dict(extra or {})
                m.update(timer.meta())
                m[self.LATENCY_KEY] = str(int((time.perf_counter() - t0) * 1000))
                schema = mime.split("schema=")[-1] if "schema=" in mime else ""
                msgs.append(pb.InferResponse(correlation_id=cid, is_final=True, result=res, result_mime=mime, meta=m,
                                             result_schema=schema))
            observe_request(self.SERVICE_NAME, task, "ok", time.perf_counter() - t0)
            return msgs
        except Exception as e:
            log.exception("task %s failed", req.task)
            code = pb.ERROR_CODE_UNAVAILABLE if _unavailable(e) else pb.ERROR_CODE_INTERNAL
            observe_request(self.SERVICE_NAME, req.task, "error", time.perf_counter() - t0)
            return [self._error(cid, code, str(e))]

    def _infer_pipelined(self, request_iterator: Iterable, context):
        import queue as _queue
        from concurrent.futures import ThreadPoolExecutor

        with BaseInferenceService._pipe_lock:
            if BaseInferenceService._pipe_pool is None:
                BaseInferenceService._pipe_pool = ThreadPoolExecutor(max_workers=int(
                    os.environ.get("LUMEN_PIPELINE_THREADS", "256")), thread_name_prefix="lumen-pipe")
        pool = BaseInferenceService._pipe_pool
        q: "_queue.Queue" = _queue.Queue()
        slots = threading.Semaphore(self.PIPELINE)
        stop = threading.Event()

        def reader():
            buffers: dict[str, bytearray] = {}
            try:
                for req in request_iterator:
                    cid = req.correlation_id or f"cid-{now_ms()}"
                    try:
                        payload, ready = self._assemble(cid, req, buffers)
                    except Exception as e:
                        q.put(("msg", [self._error(cid, pb.ERROR_CODE_INVALID_ARGUMENT, str(e))]))
                        continue
                    if not ready:
                        continue
                    while not slots.acquire(timeout=0.5):
                        if stop.is_set():
                            return
                    q.put(("fut", pool.submit(self._one, req, cid, payload, context)))
            except Exception as e:  # the stream itself failed (client cancelled, ...)
                q.put(("err", e))
            finally:
                buffers.clear()
                q.put(("end", None))

        threading.Thread(target=reader, name="lumen-pipe-reader", daemon=True).start()
        try:
            while True:
                kind, item = q.get()
                if kind == "end":
                    break
                if kind == "err":
                    raise item
                if kind == "fut":
                    msgs = item.result()
                    slots.release()
                else:
                    msgs = item
                for m in msgs:
                    yield m
        finally:
            stop.set()

    def GetCapabilities(self, request, context):
        return self.build_capability()

    def StreamCapabilities(self, request, context):
        yield self.build_capability()

    def Health(self, request, context):
        return pb.Empty()

    def build_capability(self) -> "pb.Capability":  # pragma: no cover - overridden
        return self.registry.build_capability(self.SERVICE_NAME, "unknown", "mi355x", ["bf16"])


def _unavailable(e: BaseException) -> bool:
    """Backend not ready / worker or engine gone -> UNAVAILABLE (client may retry elsewhere)."""
    name = type(e).__name__
    return ("NotInitialized" in name or "DeviceUnavailable" in name or "Unavailable" in name
            or (isinstance(e, RuntimeError) and "engine stopped" in str(e)))


def json_bytes(obj: Any) -> bytes:
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode("utf-8")


def meta_int(meta: dict, key: str, default: int) -> int:
    try:
        return int(meta.get(key, default))
    except (TypeError, ValueError):
        return default


def meta_float(meta: dict, key: str, default: float) -> float:
    try:
        return float(meta.get(key, default))
    except (TypeError, ValueError):
        return default


def meta_bool(meta: dict, key: str, default: bool) -> bool:
    v = meta.get(key)
    if v is None:
        return default
    return str(v).strip().lower() in ("1", "true", "yes", "on")
