"""FastVLMModelManager (L3) + GeneralFastVLMService (L4).

Reference: packages/lumen-vlm/src/lumen_vlm/fastvlm/fastvlm_model.py:51-403 (message
normalisation: ChatMessage or {role, content} mappings; roles user/assistant/system;
non-empty content; image <= 50 MB) and fastvlm_service.py:47-591: tasks
``vlm_generate`` / ``vlm_generate_stream`` (image MIME payload, limits
``max_image_size`` 5048x5048), meta ``messages`` (JSON list) or ``prompt``,
``max_new_tokens`` 512, ``temperature`` 0, ``top_p`` 1, ``repetition_penalty`` 1,
``do_sample``, ``add_generation_prompt`` true, ``stop_sequences`` (JSON list); response
meta ``generated_tokens``, ``finish_reason`` (+ ``streaming_chunks``) and
``processing_time_ms``; ``SERVICE_NAME`` "vlm-fast".

``vlm_generate_stream`` really streams: one InferResponse per decoded chunk
(``is_final`` false, text delta, meta ``step``) and a final TextGenerationV1 response
(the reference buffers everything into one response).
"""
from __future__ import annotations

import json
import logging
import time
from typing import Any, Iterable, Mapping, Optional, Sequence

from ...resources import schemas as rs
from ..base import IMAGE_MIMES, BaseInferenceService, RuntimeModelInfo
from ..common import backend_settings, load_model_resources, pick_model
from .backend import (ChatMessage, GenerationChunk, GenerationResult, InvalidInputError, MI355XVLMBackend,
                      create_backend)

log = logging.getLogger("lumen.vlm")

VLM_KEYS = ("general", "vlm", "fastvlm", "default")
MAX_IMAGE_BYTES = 50 * 1024 * 1024


class FastVLMModelManager:
    def __init__(self, backend: MI355XVLMBackend, resources):
        if backend is None or resources is None:
            raise ValueError("backend / resources cannot be None")
        self._backend = backend
        self._resources = resources
        self._initialized = False
        self._load_time: Optional[float] = None

    @property
    def model_name(self) -> str:
        return self._resources.model_name

    @property
    def model_id(self) -> str:
        return self._resources.model_id

    @property
    def is_initialized(self) -> bool:
        return self._initialized

    def initialize(self) -> None:
        if self._initialized:
            return
        t0 = time.time()
        self._backend.initialize()
        self._load_time = time.time() - t0
        self._initialized = True

    def _ensure(self):
        if not self._initialized:
            from .backend import BackendNotInitializedError

            raise BackendNotInitializedError("Model manager must be initialized before inference. Call initialize() first.")

    @staticmethod
    def _normalize(messages) -> list[ChatMessage]:
        if not messages:
            raise InvalidInputError("Messages cannot be empty")
        out = []
        for m in messages:
            if isinstance(m, ChatMessage):
                out.append(m)
            elif isinstance(m, Mapping):
                role, content = m.get("role"), m.get("content")
                if not isinstance(role, str) or not isinstance(content, str):
                    raise InvalidInputError("Dictionary messages must include string 'role' and 'content' keys")
                out.append(ChatMessage(role, content))
            else:
                raise InvalidInputError(f"Unsupported message type: {type(m).__name__}")
        for m in out:
            if m.role not in ("user", "assistant", "system"):
                raise InvalidInputError(f"Invalid role: {m.role}")
            if not m.content or not m.content.strip():
                raise InvalidInputError("Message content cannot be empty")
        return out

    @staticmethod
    def _validate_image(image_bytes: bytes) -> None:
        if not image_bytes:
            raise InvalidInputError("Image bytes cannot be empty")
        if len(image_bytes) > MAX_IMAGE_BYTES:
            raise InvalidInputError("Image too large (max 50MB)")

    def generate(self, messages, image_bytes: bytes, *, stream: bool = False, **kw):
        self._ensure()
        msgs = self._normalize(messages)
        self._validate_image(image_bytes)
        req = self._backend.build_generation_request(messages=msgs, image_bytes=image_bytes, stream=stream, **kw)
        return self._backend.generate(req)

    def generate_stream(self, messages, image_bytes: bytes, **kw) -> Iterable[GenerationChunk]:
        return self.generate(messages, image_bytes, stream=True, **kw)

    def info(self) -> RuntimeModelInfo:
        bi = self._backend.get_info()
        return RuntimeModelInfo(model_name=self.model_name, model_id=self.model_id, runtime=bi.runtime,
                                device=str(bi.device), precisions=list(bi.precisions),
                                model_version=bi.version or "", load_time=self._load_time or 0.0,
                                extra={k: v for k, v in bi.as_dict().items() if v is not None and k not in
                                       ("runtime", "device", "precisions", "model_id", "model_name", "version")})

    get_info = info

    def get_backend_info(self):
        self._ensure()
        return self._backend.get_info()

    def close(self) -> None:
        if self._initialized:
            self._backend.close()
            self._initialized = False


def _f(meta, k, d):
    try:
        return float(meta.get(k, d))
    except (TypeError, ValueError):
        return d


def _i(meta, k, d):
    try:
        return int(float(meta.get(k, d)))
    except (TypeError, ValueError):
        return d


def _b(meta, k, d: str):
    return str(meta.get(k, d)).lower() == "true"


class GeneralFastVLMService(BaseInferenceService):
    SERVICE_NAME = "vlm-fast"
    LATENCY_KEY = "processing_time_ms"

    def __init__(self, backend: MI355XVLMBackend, resources):
        super().__init__()
        self.backend = backend
        self.resources = resources
        self.model = FastVLMModelManager(backend, resources)
        lim = {"max_image_size": "5048x5048"}
        self.registry.register_task("vlm_generate", self._handle_generate, "Generate text from image and text input",
                                    IMAGE_MIMES, rs.MIME_TEXT_GEN, lim)
        self.registry.register_task("vlm_generate_stream", self._handle_generate_stream,
                                    "Generate text from image and text input with streaming", IMAGE_MIMES,
                                    rs.MIME_TEXT_GEN, lim)

    @classmethod
    def from_config(cls, service_config, cache_dir) -> "GeneralFastVLMService":
        mc = pick_model(service_config, VLM_KEYS)
        if mc is None:
            raise ValueError("No VLM model configured")
        resources = load_model_resources(cache_dir, mc, ("tokenizer_config.json", "lumen_vlm_config.json"))
        return cls(create_backend(backend_settings(service_config), resources, mc.runtime.value), resources)

    def _initialize(self):
        self.model.initialize()

    def engine_spec(self):
        from .backend import engine_spec

        return engine_spec(self.backend)

    def close(self):
        self.model.close()

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _messages(meta: dict) -> list[ChatMessage]:
        msgs = []
        if "messages" in meta:
            try:
                data = json.loads(meta["messages"])
                if isinstance(data, list):
                    for m in data:
                        if isinstance(m, dict) and "role" in m and "content" in m:
                            msgs.append(ChatMessage(role=m["role"], content=m["content"]))
            except (json.JSONDecodeError, KeyError, TypeError):
                log.warning("Invalid messages format in meta")
        if not msgs and "prompt" in meta:
            msgs.append(ChatMessage(role="user", content=meta["prompt"]))
        return msgs

    def _params(self, meta: dict) -> dict:
        stops = None
        if "stop_sequences" in meta:
            try:
                stops = json.loads(meta["stop_sequences"])
                if not isinstance(stops, list):
                    stops = None
            except json.JSONDecodeError:
                log.warning("Invalid stop_sequences format, ignoring")
        p = dict(max_new_tokens=_i(meta, "max_new_tokens", 512), temperature=_f(meta, "temperature", 0.0),
                 top_p=_f(meta, "top_p", 1.0), repetition_penalty=_f(meta, "repetition_penalty", 1.0),
                 do_sample=_b(meta, "do_sample", "false"), add_generation_prompt=_b(meta, "add_generation_prompt", "true"),
                 stop_sequences=stops)
        if "seed" in meta:
            p["extra"] = {"seed": _i(meta, "seed", 0)}
        return p

    def _prep(self, payload: bytes, meta: dict):
        msgs = self._messages(meta)
        if not msgs:
            raise ValueError("No messages provided in metadata")
        if not payload:
            raise ValueError("No image data provided")
        return msgs, self._params(meta)

    def _result_bytes(self, text, finish_reason, generated, input_tokens, meta_extra=None) -> bytes:
        md = rs.GenMetadata(**meta_extra) if meta_extra else None
        out = rs.TextGenerationV1(text=text, finish_reason=finish_reason, generated_tokens=generated,
                                  input_tokens=input_tokens, model_id=self.model.model_id, metadata=md)
        return rs.dumps(out)

    # ---------------------------------------------------------------- handlers
    def _handle_generate(self, payload: bytes, mime: str, meta: dict):
        msgs, p = self._prep(payload, meta)
        res: GenerationResult = self.model.generate(msgs, payload, stream=False, **p)
        n_in = res.metadata.get("input_tokens")
        body = self._result_bytes(res.text, res.finish_reason, len(res.tokens), n_in,
                                  {"temperature": p["temperature"], "top_p": p["top_p"],
                                   "max_tokens": p["max_new_tokens"]})
        m = {"generated_tokens": str(len(res.tokens)), "finish_reason": res.finish_reason}
        if res.metadata.get("ttft_ms") is not None:
            m["ttft_ms"] = f"{res.metadata['ttft_ms']:.2f}"
        return body, rs.MIME_TEXT_GEN, m

    def _handle_generate_stream(self, payload: bytes, mime: str, meta: dict):
        msgs, p = self._prep(payload, meta)
        chunks = self.model.generate_stream(msgs, payload, **p)

        def gen():
            text, n_tok, n_chunks = [], 0, 0
            t0 = time.perf_counter()
            for ch in chunks:
                if ch.is_final:
                    reason = ch.metadata.get("reason", "stop")
                    full = "".join(text)
                    body = self._result_bytes(full, reason, n_tok, ch.metadata.get("input_tokens"),
                                              {"temperature": p["temperature"], "top_p": p["top_p"],
                                               "max_tokens": p["max_new_tokens"], "streaming_chunks": n_chunks,
                                               "generation_time_ms": (time.perf_counter() - t0) * 1000})
                    yield body, rs.MIME_TEXT_GEN, {"generated_tokens": str(n_tok), "finish_reason": reason,
                                                   "streaming_chunks": str(n_chunks)}, True
                    return
                n_tok += len(ch.tokens)
                if ch.text:
                    text.append(ch.text)
                    n_chunks += 1
                    m = {"step": str(ch.metadata.get("step", n_chunks)), "tokens": str(n_tok)}
                    if "t_wall" in ch.metadata:     # when the generating process produced the chunk
                        m["t_emit"] = f"{ch.metadata['t_wall']:.6f}"
                    yield ch.text.encode("utf-8"), "text/plain;charset=utf-8", m, False

        return gen()

    def build_capability(self):
        bi = self.backend.get_info()
        extra = {k: str(v) for k, v in bi.as_dict().items() if v is not None and not isinstance(v, list)}
        return self.registry.build_capability(self.SERVICE_NAME, self.resources.model_id, bi.runtime,
                                              list(bi.precisions), extra)
