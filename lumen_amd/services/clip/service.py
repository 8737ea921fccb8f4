"""CLIP gRPC services (L4): GeneralCLIPService, BioCLIPService, SmartCLIPService.

Task names, MIME rules, request/response meta and JSON result shapes follow
SURVEY §A.2 (reference: general_clip/clip_service.py:44-414,
expert_bioclip/bioclip_service.py:46-425, unified_smartclip/smartclip_service.py:43-520).
Model-id conventions (§A.5): CLIP text embed ``"<model_name>:<model>_<runtime>"``,
other CLIP tasks ``"<model>_<runtime>"``, SmartCLIP ``"smartclip:<model>"``.
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Optional

from ...resources import schemas as rs
from ...resources.config import BackendSettings, Services
from ...resources.exceptions import ResourceNotFoundError
from ..base import IMAGE_MIMES, BaseInferenceService, meta_int
from .backend import create_backend
from .model import BioCLIPModelManager, CLIPModelManager
from .resources import ResourceLoader

log = logging.getLogger("lumen.clip.service")

GENERAL_KEYS = ("general", "clip", "general_clip")
BIO_KEYS = ("bioclip", "bio", "bioclip2")


def _pick_model(service_config: Services, keys, fallback_first: bool = False):
    for k in keys:
        if k in service_config.models:
            return service_config.models[k]
    if fallback_first and service_config.models:
        return next(iter(service_config.models.values()))
    return None


def _make_backend(service_config: Services, model_config, cache_dir):
    try:
        resources = ResourceLoader.load_model_resources(cache_dir, model_config)
    except Exception as e:
        raise ResourceNotFoundError(f"Failed to load resources for {model_config.model}: {e}") from e
    settings = service_config.backend_settings or BackendSettings(device=None, batch_size=1, onnx_providers=None)
    precision = model_config.precision if model_config.runtime.value in ("onnx", "rknn") else None
    return create_backend(settings, resources, model_config.runtime.value, precision=precision), resources


def _embedding(vec, model_id: str) -> bytes:
    v = [float(x) for x in vec]
    return rs.dumps(rs.EmbeddingV1(vector=v, dim=len(v), model_id=model_id))


def _labels(pairs, model_id: str) -> bytes:
    return rs.dumps(rs.LabelsV1(labels=[rs.Label(label=l, score=float(s)) for l, s in pairs], model_id=model_id))


class GeneralCLIPService(BaseInferenceService):
    SERVICE_NAME = "lumen_clip"
    PIPELINE = 64   # one stream's requests batch together (services/base.py Infer)
    LATENCY_KEY = "lat_ms"

    def __init__(self, backend, resources):
        super().__init__()
        self.backend = backend
        self.resources = resources
        self.model = CLIPModelManager(backend, resources)
        self._setup_registry()

    @classmethod
    def from_config(cls, service_config: Services, cache_dir) -> "GeneralCLIPService":
        mc = _pick_model(service_config, GENERAL_KEYS)
        if mc is None:
            raise ValueError("No suitable model config found; expected one of 'general', 'clip', 'general_clip'")
        backend, resources = _make_backend(service_config, mc, cache_dir)
        return cls(backend, resources)

    def _setup_registry(self):
        r = self.registry
        r.register_task("clip_text_embed", self._handle_embed, "Embed text into the CLIP space",
                        ["application/json", "text/plain"], rs.MIME_EMBEDDING)
        r.register_task("clip_image_embed", self._handle_image_embed, "Embed an image into the CLIP space",
                        IMAGE_MIMES, rs.MIME_EMBEDDING)
        if self.resources.has_classification_support():
            r.register_task("clip_classify", self._handle_classify, "Zero-shot classify against the label bank",
                            IMAGE_MIMES, rs.MIME_LABELS, {"dataset": self.resources.dataset or ""})
            r.register_task("clip_scene_classify", self._handle_scene, "High-level scene classification",
                            IMAGE_MIMES, rs.MIME_LABELS)

    def _initialize(self):
        self.model.initialize()

    def engine_spec(self):
        from .backend import engine_spec

        return engine_spec(self.resources)

    # ---- handlers
    def _handle_embed(self, payload: bytes, mime: str, meta: dict):
        text = payload.decode("utf-8")
        vec = self.model.encode_text(text)
        info = self.model.info()
        return _embedding(vec, f"{info.model_name}:{info.model_id}"), rs.MIME_EMBEDDING, {"dim": str(len(vec))}

    def _handle_image_embed(self, payload: bytes, mime: str, meta: dict):
        vec = self.model.encode_image(payload)
        return _embedding(vec, self.model.info().model_id), rs.MIME_EMBEDDING, {"dim": str(len(vec))}

    def _handle_classify(self, payload: bytes, mime: str, meta: dict):
        pairs = self.model.classify_image(payload, top_k=meta_int(meta, "topk", 5))
        return _labels(pairs, self.model.info().model_id), rs.MIME_LABELS, {"labels_count": str(len(pairs))}

    def _handle_scene(self, payload: bytes, mime: str, meta: dict):
        label, score = self.model.classify_scene(payload)
        return _labels([(label, score)], self.model.info().model_id), rs.MIME_LABELS, {"labels_count": "1"}

    def build_capability(self):
        info = self.model.info() if self.is_initialized else None
        bi = self.backend.get_info()
        extra = {"device": str(bi.device), "embedding_dim": str(bi.image_embedding_dim),
                 "model_version": self.resources.model_info.version,
                 "supports_classification": str(self.resources.has_classification_support())}
        return self.registry.build_capability(self.SERVICE_NAME, self.resources.model_name, bi.runtime,
                                              list(bi.precisions), extra)

    def close(self):
        self.backend.close()


class BioCLIPService(BaseInferenceService):
    SERVICE_NAME = "lumen_bioclip"
    PIPELINE = 64   # one stream's requests batch together (services/base.py Infer)
    LATENCY_KEY = "lat_ms"

    def __init__(self, backend, resources):
        super().__init__()
        self.backend = backend
        self.resources = resources
        self.model = BioCLIPModelManager(backend, resources)
        self._setup_registry()

    @classmethod
    def from_config(cls, service_config: Services, cache_dir) -> "BioCLIPService":
        mc = _pick_model(service_config, BIO_KEYS, fallback_first=True)
        if mc is None:
            raise ValueError("No BioCLIP model configured")
        backend, resources = _make_backend(service_config, mc, cache_dir)
        return cls(backend, resources)

    def _setup_registry(self):
        r = self.registry
        r.register_task("bioclip_text_embed", self._handle_text, "Embed text (BioCLIP)",
                        ["application/json", "text/plain"], rs.MIME_EMBEDDING)
        r.register_task("bioclip_image_embed", self._handle_image, "Embed an image (BioCLIP)", IMAGE_MIMES,
                        rs.MIME_EMBEDDING)
        if self.resources.has_classification_support():
            r.register_task("bioclip_classify", self._handle_classify, "TreeOfLife species classification",
                            IMAGE_MIMES, rs.MIME_LABELS, {"namespace": "bioatlas"})

    def _initialize(self):
        self.model.initialize()

    def engine_spec(self):
        from .backend import bio_shards_bank, engine_spec

        return engine_spec(self.resources, shard_bank=bio_shards_bank(self.resources))

    def _handle_text(self, payload: bytes, mime: str, meta: dict):
        if not (mime or "").startswith("text/"):
            raise ValueError(f"embed expects text/* payload, got {mime!r}")
        vec = self.model.encode_text(payload.decode("utf-8"))
        return _embedding(vec, self.model.info().model_id), rs.MIME_EMBEDDING, {"dim": str(len(vec))}

    def _handle_image(self, payload: bytes, mime: str, meta: dict):
        if not (mime or "").startswith("image/"):
            raise ValueError(f"image_embed expects image/* payload, got {mime!r}")
        vec = self.model.encode_image(payload)
        return _embedding(vec, self.model.info().model_id), rs.MIME_EMBEDDING, {"dim": str(len(vec))}

    def _handle_classify(self, payload: bytes, mime: str, meta: dict):
        if not (mime or "").startswith("image/"):
            raise ValueError(f"classify expects image/* payload, got {mime!r}")
        ns = meta.get("namespace", "bioatlas")
        if ns != "bioatlas":
            raise ValueError(f"unsupported namespace {ns!r}, expected 'bioatlas'")
        pairs = self.model.classify_image(payload, top_k=meta_int(meta, "topk", 5))
        return _labels(pairs, self.model.info().model_id), rs.MIME_LABELS, {"labels_count": str(len(pairs))}

    def build_capability(self):
        bi = self.backend.get_info()
        extra = {"device": str(bi.device), "embedding_dim": str(bi.image_embedding_dim),
                 "supports_classification": str(self.resources.has_classification_support())}
        return self.registry.build_capability(self.SERVICE_NAME, self.resources.model_name, bi.runtime,
                                              list(bi.precisions), extra)

    def close(self):
        self.backend.close()


class SmartCLIPService(BaseInferenceService):
    """General CLIP + BioCLIP behind one service (both use the CLIP model's runtime)."""

    SERVICE_NAME = "lumen_smartclip"
    PIPELINE = 64   # one stream's requests batch together (services/base.py Infer)
    LATENCY_KEY = "lat_ms"

    def __init__(self, clip_backend, clip_resources, bio_backend, bio_resources):
        super().__init__()
        self.clip_backend, self.bio_backend = clip_backend, bio_backend
        self.clip_resources, self.bio_resources = clip_resources, bio_resources
        self.clip_model = CLIPModelManager(clip_backend, clip_resources)
        self.bioclip_model = BioCLIPModelManager(bio_backend, bio_resources)
        self._setup_registry()

    @classmethod
    def from_config(cls, service_config: Services, cache_dir) -> "SmartCLIPService":
        mc = _pick_model(service_config, GENERAL_KEYS)
        mb = _pick_model(service_config, BIO_KEYS)
        if mc is None or mb is None:
            raise ValueError("SmartCLIP needs both a general CLIP model and a BioCLIP model")
        mb = mb.model_copy(update={"runtime": mc.runtime})
        cb, cr = _make_backend(service_config, mc, cache_dir)
        bb, br = _make_backend(service_config, mb, cache_dir)
        cb.remote_key, bb.remote_key = "general", "bio"     # their parts of the shared engine
        return cls(cb, cr, bb, br)

    def engine_spec(self):
        """Both towers on one engine (parallel.engine.multi_worker): kinds "general:*" / "bio:*"."""
        from .backend import bio_shards_bank, engine_spec

        return ("lumen_amd.parallel.engine:multi_worker",
                {"parts": {"general": engine_spec(self.clip_resources),
                           "bio": engine_spec(self.bio_resources, shard_bank=bio_shards_bank(self.bio_resources))}})

    def _setup_registry(self):
        r = self.registry
        r.register_task("smartclip_text_embed", self._handle_text, "Embed text (general CLIP)",
                        ["application/json", "text/plain"], rs.MIME_EMBEDDING)
        r.register_task("smartclip_image_embed", self._handle_image, "Embed an image (general CLIP)", IMAGE_MIMES,
                        rs.MIME_EMBEDDING)
        if self.clip_resources.has_classification_support():
            r.register_task("smartclip_classify", self._handle_classify, "Zero-shot classification", IMAGE_MIMES,
                            rs.MIME_LABELS)
        r.register_task("smartclip_scene_classify", self._handle_scene, "Scene classification", IMAGE_MIMES,
                        rs.MIME_LABELS)
        if self.bio_resources.has_classification_support():
            r.register_task("smartclip_bioclassify", self._handle_bio, "TreeOfLife species classification",
                            IMAGE_MIMES, rs.MIME_LABELS, {"namespace": "bioatlas"})

    def _initialize(self):
        self.clip_model.initialize()
        self.bioclip_model.initialize()

    def _mid(self) -> str:
        return f"smartclip:{self.clip_resources.model_name}"

    def _handle_text(self, payload, mime, meta):
        if not (mime or "").startswith("text/"):
            raise ValueError(f"text_embed expects text/* payload, got {mime!r}")
        vec = self.clip_model.encode_text(payload.decode("utf-8"))
        return _embedding(vec, self._mid()), rs.MIME_EMBEDDING, {}

    def _handle_image(self, payload, mime, meta):
        if not (mime or "").startswith("image/"):
            raise ValueError(f"image_embed expects image/* payload, got {mime!r}")
        vec = self.clip_model.encode_image(payload)
        return _embedding(vec, self._mid()), rs.MIME_EMBEDDING, {}

    def _handle_classify(self, payload, mime, meta):
        pairs = self.clip_model.classify_image(payload, top_k=meta_int(meta, "topk", 5))
        return _labels(pairs, self._mid()), rs.MIME_LABELS, {"labels_count": str(len(pairs))}

    def _handle_scene(self, payload, mime, meta):
        label, score = self.clip_model.classify_scene(payload)
        return _labels([(label, score)], self._mid()), rs.MIME_LABELS, {"labels_count": "1"}

    def _handle_bio(self, payload, mime, meta):
        ns = meta.get("namespace", "bioatlas")
        if ns != "bioatlas":
            raise ValueError(f"unsupported namespace {ns!r}, expected 'bioatlas'")
        pairs = self.bioclip_model.classify_image(payload, top_k=meta_int(meta, "topk", 5))
        return _labels(pairs, self._mid()), rs.MIME_LABELS, {"labels_count": str(len(pairs))}

    def build_capability(self):
        bi = self.clip_backend.get_info()
        return self.registry.build_capability(
            self.SERVICE_NAME, f"{self.clip_resources.model_name}+{self.bio_resources.model_name}", bi.runtime,
            list(bi.precisions), {"device": str(bi.device), "embedding_dim": str(bi.image_embedding_dim)})

    def close(self):
        self.clip_backend.close()
        self.bio_backend.close()
