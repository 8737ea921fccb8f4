"""OcrModelManager (L3) + GeneralOcrService (L4).

Reference: packages/lumen-ocr/src/lumen_ocr/general_ocr/ocr_model.py:27-214 (the manager
owns resource loading + backend creation inside ``initialize()``) and
general_ocr/ocr_service.py:32-293: task ``ocr`` (also the default for an empty task),
lazy initialisation on the first ``Infer`` / ``GetCapabilities``, meta = gRPC invocation
metadata overlaid with ``req.meta``; keys ``detection_threshold`` (0.3),
``recognition_threshold`` (0.5), ``use_angle_cls``, ``ocr.box_thresh`` (0.6),
``ocr.unclip_ratio`` (1.5); response meta ``duration_ms``, ``result_schema`` ocr_v1; every
failure (including unknown tasks) -> ``ERROR_CODE_INTERNAL``.
"""
from __future__ import annotations

import logging
import time
from typing import Optional

from ...proto import ml_service as pb
from ...resources import schemas as rs
from ...resources.config import ModelConfig, Services
from ..base import BaseInferenceService, RuntimeModelInfo
from ..common import backend_settings, load_model_resources, pick_model
from .backend import MI355XOcrBackend, OcrResult, create_backend

log = logging.getLogger("lumen.ocr")

OCR_MIMES = ["image/jpeg", "image/png", "image/bmp", "image/webp"]
OCR_KEYS = ("general", "ocr", "general_ocr", "ppocr")


class OcrModelManager:
    def __init__(self, config: ModelConfig, cache_dir, settings=None, backend: Optional[MI355XOcrBackend] = None):
        self.config = config
        self.cache_dir = cache_dir
        self.settings = settings
        self.backend = backend
        self.resources = backend.resources if backend is not None else None
        self.is_initialized = False
        self._load_time = 0.0

    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        if self.backend is None:
            self.resources = load_model_resources(self.cache_dir, self.config, ("lumen_ocr_config.json",))
            self.backend = create_backend(self.settings, self.resources, self.config.runtime.value)
        self.backend.initialize()
        self._load_time = time.time() - t0
        self.is_initialized = True

    def predict(self, image_bytes: bytes, det_threshold: float = 0.3, rec_threshold: float = 0.5,
                use_angle_cls: bool = False, **kwargs) -> list[OcrResult]:
        if not self.is_initialized:
            self.initialize()
        return self.backend.predict(image_bytes, det_threshold, rec_threshold, use_angle_cls, **kwargs)

    def get_info(self) -> RuntimeModelInfo:
        if not self.is_initialized or self.backend is None:
            return RuntimeModelInfo(model_name=self.config.model, model_id=f"{self.config.model}_uninitialized")
        bi = self.backend.get_info()
        return RuntimeModelInfo(model_name=self.config.model, model_id=f"{self.config.model}_{self.config.runtime.value}",
                                runtime=bi.runtime, device=str(bi.device), precisions=list(bi.precisions),
                                model_version=bi.version, load_time=self._load_time, extra=dict(bi.extra))

    info = get_info

    def close(self):
        if self.backend is not None:
            self.backend.close()


def _f(v, default: float) -> float:
    if v is None:
        return default
    try:
        return float(v)
    except (TypeError, ValueError):
        return default


class GeneralOcrService(BaseInferenceService):
    SERVICE_NAME = "ocr"
    PIPELINE = 64   # one stream's requests batch together (services/base.py Infer)
    LATENCY_KEY = "duration_ms"
    UNKNOWN_TASK_CODE = pb.ERROR_CODE_INTERNAL
    DEFAULT_TASK = "ocr"

    def __init__(self, manager: OcrModelManager):
        super().__init__()
        self.manager = manager
        self.registry.register_task("ocr", self._handle_ocr, "Optical Character Recognition", OCR_MIMES, rs.MIME_OCR)

    @classmethod
    def from_config(cls, service_config: Services, cache_dir) -> "GeneralOcrService":
        mc = pick_model(service_config, OCR_KEYS)
        if mc is None:
            raise ValueError("No OCR model configured")
        return cls(OcrModelManager(mc, cache_dir, backend_settings(service_config)))

    def _initialize(self):
        self.manager.initialize()

    def engine_spec(self):
        """DBNet + SVTR on the GPU engines (the front end decodes nothing: JPEG bytes go whole)."""
        m = self.manager
        res = m.resources or load_model_resources(m.cache_dir, m.config, ("lumen_ocr_config.json",))
        from .backend import engine_spec

        return engine_spec(res)

    def close(self):
        self.manager.close()

    def _request_meta(self, req, context) -> dict:
        meta = {}
        if context is not None and hasattr(context, "invocation_metadata"):
            try:
                meta.update({k: v for k, v in context.invocation_metadata() if isinstance(v, str)})
            except Exception:  # pragma: no cover
                pass
        meta.update(dict(req.meta))
        return meta

    def _handle_ocr(self, payload: bytes, mime: str, meta: dict):
        results = self.manager.predict(
            payload, det_threshold=_f(meta.get("detection_threshold"), 0.3),
            rec_threshold=_f(meta.get("recognition_threshold"), 0.5),
            use_angle_cls=str(meta.get("use_angle_cls", "false")).lower() == "true",
            box_thresh=_f(meta.get("ocr.box_thresh"), 0.6), unclip_ratio=_f(meta.get("ocr.unclip_ratio"), 1.5))
        items = [rs.Item(box=[rs.BoxItem(root=[int(x), int(y)]) for x, y in r.box], text=r.text,
                         confidence=float(r.confidence)) for r in results]
        out = rs.OCRV1(items=items, count=len(items), model_id=self.manager.get_info().model_id)
        return rs.dumps(out), rs.MIME_OCR, {}

    def build_capability(self):
        if not self.is_initialized:
            self.initialize()
        info = self.manager.get_info()
        bi = self.manager.backend.get_info()
        return self.registry.build_capability(self.SERVICE_NAME, info.model_id, bi.runtime, list(bi.precisions),
                                              {k: str(v) for k, v in bi.extra.items()})
