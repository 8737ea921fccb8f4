"""GeneralFaceService (L4) — reference packages/lumen-face/src/lumen_face/general_face/
face_service.py:41-621.

Tasks: ``face_detect`` -> face_v1, ``face_embed`` -> embedding_v1
(optional ``landmarks`` meta ``[{x,y}x5]``), ``face_detect_and_embed`` -> face_v1 with an
embedding per face (+ ``max_faces``).  Meta: ``detection_confidence_threshold`` 0.7,
``nms_threshold`` 0.4, ``face_size_min`` 50, ``face_size_max`` 1000 (int-like parsing);
response meta ``face_count`` / ``dim`` + ``processing_time_ms``.  Unknown tasks map to
``ERROR_CODE_INTERNAL`` like the reference.  ``face_embed`` serialises via the pydantic
model (the reference ``json.dumps(EmbeddingV1)`` raises TypeError — SURVEY §A.6 Q5).
"""
from __future__ import annotations

import json
import logging

from ...proto import ml_service as pb
from ...resources import schemas as rs
from ...resources.exceptions import ResourceNotFoundError
from ..base import IMAGE_MIMES, BaseInferenceService
from ..common import backend_settings, load_model_resources, pick_model
from .backend import create_backend
from .model import FaceModelManager

log = logging.getLogger("lumen.face.service")

FACE_KEYS = ("general", "face", "general_face", "buffalo_l", "antelopev2")


def _int_like(v, default: int) -> int:
    try:
        return int(float(v))
    except (TypeError, ValueError):
        return default


def _float(v, default: float) -> float:
    try:
        return float(v)
    except (TypeError, ValueError):
        return default


def _det_params(meta: dict):
    return dict(detection_confidence_threshold=_float(meta.get("detection_confidence_threshold", "0.7"), 0.7),
                nms_threshold=_float(meta.get("nms_threshold", "0.4"), 0.4),
                face_size_min=_int_like(meta.get("face_size_min", "50"), 50),
                face_size_max=_int_like(meta.get("face_size_max", "1000"), 1000))


def _face(f, embedding=None) -> rs.Face:
    return rs.Face(bbox=[rs.BboxItem(root=max(float(c), 0.0)) for c in f.bbox],
                   confidence=min(max(float(f.confidence), 0.0), 1.0),
                   landmarks=[float(c) for p in f.landmarks for c in p] if f.landmarks else None,
                   embedding=[float(x) for x in embedding] if embedding is not None else None)


class GeneralFaceService(BaseInferenceService):
    SERVICE_NAME = "face-general"
    PIPELINE = 64   # one stream's requests batch together (services/base.py Infer)
    LATENCY_KEY = "processing_time_ms"
    UNKNOWN_TASK_CODE = pb.ERROR_CODE_INTERNAL

    def __init__(self, backend, resources):
        super().__init__()
        self.backend = backend
        self.resources = resources
        self.model = FaceModelManager(backend, resources)
        self._setup_registry()

    def engine_spec(self):
        from .backend import engine_spec

        return engine_spec(self.resources, self.backend.max_batch)

    @classmethod
    def from_config(cls, service_config, cache_dir) -> "GeneralFaceService":
        mc = pick_model(service_config, FACE_KEYS)
        if mc is None:
            raise ValueError("No face model configured")
        try:
            resources = load_model_resources(cache_dir, mc, ("lumen_face_config.json",))
        except Exception as e:
            raise ResourceNotFoundError(f"Failed to load resources for {mc.model}: {e}") from e
        return cls(create_backend(backend_settings(service_config), resources, mc.runtime.value), resources)

    def _setup_registry(self):
        r = self.registry
        r.register_task("face_detect", self._handle_detect, "Detect faces (bbox, confidence, 5 landmarks)",
                        IMAGE_MIMES, rs.MIME_FACE)
        r.register_task("face_embed", self._handle_embed, "Embed a face crop (optional 5-point alignment)",
                        IMAGE_MIMES, rs.MIME_EMBEDDING)
        r.register_task("face_detect_and_embed", self._handle_detect_and_embed,
                        "Detect faces and embed each of them", IMAGE_MIMES, rs.MIME_FACE)

    def _initialize(self):
        self.model.initialize()

    def close(self):
        self.model.close()

    # ---------------------------------------------------------------- handlers
    def _model_id(self) -> str:
        return self.model.get_info().model_id

    def _handle_detect(self, payload: bytes, mime: str, meta: dict):
        faces = self.model.detect_faces(payload, **_det_params(meta))
        out = rs.FaceV1(faces=[_face(f) for f in faces], count=len(faces), model_id=self._model_id())
        return rs.dumps(out), rs.MIME_FACE, {"face_count": str(len(faces))}

    def _handle_embed(self, payload: bytes, mime: str, meta: dict):
        landmarks = None
        if "landmarks" in meta:
            try:
                landmarks = [(float(p["x"]), float(p["y"])) for p in json.loads(meta["landmarks"])]
            except (json.JSONDecodeError, KeyError, TypeError, ValueError):
                log.warning("Invalid landmarks format in meta, proceeding without alignment")
        vec = self.model.extract_embedding(face_image=payload, landmarks=landmarks)
        out = rs.EmbeddingV1(vector=[float(x) for x in vec], dim=len(vec), model_id=self._model_id())
        return rs.dumps(out), rs.MIME_EMBEDDING, {"dim": str(len(vec))}

    def _handle_detect_and_embed(self, payload: bytes, mime: str, meta: dict):
        max_faces = _int_like(meta.get("max_faces", "-1"), -1)
        pairs = self.model.detect_and_extract(payload, max_faces=max_faces, **_det_params(meta))
        out = rs.FaceV1(faces=[_face(f, e) for f, e in pairs], count=len(pairs), model_id=self._model_id())
        return rs.dumps(out), rs.MIME_FACE, {"face_count": str(len(pairs))}

    # ---------------------------------------------------------------- capabilities
    def build_capability(self):
        bi = self.backend.get_info()
        extra = {"model_name": self.resources.model_name, "model_id": bi.model_id,
                 "face_embedding_dim": str(bi.embedding_dim or 512), "supports_landmarks": "true"}
        extra.update({k: str(v) for k, v in bi.extra.items() if v is not None})
        return self.registry.build_capability(self.SERVICE_NAME, bi.model_id, bi.runtime, list(bi.precisions), extra)
