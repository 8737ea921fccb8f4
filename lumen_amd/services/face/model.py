"""FaceModelManager (L3) — reference packages/lumen-face/src/lumen_face/general_face/
face_model.py:45-517: ``detect_faces``, ``extract_embedding``, ``detect_and_extract``,
``compare_faces`` (cosine), ``find_best_match``, ``crop_face_from_image``, ``get_info``.

``detect_and_extract`` decodes the image ONCE and embeds all its faces as one batch
aligned from the full image (the reference re-decodes the image with PIL per face
and embeds faces one by one).  A failed embedding still yields a zero vector like
the reference (:357-364).
"""
from __future__ import annotations

import logging
import time
from typing import Optional, Sequence

import numpy as np

from ..base import RuntimeModelInfo
from .backend import DetParams, FaceDetection, MI355XFaceBackend

log = logging.getLogger("lumen.face.model")


class FaceModelManager:
    def __init__(self, backend: MI355XFaceBackend, resources=None):
        self.backend = backend
        self.resources = resources or backend.resources
        self.is_initialized = False
        self._load_time = 0.0

    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        try:
            self.backend.initialize()
        except Exception as e:
            raise RuntimeError(f"Model initialization failed: {e}") from e
        self._load_time = time.time() - t0
        self.is_initialized = True

    def close(self) -> None:
        self.backend.close()

    # ---------------------------------------------------------------- detection / embedding
    def detect_faces(self, image_bytes: bytes, detection_confidence_threshold: float = 0.7,
                     nms_threshold: float = 0.4, face_size_min: int = 50, face_size_max: int = 1000
                     ) -> list[FaceDetection]:
        return self.backend.image_to_faces(image_bytes, detection_confidence_threshold, nms_threshold, face_size_min,
                                           face_size_max)

    def extract_embedding(self, face_image: Optional[bytes] = None, landmarks: Optional[list] = None,
                          cropped_face_array: Optional[np.ndarray] = None) -> np.ndarray:
        return self.backend.face_to_embedding(face_image=face_image, cropped_face_array=cropped_face_array,
                                              landmarks=landmarks)

    def detect_and_extract(self, image_bytes: bytes, detection_confidence_threshold: float = 0.7,
                           nms_threshold: float = 0.4, face_size_min: int = 50, face_size_max: int = 1000,
                           max_faces: int = -1) -> list[tuple[FaceDetection, np.ndarray]]:
        return self.backend.detect_and_embed(image_bytes, DetParams(detection_confidence_threshold, nms_threshold,
                                                                    face_size_min, face_size_max), max_faces)

    # ---------------------------------------------------------------- comparisons
    @staticmethod
    def compare_faces(embedding1: np.ndarray, embedding2: np.ndarray) -> float:
        a, b = np.asarray(embedding1, np.float32).ravel(), np.asarray(embedding2, np.float32).ravel()
        na, nb = np.linalg.norm(a), np.linalg.norm(b)
        if na == 0 or nb == 0:
            return 0.0
        return float(np.dot(a, b) / (na * nb))

    def find_best_match(self, query_embedding: np.ndarray, candidate_embeddings: Sequence[np.ndarray],
                        threshold: float = 0.4) -> Optional[tuple[int, float]]:
        if len(candidate_embeddings) == 0:
            return None
        c = np.asarray(candidate_embeddings, np.float32).reshape(len(candidate_embeddings), -1)
        q = np.asarray(query_embedding, np.float32).ravel()
        cn = np.linalg.norm(c, axis=1)
        qn = np.linalg.norm(q)
        sims = np.where(cn > 0, c @ q / np.maximum(cn * qn, 1e-12), 0.0)
        i = int(np.argmax(sims))
        return (i, float(sims[i])) if sims[i] >= threshold else None

    def crop_face_from_image(self, image_bytes: bytes, bbox) -> np.ndarray:
        try:
            img = self.backend.decode(image_bytes)
            h, w = img.shape[:2]
            x1, y1, x2, y2 = [int(v) for v in bbox]
            x1, x2 = max(0, min(x1, w)), max(0, min(x2, w))
            y1, y2 = max(0, min(y1, h)), max(0, min(y2, h))
            return img[y1:y2, x1:x2].astype(np.float32)
        except Exception as e:
            log.warning("Failed to crop face: %s", e)
            return np.zeros((112, 112, 3), np.float32)

    # ---------------------------------------------------------------- info
    def get_info(self) -> RuntimeModelInfo:
        bi = self.backend.get_info()
        return RuntimeModelInfo(model_name=self.resources.model_name, model_id=bi.model_id, runtime=bi.runtime,
                                device=str(bi.device), precisions=list(bi.precisions), embedding_dim=bi.embedding_dim,
                                model_version=bi.version, load_time=self._load_time, extra=dict(bi.extra))

    info = get_info
