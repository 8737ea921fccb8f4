"""CLIP / BioCLIP model managers (L3 business logic).

Behaviour parity with the reference managers:
* CLIPModelManager (packages/lumen-clip/src/lumen_clip/general_clip/clip_model.py:48-403):
  label bank from the dataset (computes ``"a photo of a {label}"`` embeddings when the
  manifest has none), 8 fixed scene prompts, ``encode_text`` prepends
  ``"a photo of a "``, ``classify_image`` = softmax(100 * cos) over the bank -> top-k,
  ``classify_scene`` = softmax of raw cosines over the scene prompts, label = prompt
  minus "a photo of " / "an ".
* BioCLIPModelManager (expert_bioclip/bioclip_model.py:45-379): TreeOfLife label names
  (common name, else "Genus species"), bank prompt ``"a photo of {name}"``, query prompt
  ``"a photo of a {text}"``, classification = raw cosine top-k (no softmax), bank
  auto-transposed if stored (D, N).
Scoring runs on the GPU against a device-resident :class:`LabelBank`.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Optional

import numpy as np

from ...runtime.label_bank import LabelBank, PoolShardedBank, orient_bank
from ..base import RuntimeModelInfo
from .backend import MI355XClipBackend

log = logging.getLogger("lumen.clip.model")

SCENE_PROMPTS = [
    "a photo of a person",
    "a photo of an animal",
    "a photo of a vehicle",
    "a photo of food",
    "a photo of a building",
    "a photo of nature",
    "a photo of an object",
    "a photo of a landscape",
]


class CLIPModelManager:
    def __init__(self, backend: MI355XClipBackend, resources=None, dataset: Optional[str] = None):
        self.backend = backend
        self.resources = resources or backend.resources
        self.dataset = dataset or self.resources.dataset
        self.labels: list[str] = [str(x) for x in self.resources.labels] if self.resources.labels is not None else []
        self.text_embeddings: Optional[np.ndarray] = None
        self.scene_prompts = list(SCENE_PROMPTS)
        self.scene_prompt_embeddings: Optional[np.ndarray] = None
        self.bank: Optional[LabelBank] = None
        self.scene_bank: Optional[LabelBank] = None
        self.is_initialized = False
        self._load_time = 0.0

    @property
    def supports_classification(self) -> bool:
        return bool(self.labels)

    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        self.backend.initialize()
        if self.labels:
            emb = self.resources.label_embeddings
            if emb is None:
                emb = self.backend.text_batch_to_vectors([f"a photo of a {l}" for l in self.labels])
            self.text_embeddings = np.asarray(emb, dtype=np.float32)
            self.bank = LabelBank(self.text_embeddings, self.backend.device)
        self.scene_prompt_embeddings = self.backend.text_batch_to_vectors(self.scene_prompts)
        self.scene_bank = LabelBank(self.scene_prompt_embeddings, self.backend.device)
        self._load_time = time.time() - t0
        self.is_initialized = True

    def _ensure(self):
        if not self.is_initialized:
            raise RuntimeError("CLIP model manager not initialized")

    def encode_image(self, image_bytes: bytes) -> np.ndarray:
        self._ensure()
        return self.backend.image_to_vector(image_bytes)

    def encode_text(self, text: str) -> np.ndarray:
        self._ensure()
        return self.backend.text_to_vector(f"a photo of a {text}")

    def classify_image(self, image_bytes: bytes, top_k: int = 5) -> list[tuple[str, float]]:
        self._ensure()
        if not self.supports_classification or self.bank is None:
            raise RuntimeError("Classification not supported: no dataset loaded")
        emb = self.encode_image(image_bytes)
        if not np.all(np.isfinite(emb)):
            raise RuntimeError("Image embedding contains invalid values (NaN/Inf)")
        p, idx = self.bank.topk(emb, top_k, scale=100.0, softmax=True)
        return [(self.labels[int(i)], float(s)) for s, i in zip(p[0], idx[0])]

    def classify_scene(self, image_bytes: bytes) -> tuple[str, float]:
        self._ensure()
        emb = self.encode_image(image_bytes)
        p, idx = self.scene_bank.topk(emb, 1, scale=1.0, softmax=True)
        label = self.scene_prompts[int(idx[0][0])].replace("a photo of ", "").replace("an ", "")
        return label, float(p[0][0])

    def info(self) -> RuntimeModelInfo:
        bi = self.backend.get_info()
        return RuntimeModelInfo(model_name=self.resources.model_name, model_id=self.resources.model_id,
                                runtime=bi.runtime, device=str(bi.device), precisions=list(bi.precisions),
                                embedding_dim=bi.image_embedding_dim, model_version=self.resources.model_info.version,
                                load_time=self.backend.load_time, supports_classification=self.supports_classification,
                                backend_info=f"{bi.runtime}@{bi.device}")


class BioCLIPModelManager:
    def __init__(self, backend: MI355XClipBackend, resources=None):
        self.backend = backend
        self.resources = resources or backend.resources
        raw = self.resources.labels
        self.raw_labels: list[Any] = list(raw) if raw is not None else []
        self.labels = [self.extract_name(l) for l in self.raw_labels]
        self.text_embeddings: Optional[np.ndarray] = None
        self.bank: Optional[LabelBank] = None
        self.is_initialized = False

    @property
    def supports_classification(self) -> bool:
        return bool(self.labels)

    @staticmethod
    def extract_name(label: Any) -> str:
        if isinstance(label, (list, tuple)) and len(label) == 2:
            taxonomy, common = label
            if isinstance(common, str) and common.strip():
                return common
            if isinstance(taxonomy, (list, tuple)) and len(taxonomy) >= 2:
                return f"{taxonomy[-2]} {taxonomy[-1]}"
        return str(label)

    def initialize(self) -> None:
        if self.is_initialized:
            return
        # with DP workers and a stored bank (TreeOfLife, 10^5-10^6 x 768), every GPU worker
        # holds 1/world of it (K13): queries are broadcast, candidates merged here
        from ...parallel.engine import current_remote

        # serving front end: the engines hold the bank slices (services/clip engine_spec(shard_bank=True))
        shard = self.labels and self.resources.label_embeddings is not None and \
            (self.backend.dp_size > 1 or current_remote() is not None)
        self.backend.shard_bank = bool(shard)
        self.backend.initialize()
        if self.labels:
            dim = self.backend.cfg.embed_dim
            if shard and self.backend._pool is not None:
                emb = orient_bank(self.resources.label_embeddings, len(self.labels), dim)
                self.text_embeddings = emb                  # memory-mapped; never loaded whole here
                self.bank = PoolShardedBank(self.backend._pool, emb.shape[0])
                log.info("BioCLIP bank %d x %d sharded over %d GPU worker(s) / engine(s)", emb.shape[0], emb.shape[1],
                         self.backend._pool.size)
            else:
                emb = self.resources.label_embeddings
                if emb is None:
                    emb = self.backend.text_batch_to_vectors([f"a photo of {n}" for n in self.labels])
                emb = np.asarray(emb, dtype=np.float32)
                if emb.shape[0] != len(self.labels) and emb.shape[1] == len(self.labels) and emb.shape[0] == dim:
                    log.warning("BioCLIP bank stored (D, N); transposing")
                emb = orient_bank(emb, len(self.labels), dim)
                self.text_embeddings = emb
                self.bank = LabelBank(emb, self.backend.device)
        self.is_initialized = True

    def _ensure(self):
        if not self.is_initialized:
            raise RuntimeError("BioCLIP model manager not initialized")

    def encode_image(self, image_bytes: bytes) -> np.ndarray:
        self._ensure()
        return self.backend.image_to_vector(image_bytes)

    def encode_text(self, text: str) -> np.ndarray:
        self._ensure()
        return self.backend.text_to_vector(f"a photo of a {text}")

    def classify_image(self, image_bytes: bytes, top_k: int = 3) -> list[tuple[str, float]]:
        self._ensure()
        if not self.supports_classification or self.bank is None:
            raise RuntimeError("Classification not supported: no dataset loaded")
        emb = self.encode_image(image_bytes)
        s, idx = self.bank.topk(emb, top_k, scale=1.0, softmax=False)
        return [(self.labels[int(i)], float(v)) for v, i in zip(s[0], idx[0])]

    def info(self) -> RuntimeModelInfo:
        bi = self.backend.get_info()
        return RuntimeModelInfo(model_name=self.resources.model_name, model_id=self.resources.model_id,
                                runtime=bi.runtime, device=str(bi.device), precisions=list(bi.precisions),
                                embedding_dim=bi.image_embedding_dim, model_version=self.resources.model_info.version,
                                load_time=self.backend.load_time, supports_classification=self.supports_classification)
