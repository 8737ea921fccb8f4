"""Result schemas returned in ``InferResponse.result`` (JSON; wire compatible).

EmbeddingV1 / LabelsV1 / FaceV1 / OCRV1 / TextGenerationV1 with the same field
names and constraints as packages/lumen-resources/src/lumen_resources/result_schemas/
(embedding_v1.py:10, labels_v1.py:10-40, face_v1.py:10-56, ocr_v1.py:10-54,
text_generation_v1.py:12-89). All forbid extra keys.
"""
from __future__ import annotations

import json
from enum import Enum
from typing import Optional

from pydantic import BaseModel, ConfigDict, Field, RootModel


class EmbeddingV1(BaseModel):
    model_config = ConfigDict(extra="forbid")
    vector: list[float] = Field(..., min_length=1)
    dim: int = Field(..., ge=1)
    model_id: str = Field(..., min_length=1)


class Label(BaseModel):
    model_config = ConfigDict(extra="forbid")
    label: str
    score: float


class LabelsV1(BaseModel):
    model_config = ConfigDict(extra="forbid")
    labels: list[Label]
    model_id: str = Field(..., min_length=1)


class BboxItem(RootModel[float]):
    root: float = Field(..., ge=0.0)


class Face(BaseModel):
    model_config = ConfigDict(extra="forbid")
    bbox: list[BboxItem] = Field(..., min_length=4, max_length=4)
    confidence: float = Field(..., ge=0.0, le=1.0)
    landmarks: Optional[list[float]] = None
    embedding: Optional[list[float]] = None


class FaceV1(BaseModel):
    model_config = ConfigDict(extra="forbid")
    faces: list[Face]
    count: int = Field(..., ge=0)
    model_id: str = Field(..., min_length=1)


class BoxItem(RootModel[list[int]]):
    root: list[int] = Field(..., min_length=2, max_length=2)


class Item(BaseModel):
    model_config = ConfigDict(extra="forbid")
    box: list[BoxItem] = Field(..., min_length=3)
    text: str
    confidence: float = Field(..., ge=0.0, le=1.0)


class OCRV1(BaseModel):
    model_config = ConfigDict(extra="forbid")
    items: list[Item]
    count: int = Field(..., ge=0)
    model_id: str = Field(..., min_length=1)


class FinishReason(Enum):
    stop = "stop"
    length = "length"
    eos_token = "eos_token"
    stop_sequence = "stop_sequence"
    error = "error"


class GenMetadata(BaseModel):
    model_config = ConfigDict(extra="forbid")
    temperature: Optional[float] = Field(None, ge=0.0)
    top_p: Optional[float] = Field(None, ge=0.0, le=1.0)
    max_tokens: Optional[int] = Field(None, ge=1)
    seed: Optional[int] = None
    generation_time_ms: Optional[float] = Field(None, ge=0.0)
    streaming_chunks: Optional[int] = Field(None, ge=0)


class TextGenerationV1(BaseModel):
    model_config = ConfigDict(extra="forbid")
    text: str = Field(..., min_length=0)
    finish_reason: FinishReason
    generated_tokens: int = Field(..., ge=0)
    input_tokens: Optional[int] = Field(None, ge=0)
    model_id: str = Field(..., min_length=1)
    metadata: Optional[GenMetadata] = None


def dumps(model: BaseModel) -> bytes:
    """Compact JSON bytes (the services emit separators=(',', ':'))."""
    return json.dumps(model.model_dump(mode="json"), separators=(",", ":"), ensure_ascii=False).encode("utf-8")


# MIME strings used on the wire
MIME_EMBEDDING = "application/json;schema=embedding_v1"
MIME_LABELS = "application/json;schema=labels_v1"
MIME_FACE = "application/json;schema=face_v1"
MIME_OCR = "application/json;schema=ocr_v1"
MIME_TEXT_GEN = "application/json;schema=text_generation_v1"
