"""``model_info.json`` manifest schema (on-disk compatible with the reference).

Same fields as packages/lumen-resources/src/lumen_resources/model_info.py:14-101
(name, version, description, model_type, embedding_dim, source{format, repo_id},
runtimes{<rt>: {available, files, devices, requirements}}, datasets{<name>:
{labels, embeddings}}, extra_metadata, metadata).
"""
from __future__ import annotations

import json
from datetime import date
from enum import Enum
from pathlib import Path
from typing import Any, Optional, Union

from pydantic import AwareDatetime, BaseModel, ConfigDict, Field

from .exceptions import ModelInfoError


class Format(Enum):
    huggingface = "huggingface"
    openclip = "openclip"
    modelscope = "modelscope"
    custom = "custom"


class Source(BaseModel):
    model_config = ConfigDict(extra="forbid")
    format: Format
    repo_id: str = Field(..., min_length=1)


class Requirements(BaseModel):
    python: Optional[str] = None
    dependencies: Optional[list[str]] = None


class Runtimes(BaseModel):
    model_config = ConfigDict(extra="forbid")
    available: bool
    files: Optional[Union[list[str], dict[str, list[str]]]] = None
    devices: Optional[list[str]] = None
    requirements: Optional[Requirements] = None


class Datasets(BaseModel):
    model_config = ConfigDict(extra="forbid")
    labels: str
    embeddings: str


class Metadata(BaseModel):
    model_config = ConfigDict(extra="forbid")
    license: Optional[str] = None
    author: Optional[str] = None
    created_at: Optional[date] = None
    updated_at: Optional[AwareDatetime] = None
    tags: Optional[list[str]] = None


class ModelInfo(BaseModel):
    """Schema for Lumen model manifests."""

    model_config = ConfigDict(extra="forbid")
    name: str = Field(..., min_length=1, max_length=100)
    version: str = Field(..., pattern=r"^[0-9]+\.[0-9]+\.[0-9]+$")
    description: str = Field(..., min_length=1, max_length=500)
    model_type: str
    embedding_dim: Optional[int] = Field(None, ge=1, le=100000)
    source: Source
    runtimes: dict[str, Runtimes]
    datasets: Optional[dict[str, Datasets]] = None
    extra_metadata: Optional[dict[str, Any]] = None
    metadata: Optional[Metadata] = None


def model_info_schema_errors(data: Any) -> list[str]:
    """Draft-7 schema check of a parsed manifest (``validate-model-info --schema-only``)."""
    from .jsonschema_lite import SchemaValidator

    return SchemaValidator.from_file(Path(__file__).resolve().parent / "schemas" / "model_info-schema.json").errors(data)


def load_and_validate_model_info(path: Union[str, Path]) -> ModelInfo:
    p = Path(path)
    if p.is_dir():
        p = p / "model_info.json"
    if not p.exists():
        raise ModelInfoError(f"model_info.json not found: {p}")
    try:
        data = json.loads(p.read_text(encoding="utf-8"))
    except json.JSONDecodeError as e:
        raise ModelInfoError(f"invalid JSON in {p}: {e}") from e
    try:
        return ModelInfo.model_validate(data)
    except Exception as e:  # pydantic.ValidationError
        raise ModelInfoError(f"model_info validation failed for {p}: {e}") from e
