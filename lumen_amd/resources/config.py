"""LumenConfig — the YAML deployment configuration (wire/on-disk compatible).

Field-for-field the same schema as the reference's generated models
(packages/lumen-resources/src/lumen_resources/lumen_config.py:13-256 and
schemas/config-schema.yaml): metadata / deployment (single | hub) / server /
services.<name>{enabled, package, import_info, backend_settings, models}.
``BackendSettings`` forbids extra keys, so MI355X-specific knobs (dp/tp size,
max batch, KV blocks) live in :class:`lumen_amd.resources.config.AmdRuntimeSettings`
read from the environment / a side file, and reference configs validate unchanged.
"""
from __future__ import annotations

import os
from enum import Enum
from typing import Any, Literal, Optional, Union

from pydantic import BaseModel, ConfigDict, Field, RootModel


class Region(Enum):
    """`cn` -> ModelScope; `other` currently also resolves to ModelScope (reference behaviour)."""

    cn = "cn"
    other = "other"


class Metadata(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    version: str = Field(..., pattern=r"^\d+\.\d+\.\d+$")
    region: Region
    cache_dir: str


class Mode(Enum):
    single = "single"
    hub = "hub"


class Service(RootModel[str]):
    root: str = Field(..., pattern=r"^[a-z][a-z0-9_]*$")


class Deployment(BaseModel):
    """Single-service deployment."""

    model_config = ConfigDict(populate_by_name=True)
    mode: Literal["single"]
    service: str = Field(..., pattern=r"^[a-z][a-z0-9_]*$")
    services: Optional[list[Service]] = Field(None, min_length=1)


class Deployment1(BaseModel):
    """Hub deployment (several services behind one port)."""

    model_config = ConfigDict(populate_by_name=True)
    mode: Literal["hub"]
    service: Optional[str] = Field(None, pattern=r"^[a-z][a-z0-9_]*$")
    services: list[Service] = Field(..., min_length=1)


class Mdns(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    enabled: Optional[bool] = False
    service_name: Optional[str] = Field(None, pattern=r"^[a-z][a-z0-9-]*$")


class Server(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    port: int = Field(..., ge=1024, le=65535)
    host: Optional[str] = "0.0.0.0"
    mdns: Optional[Mdns] = None


class ImportInfo(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    registry_class: str = Field(..., pattern=r"^[a-z_][a-z0-9_.]*\.[A-Z][a-zA-Z0-9]*$")
    add_to_server: str = Field(..., pattern=r"^[a-z_][a-z0-9_.]*\.add_[A-Za-z0-9_]+_to_server$")


class BackendSettings(BaseModel):
    model_config = ConfigDict(extra="forbid", populate_by_name=True)
    device: Optional[str] = None
    batch_size: Optional[int] = Field(8, ge=1)
    onnx_providers: Optional[list[Any]] = None


class Runtime(Enum):
    torch = "torch"
    onnx = "onnx"
    rknn = "rknn"


class ModelConfig(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    model: str
    runtime: Runtime
    rknn_device: Optional[str] = Field(None, pattern=r"^rk\d+$")
    dataset: Optional[str] = None
    precision: Optional[str] = None


class Services(BaseModel):
    model_config = ConfigDict(populate_by_name=True)
    enabled: bool
    package: str = Field(..., pattern=r"^[a-z][a-z0-9_]*$")
    import_info: ImportInfo
    backend_settings: Optional[BackendSettings] = None
    models: dict[str, ModelConfig]


class LumenConfig(BaseModel):
    """Unified configuration schema for all Lumen ML services."""

    model_config = ConfigDict(extra="forbid", populate_by_name=True)
    metadata: Metadata
    deployment: Union[Deployment, Deployment1]
    server: Server
    services: dict[str, Services]

    # ---- helpers (not part of the schema)
    def enabled_services(self) -> dict[str, Services]:
        return {k: v for k, v in self.services.items() if v.enabled}

    def cache_path(self) -> str:
        return os.path.expanduser(self.metadata.cache_dir)


class AmdRuntimeSettings(BaseModel):
    """MI355X runtime knobs kept OUT of the reference schema (env: LUMEN_*).

    dp_size      data-parallel GPU workers for CLIP/face/OCR (image-batch DP)
    tp_size      tensor-parallel degree of the VLM decoder
    max_batch    dynamic batcher cap (images per GPU per batch)
    max_wait_ms  dynamic batcher flush deadline
    kv_blocks    paged-KV blocks per GPU for the VLM (0 = size from free HBM)
    synthetic    allow random-init synthetic models when artefacts are absent
    """

    dp_size: int = 1
    tp_size: int = 1
    max_batch: int = 256
    max_wait_ms: float = 2.0
    kv_blocks: int = 0
    synthetic: bool = False

    @staticmethod
    def from_env() -> "AmdRuntimeSettings":
        def _i(name, d):
            return int(os.environ.get(name, d))

        return AmdRuntimeSettings(
            dp_size=_i("LUMEN_DP_SIZE", 1),
            tp_size=_i("LUMEN_TP_SIZE", 1),
            max_batch=_i("LUMEN_MAX_BATCH", 256),
            max_wait_ms=float(os.environ.get("LUMEN_MAX_WAIT_MS", 2.0)),
            kv_blocks=_i("LUMEN_KV_BLOCKS", 0),
            synthetic=os.environ.get("LUMEN_SYNTHETIC", "0") == "1",
        )
