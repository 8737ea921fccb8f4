"""Resource loading / device selection shared by the face, OCR and VLM services.

The reference carries four near-identical per-package loaders
(packages/lumen-face/src/lumen_face/resources/loader.py:99-254,
packages/lumen-ocr/src/lumen_ocr/resources/loader.py, packages/lumen-vlm/src/lumen_vlm/
resources/loader.py); one implementation here: ``<cache_dir>/models/<model>/`` +
``model_info.json`` validated, requested runtime must be declared available, the
runtime directory resolved (``onnx/``, ``rknn/<device>/``, else the root) and — like
the face loader — every file the manifest lists for that runtime must exist.
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Optional

import torch

from ..resources.config import BackendSettings, ModelConfig, Runtime, Services
from ..resources.exceptions import ModelInfoError, ResourceNotFoundError, RuntimeNotSupportedError
from ..resources.model_info import ModelInfo, load_and_validate_model_info

log = logging.getLogger("lumen.resources")


@dataclass
class GenericResources:
    model_root_path: Path
    runtime_files_path: Path
    model_name: str
    runtime: str
    model_info: ModelInfo
    precision: Optional[str] = None
    configs: dict = field(default_factory=dict)

    @property
    def model_id(self) -> str:
        return f"{self.model_name}_{self.runtime}"

    def get_model_file(self, filename: str) -> Path:
        for base in (self.runtime_files_path, self.model_root_path):
            p = base / filename
            if p.exists():
                return p
        raise ResourceNotFoundError(f"{filename} not found under {self.model_root_path}")

    def get_embedding_dim(self) -> Optional[int]:
        return int(self.model_info.embedding_dim) if self.model_info.embedding_dim else None

    @property
    def extra(self) -> dict:
        return dict(self.model_info.extra_metadata or {})


def _manifest_files(info: ModelInfo, runtime: str) -> list[str]:
    rt = info.runtimes.get(runtime)
    if rt is None or rt.files is None:
        return []
    files = rt.files
    if isinstance(files, dict):
        out = []
        for v in files.values():
            out.extend(v)
        return out
    return list(files)


def load_json(p: Path) -> dict:
    try:
        return json.loads(Path(p).read_text(encoding="utf-8"))
    except FileNotFoundError as e:
        raise ResourceNotFoundError(f"required file missing: {p}") from e
    except json.JSONDecodeError as e:
        raise ModelInfoError(f"invalid JSON {p}: {e}") from e


def load_model_resources(cache_dir, model_config: ModelConfig, config_files=(), verify_files: bool = True
                         ) -> GenericResources:
    root = Path(cache_dir).expanduser().resolve() / "models" / model_config.model
    if not (root / "model_info.json").exists():
        raise ResourceNotFoundError(f"model_info.json not found in {root}")
    info = load_and_validate_model_info(root / "model_info.json")
    rt = model_config.runtime.value
    if rt not in info.runtimes or not info.runtimes[rt].available:
        raise RuntimeNotSupportedError(f"runtime '{rt}' not available for {info.name}")
    if model_config.runtime == Runtime.onnx:
        rdir = root / "onnx"
    elif model_config.runtime == Runtime.rknn:
        rdir = root / "rknn" / (model_config.rknn_device or "")
    else:
        rdir = root
    if not rdir.exists():
        rdir = root
    if verify_files:
        missing = [f for f in _manifest_files(info, rt) if not ((rdir / f).exists() or (root / f).exists())]
        if missing:
            raise ResourceNotFoundError(f"{info.name}: manifest files missing for runtime {rt}: {missing}")
    configs = {}
    for name in config_files:
        if (root / name).exists():
            configs[name] = load_json(root / name)
    return GenericResources(model_root_path=root, runtime_files_path=rdir, model_name=model_config.model, runtime=rt,
                            model_info=info, precision=model_config.precision, configs=configs)


def pick_device(pref: Optional[str]) -> torch.device:
    """``cpu`` -> fp32 reference path; otherwise the GPU of this rank (LOCAL_RANK)."""
    if pref and pref.startswith("cpu"):
        return torch.device("cpu")
    if torch.cuda.is_available():
        if pref and pref.startswith("cuda"):
            return torch.device(pref)
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


def pick_model(service_config: Services, keys, fallback_first: bool = True) -> Optional[ModelConfig]:
    for k in keys:
        if k in service_config.models:
            return service_config.models[k]
    if fallback_first and service_config.models:
        return next(iter(service_config.models.values()))
    return None


def backend_settings(service_config: Services) -> BackendSettings:
    return service_config.backend_settings or BackendSettings(device=None, batch_size=1, onnx_providers=None)


def load_safetensors(path: Path) -> dict[str, Any]:
    from safetensors.torch import load_file

    return load_file(str(path))


@dataclass
class BackendInfo:
    """Backend description (reference backends/base.py BackendInfo across packages)."""

    runtime: str
    device: Optional[str]
    model_id: str
    model_name: str
    version: str = "1.0.0"
    precisions: tuple = ("bf16",)
    embedding_dim: Optional[int] = None
    extra: dict = field(default_factory=dict)

    def as_dict(self) -> dict:
        return {"runtime": self.runtime, "device": self.device, "model_id": self.model_id,
                "model_name": self.model_name, "version": self.version, "precisions": list(self.precisions),
                "embedding_dim": self.embedding_dim, **{k: v for k, v in self.extra.items()}}


def runtime_name(device: torch.device) -> str:
    return "mi355x-hip" if device.type == "cuda" else "torch-cpu-reference"
