"""Model resolver / downloader.

Behaviour mirrors packages/lumen-resources/src/lumen_resources/downloader.py:19-513:
for every enabled ``service:alias`` it computes the file patterns for the
requested runtime/precision, fetches the repository snapshot into
``<cache_dir>/models/<repo>``, validates ``model_info.json`` (runtime available,
dataset present, rknn device supported), fetches dataset files and verifies
that every required file exists, rolling the model directory back on failure.

MI355X build differences:
* the platform layer (ModelScope / HF hub, reference platform.py:30-270) is used
  only when its SDK is importable and the network is reachable; an already
  populated cache is accepted as-is (offline-first);
* ``synthetic=True`` (or LUMEN_SYNTHETIC=1) materialises a random-init model
  directory of the right architecture when nothing is cached (benchmarks/tests,
  see :mod:`lumen_amd.resources.synthetic`).
"""
from __future__ import annotations

import fnmatch
import logging
import os
import shutil
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional

from .config import LumenConfig, ModelConfig, Region, Runtime
from .exceptions import DownloadError, ModelInfoError, PlatformUnavailableError
from .model_info import ModelInfo, load_and_validate_model_info

log = logging.getLogger("lumen.resources")

HF_OWNER = "Lumilio-Photos"
MODELSCOPE_OWNER = "LumilioPhotos"


@dataclass
class DownloadResult:
    model_type: str
    model_path: Optional[Path] = None
    success: bool = False
    error: Optional[str] = None
    missing_files: list[str] = field(default_factory=list)
    synthetic: bool = False


def file_patterns(runtime: Runtime, precision: Optional[str], rknn_device: Optional[str] = None) -> list[str]:
    """Glob patterns of the artefacts a runtime needs (reference downloader.py:179-251)."""
    common = ["model_info.json", "*config*.json", "tokenizer*", "*vocab*", "*merges*", "*.txt", "*.model",
              "preprocessor_config.json", "special_tokens_map.json"]
    if runtime == Runtime.torch:
        return common + ["*.bin", "*.pt", "*.pth", "*.safetensors"]
    if runtime == Runtime.onnx:
        if precision:
            return common + [f"onnx/*.{precision}.onnx", f"onnx/*.{precision}.onnx.data", "onnx/*.onnx_data"]
        return common + ["onnx/*.onnx", "onnx/*.onnx.data"]
    if runtime == Runtime.rknn:
        dev = rknn_device or "*"
        return common + [f"rknn/{dev}/*.rknn"]
    return common


class Platform:
    """Snapshot fetcher (ModelScope / HF). Unavailable offline -> PlatformUnavailableError."""

    def __init__(self, region: Region, cache_dir: Path):
        self.region = region
        self.cache_dir = cache_dir
        # the reference routes both regions to ModelScope for now (downloader.py:81-121)
        self.kind = "modelscope"
        self.owner = MODELSCOPE_OWNER

    def repo_id(self, model: str) -> str:
        return f"{self.owner}/{model}"

    def model_dir(self, model: str) -> Path:
        return self.cache_dir / "models" / model

    def download_model(self, model: str, patterns: list[str], force: bool = False) -> Path:
        target = self.model_dir(model)
        if target.exists() and (target / "model_info.json").exists() and not force:
            return target
        try:
            if self.kind == "modelscope":
                from modelscope import snapshot_download  # type: ignore
            else:
                from huggingface_hub import snapshot_download  # type: ignore
        except Exception as e:  # pragma: no cover - depends on environment
            raise PlatformUnavailableError(f"{self.kind} SDK unavailable ({e}); and {target} is not cached") from e
        try:  # pragma: no cover - needs network
            path = snapshot_download(self.repo_id(model), local_dir=str(target), allow_patterns=patterns)
        except Exception as e:  # pragma: no cover
            raise DownloadError(f"snapshot of {self.repo_id(model)} failed: {e}") from e
        return Path(path)

    def cleanup_model(self, model: str) -> None:
        shutil.rmtree(self.model_dir(model), ignore_errors=True)


class Downloader:
    def __init__(self, config: LumenConfig, verbose: bool = False, synthetic: Optional[bool] = None):
        self.config = config
        self.verbose = verbose
        self.cache_dir = Path(config.cache_path())
        self.platform = Platform(config.metadata.region, self.cache_dir)
        self.synthetic = synthetic if synthetic is not None else os.environ.get("LUMEN_SYNTHETIC", "0") == "1"

    def download_all(self, force: bool = False) -> dict[str, DownloadResult]:
        results: dict[str, DownloadResult] = {}
        for svc_name, svc in self.config.enabled_services().items():
            for alias, mc in svc.models.items():
                key = f"{svc_name}:{alias}"
                results[key] = self._download_one(key, svc_name, mc, force)
        return results

    # ------------------------------------------------------------------
    def _download_one(self, key: str, svc_name: str, mc: ModelConfig, force: bool) -> DownloadResult:
        res = DownloadResult(model_type=key)
        target = self.platform.model_dir(mc.model)
        created = not target.exists()
        try:
            patterns = file_patterns(mc.runtime, mc.precision, mc.rknn_device)
            try:
                path = self.platform.download_model(mc.model, patterns, force=force)
            except (PlatformUnavailableError, DownloadError):
                if not self.synthetic:
                    raise
                from .synthetic import write_synthetic_model

                path = write_synthetic_model(self.cache_dir, mc.model, service=svc_name, dataset=mc.dataset)
                res.synthetic = True
            info = load_and_validate_model_info(path)
            self._validate_model_config(info, mc)
            res.missing_files = self._missing_files(path, info, mc)
            if res.missing_files:
                raise DownloadError(f"missing files for {key}: {res.missing_files}")
            res.model_path = path
            res.success = True
        except Exception as e:
            res.error = str(e)
            res.success = False
            if created and target.exists() and not res.synthetic:
                self.platform.cleanup_model(mc.model)  # rollback (reference downloader.py:371-380)
        return res

    @staticmethod
    def _validate_model_config(info: ModelInfo, mc: ModelConfig) -> None:
        rt = mc.runtime.value
        if rt not in info.runtimes or not info.runtimes[rt].available:
            raise ModelInfoError(f"runtime '{rt}' not available for {info.name} (have {list(info.runtimes)})")
        if mc.runtime == Runtime.rknn:
            devs = info.runtimes[rt].devices or []
            if mc.rknn_device not in devs:
                raise ModelInfoError(f"rknn device {mc.rknn_device} not supported by {info.name}: {devs}")
        if mc.dataset:
            if not info.datasets or mc.dataset not in info.datasets:
                raise ModelInfoError(f"dataset '{mc.dataset}' not declared by {info.name}")

    @staticmethod
    def _missing_files(path: Path, info: ModelInfo, mc: ModelConfig) -> list[str]:
        rt = info.runtimes[mc.runtime.value]
        files = rt.files or []
        if isinstance(files, dict):
            files = files.get(mc.rknn_device or "", []) if mc.runtime == Runtime.rknn else sum(files.values(), [])
        missing = []
        for f in files:
            if mc.precision and mc.runtime == Runtime.onnx and f.endswith(".onnx"):
                # only the requested precision must exist
                if f".{mc.precision}." not in f and any(p in f for p in (".fp32.", ".fp16.", ".int8.", ".q4fp16.")):
                    continue
            if not (path / f).exists() and not any(fnmatch.fnmatch(str(p.relative_to(path)), f)
                                                    for p in path.rglob("*")):
                missing.append(f)
        if mc.dataset and info.datasets and mc.dataset in info.datasets:
            ds = info.datasets[mc.dataset]
            for f in (ds.labels, ds.embeddings):
                if not (path / f).exists():
                    missing.append(f)
        return missing
