"""Device presets and canned LumenConfig generators.

Reference: lumen-app/src/lumen_app/services/config.py:20-682 (``DeviceConfig`` presets,
``Config.minimal / light_weight / basic / brave``) and utils/preset_registry.py:40-244
(priority-ordered registry, aliases, platform support).  The MI355X build adds the
``amd_mi355x`` preset (runtime ``torch`` = the native HIP path, batch size left to the
dynamic batcher, bf16) which ranks first when gfx950 GPUs are present; the other
presets are kept so configs written for the reference validate and load unchanged
(they all execute on the same native path here).
"""
from __future__ import annotations

import platform
from dataclasses import dataclass, field
from typing import Callable, Literal, Optional

from ..resources.config import (BackendSettings, Deployment1, ImportInfo, LumenConfig, Mdns, Metadata, ModelConfig,
                                Region, Runtime, Server, Service, Services)


@dataclass
class DeviceConfig:
    runtime: Runtime
    onnx_providers: Optional[list] = None
    rknn_device: Optional[str] = None
    batch_size: Optional[int] = None
    description: str = ""
    precision: Optional[str] = None
    env: str = "default"
    os: Optional[str] = None
    device: Optional[str] = None
    drivers: tuple = ()


def _p(name, desc, factory, priority, systems=("Linux", "Windows", "Darwin"), requires_drivers=True):
    return PresetInfo(name, desc, factory, priority, tuple(systems), requires_drivers)


@dataclass
class PresetInfo:
    name: str
    description: str
    factory: Callable[[], DeviceConfig]
    priority: int
    supported_systems: tuple = ("Linux", "Windows", "Darwin")
    requires_drivers: bool = True
    aliases: tuple = ()

    def create_config(self) -> DeviceConfig:
        return self.factory()


PRESETS: dict[str, PresetInfo] = {p.name: p for p in [
    _p("amd_mi355x", "AMD Instinct MI355X (gfx950): native HIP/MFMA kernels, RCCL over xGMI",
       lambda: DeviceConfig(Runtime.torch, None, batch_size=None, precision="bf16", device="cuda",
                            description="AMD Instinct MI355X", drivers=("rocm", "hip_runtime", "lumen_native")),
       1, ("Linux",)),
    _p("nvidia_gpu_high", "Preset for high RAM (>= 12GB) Nvidia GPUs",
       lambda: DeviceConfig(Runtime.onnx, ["TensorrtExecutionProvider", "CUDAExecutionProvider", "CPUExecutionProvider"],
                            precision="fp16", env="tensorrt", drivers=("cuda",)), 5, ("Linux", "Windows")),
    _p("nvidia_gpu", "Preset for low RAM (< 12GB) Nvidia GPUs",
       lambda: DeviceConfig(Runtime.onnx, ["CUDAExecutionProvider", "CPUExecutionProvider"], batch_size=4, env="cuda",
                            drivers=("cuda",)), 10, ("Linux", "Windows")),
    _p("nvidia_jetson_high", "Preset for high RAM (>= 12GB) Nvidia Jetson Devices",
       lambda: DeviceConfig(Runtime.onnx, ["TensorrtExecutionProvider", "CUDAExecutionProvider", "CPUExecutionProvider"],
                            os="linux", drivers=("cuda",)), 12, ("Linux",)),
    _p("nvidia_jetson", "Preset for low RAM (< 12GB) Nvidia Jetson Devices",
       lambda: DeviceConfig(Runtime.onnx, ["CUDAExecutionProvider", "CPUExecutionProvider"], batch_size=1, os="linux",
                            drivers=("cuda",)), 15, ("Linux",)),
    _p("apple_silicon", "Preset for Apple Silicon",
       lambda: DeviceConfig(Runtime.onnx, ["CoreMLExecutionProvider", "CPUExecutionProvider"], batch_size=1,
                            drivers=("coreml",)), 20, ("Darwin",)),
    _p("intel_gpu", "Preset for Intel iGPU or Arc GPU",
       lambda: DeviceConfig(Runtime.onnx, ["OpenVINOExecutionProvider", "CPUExecutionProvider"], batch_size=1,
                            env="openvino", drivers=("openvino",)), 30, ("Linux", "Windows")),
    _p("amd_gpu_win", "Preset for AMD Ryzen GPUs",
       lambda: DeviceConfig(Runtime.onnx, ["DmlExecutionProvider", "CPUExecutionProvider"], batch_size=1,
                            drivers=("directml",)), 35, ("Windows",)),
    _p("amd_npu", "Preset for AMD Ryzen NPUs",
       lambda: DeviceConfig(Runtime.onnx, ["VitisAIExecutionProvider", "CPUExecutionProvider"], batch_size=1,
                            drivers=("vitisai",)), 40, ("Windows",)),
    _p("cpu", "Preset General CPUs",
       lambda: DeviceConfig(Runtime.onnx, ["CPUExecutionProvider"], batch_size=1, device="cpu"), 100,
       requires_drivers=False),
]}
ALIASES = {"mi355x": "amd_mi355x", "rocm": "amd_mi355x", "amd_instinct": "amd_mi355x"}


def canonical(name: str) -> str:
    return ALIASES.get(name, name)


def get_preset(name: str) -> Optional[PresetInfo]:
    return PRESETS.get(canonical(name))


def detection_order() -> list[str]:
    return [p.name for p in sorted(PRESETS.values(), key=lambda p: p.priority)]


def supported_here(p: PresetInfo) -> bool:
    return platform.system() in p.supported_systems


# ----------------------------------------------------------------------------- config generator
_SVC = {
    "ocr": ("lumen_ocr", "lumen_ocr.general_ocr.GeneralOcrService"),
    "clip": ("lumen_clip", "lumen_clip.general_clip.clip_service.GeneralCLIPService"),
    "bioclip": ("lumen_clip", "lumen_clip.expert_bioclip.BioCLIPService"),
    "face": ("lumen_face", "lumen_face.general_face.GeneralFaceService"),
    "vlm": ("lumen_vlm", "lumen_vlm.fastvlm.GeneralFastVLMService"),
}


class Config:
    """Canned configurations (reference services/config.py:272-682)."""

    def __init__(self, cache_dir: str, device_config: DeviceConfig, region: Region, service_name: str,
                 port: Optional[int]):
        self.cache_dir = cache_dir
        self.region = region
        self.port = port or 50051
        self.service_name = service_name
        self.device_config = device_config
        self.runtime = device_config.runtime
        self.rknn_device = device_config.rknn_device

    def default_light_weight_clip_model(self) -> str:
        return "CN-CLIP_ViT-B-16" if self.region == Region.cn else "MobileCLIP2-S2"

    def default_basic_clip_model(self) -> str:
        return "CN-CLIP_ViT-L-14" if self.region == Region.cn else "MobileCLIP2-S4"

    def _service(self, key: str, model: str, batch: int, precision: str, dataset: Optional[str] = None,
                 kind: Optional[str] = None) -> Services:
        pkg, cls = _SVC[kind or key]
        dc = self.device_config
        return Services(enabled=True, package=pkg,
                        import_info=ImportInfo(registry_class=cls,
                                               add_to_server=f"{pkg}.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"),
                        backend_settings=BackendSettings(device=dc.device, batch_size=dc.batch_size or batch,
                                                         onnx_providers=dc.onnx_providers),
                        models={"general": ModelConfig(model=model, runtime=self.runtime, rknn_device=self.rknn_device,
                                                       precision=precision, dataset=dataset)})

    def _config(self, services: dict[str, Services]) -> LumenConfig:
        return LumenConfig(metadata=Metadata(version="1.0.0", region=self.region, cache_dir=self.cache_dir),
                           deployment=Deployment1(mode="hub", services=[Service(root=k) for k in services], service=None),
                           server=Server(port=self.port, host="0.0.0.0",
                                         mdns=Mdns(enabled=True, service_name=self.service_name)),
                           services=services)

    def minimal(self) -> LumenConfig:
        return self._config({"ocr": self._service("ocr", "PP-OCRv5", 1, "fp32")})

    def light_weight(self, clip_model: Optional[str] = None) -> LumenConfig:
        prec = self.device_config.precision or "fp16"
        return self._config({
            "ocr": self._service("ocr", "PP-OCRv5", 1, "fp32"),
            "clip": self._service("clip", clip_model or self.default_light_weight_clip_model(), 1, prec, "ImageNet_1k"),
            "face": self._service("face", "buffalo_l", 1, "fp32"),
        })

    def basic(self, clip_model: Optional[str] = None) -> LumenConfig:
        prec = self.device_config.precision or "fp16"
        return self._config({
            "ocr": self._service("ocr", "PP-OCRv5", 5, self.device_config.precision or "fp32"),
            "clip": self._service("clip", clip_model or self.default_basic_clip_model(), 5, prec, "ImageNet_1k"),
            "face": self._service("face", "antelopev2", 5, "fp32"),
            "vlm": self._service("vlm", "FastVLM-0.5B", 1, self.device_config.precision or "fp16"),
        })

    def brave(self) -> LumenConfig:
        prec = self.device_config.precision or "fp16"
        return self._config({
            "ocr": self._service("ocr", "PP-OCRv5", 5, self.device_config.precision or "fp32"),
            "clip": self._service("clip", "bioclip-2", 5, prec, "TreeOfLife-200M", kind="bioclip"),
            "face": self._service("face", "antelopev2", 5, "fp32"),
            "vlm": self._service("vlm", "FastVLM-0.5B", 1, self.device_config.precision or "fp16"),
        })
