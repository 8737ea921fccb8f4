"""Hardware / driver detection (reference lumen-app/src/lumen_app/utils/env_checker.py and
api/hardware.py:115-238), extended with ROCm / gfx950 detection for the MI355X preset."""
from __future__ import annotations

import os
import platform
import shutil
from pathlib import Path
from typing import Optional

from . import presets as P
from .schemas import DriverCheckResponse, HardwareInfoResponse, HardwarePresetResponse


def rocm_version() -> Optional[str]:
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        try:
            return Path(p).read_text().strip()
        except OSError:
            continue
    return None


def gpus() -> list[dict]:
    """Visible GPUs (gfx arch, memory).  Counting does not initialise HIP on this image."""
    try:
        import torch

        n = torch.cuda.device_count()
        out = []
        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            out.append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""),
                        "memory_gb": round(p.total_memory / 2 ** 30, 1), "cu": p.multi_processor_count})
        return out
    except Exception:  # noqa: BLE001
        return []


def check_driver(name: str) -> DriverCheckResponse:
    if name == "rocm":
        v = rocm_version()
        return DriverCheckResponse(name="rocm", status="available" if v else "missing", details=f"ROCm {v}" if v else
                                   "/opt/rocm not found")
    if name == "hip_runtime":
        try:
            import torch

            hip = torch.version.hip
        except Exception:  # noqa: BLE001
            hip = None
        if not hip:
            return DriverCheckResponse(name=name, status="missing", details="PyTorch built without HIP")
        g = gpus()
        if g and not any(x["arch"].startswith("gfx950") for x in g):
            return DriverCheckResponse(name=name, status="incompatible",
                                       details=f"HIP {hip}; GPUs {[x['arch'] for x in g]} (gfx950 kernels)")
        return DriverCheckResponse(name=name, status="available",
                                   details=f"HIP {hip}; {len(g)} GPU(s) {[x['arch'] for x in g]}")
    if name == "lumen_native":
        from .._native import HIP_SO, HOST_SO

        ok = HIP_SO.exists() and HOST_SO.exists()
        return DriverCheckResponse(name=name, status="available" if ok else "missing",
                                   details="gfx950 kernel library built" if ok else "run: python -m lumen_amd._build")
    if name == "cuda":
        try:
            import torch

            ok = bool(torch.version.cuda)
        except Exception:  # noqa: BLE001
            ok = False
        return DriverCheckResponse(name=name, status="available" if ok else "missing",
                                   details="CUDA runtime" if ok else "no CUDA runtime (ROCm build)")
    if name == "coreml":
        return DriverCheckResponse(name=name, status="available" if platform.system() == "Darwin" else "missing")
    return DriverCheckResponse(name=name, status="missing", details=f"{name} runtime not present in this build")


def preset_response(p: P.PresetInfo, check: bool = True) -> HardwarePresetResponse:
    dc = p.create_config()
    drivers = [check_driver(d) for d in dc.drivers] if check else []
    ok = all(d.status == "available" for d in drivers)
    supported = P.supported_here(p)
    avail = "not_checked" if not check else ("incompatible" if not supported else ("ready" if ok else "missing_drivers"))
    return HardwarePresetResponse(name=p.name, description=p.description, requires_drivers=p.requires_drivers,
                                  runtime=dc.runtime.value, providers=list(dc.onnx_providers or []),
                                  supported_on_current_platform=supported, supported_systems=list(p.supported_systems),
                                  environment_checked=check, availability=avail, ready=check and ok and supported,
                                  drivers=drivers, missing_installable=[])


def recommend() -> str:
    for name in P.detection_order():
        r = preset_response(P.PRESETS[name])
        if r.ready:
            return name
    return "cpu"


def hardware_info() -> HardwareInfoResponse:
    pres = [preset_response(P.PRESETS[n]) for n in P.detection_order()]
    rec = next((p.name for p in pres if p.ready), "cpu")
    drivers = next(p.drivers for p in pres if p.name == rec)
    return HardwareInfoResponse(platform=platform.system(), machine=platform.machine(),
                                processor=platform.processor() or platform.machine(),
                                python_version=platform.python_version(), presets=pres, recommended_preset=rec,
                                drivers=drivers, all_drivers_available=all(d.status == "available" for d in drivers),
                                missing_installable=[], gpus=gpus())


def free_space_gb(path: str) -> float:
    p = Path(os.path.expanduser(path))
    while not p.exists() and p != p.parent:
        p = p.parent
    return shutil.disk_usage(str(p)).free / 2 ** 30
