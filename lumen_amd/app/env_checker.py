"""Environment checker (reference lumen-app/src/lumen_app/utils/env_checker.py:27-826):
driver probes per preset, a readiness report, and the driver installer.

Probes cover the reference's accelerators (NVIDIA CUDA / TensorRT, Apple CoreML, Intel
OpenVINO, DirectML, AMD Ryzen-AI NPU, Rockchip RKNN) — reported missing on an MI355X
host with the reason — and the MI355X stack in depth: ROCm install, the amdgpu kernel
driver and ``/dev/kfd`` access, ``amd-smi`` / ``rocm-smi``, HIP in PyTorch and the gfx
arch of every GPU, RCCL, hipBLASLt, the xGMI peer topology and the gfx950 native library.
"""
from __future__ import annotations

import ctypes.util
import glob
import os
import platform
import shutil
import subprocess
import threading
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, Optional

from . import presets as P
from .hardware import check_driver as _basic_check, gpus, rocm_version
from .schemas import DriverCheckResponse

DRIVER_YAMLS = Path(__file__).resolve().parent / "envs" / "drivers"   # <driver>.yaml (micromamba install -f)


def _cmd(args, timeout=20) -> Optional[str]:
    exe = shutil.which(args[0])
    if exe is None:
        return None
    try:
        r = subprocess.run([exe, *args[1:]], capture_output=True, text=True, timeout=timeout)
        return r.stdout if r.returncode == 0 else None
    except (OSError, subprocess.TimeoutExpired):
        return None


def _lib(name: str) -> Optional[str]:
    found = ctypes.util.find_library(name)
    if found:
        return found
    hits = glob.glob(f"/opt/rocm*/lib/lib{name}.so*")
    return hits[0] if hits else None


class DriverChecker:
    """One probe per driver name (``check(name) -> DriverCheckResponse``)."""

    @staticmethod
    def check(name: str) -> DriverCheckResponse:
        fn = getattr(DriverChecker, f"_p_{name}", None)
        if fn is None:
            return _basic_check(name)
        return fn()

    # ---- MI355X / ROCm
    @staticmethod
    def _p_rocm() -> DriverCheckResponse:
        v = rocm_version()
        if not v:
            return DriverCheckResponse(name="rocm", status="missing", details="/opt/rocm not found")
        return DriverCheckResponse(name="rocm", status="available", details=f"ROCm {v}")

    @staticmethod
    def _p_amdgpu_kernel() -> DriverCheckResponse:
        ver = None
        try:
            ver = Path("/sys/module/amdgpu/version").read_text().strip()
        except OSError:
            pass
        kfd = os.path.exists("/dev/kfd")
        ok = kfd and os.access("/dev/kfd", os.R_OK | os.W_OK)
        if not kfd:
            return DriverCheckResponse(name="amdgpu_kernel", status="missing", details="/dev/kfd absent (amdgpu KFD)")
        if not ok:
            return DriverCheckResponse(name="amdgpu_kernel", status="incompatible",
                                       details="/dev/kfd not accessible: add the user to the render/video groups")
        return DriverCheckResponse(name="amdgpu_kernel", status="available", details=f"amdgpu {ver or 'loaded'}")

    @staticmethod
    def _p_amd_smi() -> DriverCheckResponse:
        for tool in (["amd-smi", "version"], ["rocm-smi", "--showdriverversion"]):
            out = _cmd(tool)
            if out is not None:
                return DriverCheckResponse(name="amd_smi", status="available",
                                           details=f"{tool[0]}: {out.strip().splitlines()[-1][:120] if out.strip() else 'ok'}")
        return DriverCheckResponse(name="amd_smi", status="missing", details="neither amd-smi nor rocm-smi on PATH")

    @staticmethod
    def _p_hip_runtime() -> DriverCheckResponse:
        return _basic_check("hip_runtime")

    @staticmethod
    def _p_rccl() -> DriverCheckResponse:
        lib = _lib("rccl")
        try:
            import torch.distributed as dist

            nccl = dist.is_nccl_available()
        except Exception:  # noqa: BLE001
            nccl = False
        if lib and nccl:
            return DriverCheckResponse(name="rccl", status="available", details=f"{lib}; torch.distributed nccl backend")
        return DriverCheckResponse(name="rccl", status="missing",
                                   details=f"librccl {'found' if lib else 'missing'}; nccl backend {'on' if nccl else 'off'}")

    @staticmethod
    def _p_hipblaslt() -> DriverCheckResponse:
        lib = _lib("hipblaslt")
        return DriverCheckResponse(name="hipblaslt", status="available" if lib else "missing",
                                   details=lib or "libhipblaslt not found (only the torch reference path uses it)")

    @staticmethod
    def _p_xgmi() -> DriverCheckResponse:
        out = _cmd(["rocm-smi", "--showtopotype"]) or _cmd(["amd-smi", "topology"])
        g = gpus()
        if out is None:
            return DriverCheckResponse(name="xgmi", status="available" if len(g) <= 1 else "missing",
                                       details=f"{len(g)} GPU(s); topology tool unavailable")
        links = out.count("XGMI")
        return DriverCheckResponse(name="xgmi", status="available",
                                   details=f"{len(g)} GPU(s), {links} xGMI peer entries")

    @staticmethod
    def _p_gfx950() -> DriverCheckResponse:
        g = gpus()
        if not g:
            return DriverCheckResponse(name="gfx950", status="missing", details="no GPU visible")
        archs = sorted({x["arch"].split(":")[0] for x in g})
        ok = all(a == "gfx950" for a in archs)
        return DriverCheckResponse(name="gfx950", status="available" if ok else "incompatible",
                                   details=f"{len(g)} x {archs} ({sum(x['memory_gb'] for x in g):.0f} GB HBM)")

    @staticmethod
    def _p_lumen_native() -> DriverCheckResponse:
        return _basic_check("lumen_native")

    # ---- accelerators of the reference presets (not present on an MI355X build)
    @staticmethod
    def _p_cuda() -> DriverCheckResponse:
        out = _cmd(["nvidia-smi", "--query-gpu=name,driver_version", "--format=csv,noheader"])
        if out:
            return DriverCheckResponse(name="cuda", status="available", details=out.strip().splitlines()[0])
        return DriverCheckResponse(name="cuda", status="missing", details="nvidia-smi not found")

    @staticmethod
    def _p_tensorrt() -> DriverCheckResponse:
        lib = _lib("nvinfer")
        return DriverCheckResponse(name="tensorrt", status="available" if lib else "missing", details=lib or "libnvinfer not found")

    @staticmethod
    def _p_openvino() -> DriverCheckResponse:
        try:
            import openvino  # noqa: F401

            return DriverCheckResponse(name="openvino", status="available", details="openvino importable")
        except Exception:  # noqa: BLE001
            return DriverCheckResponse(name="openvino", status="missing", details="openvino not installed")

    @staticmethod
    def _p_directml() -> DriverCheckResponse:
        ok = platform.system() == "Windows"
        return DriverCheckResponse(name="directml", status="available" if ok else "missing",
                                   details="Windows only" if not ok else "Windows")

    @staticmethod
    def _p_coreml() -> DriverCheckResponse:
        ok = platform.system() == "Darwin"
        return DriverCheckResponse(name="coreml", status="available" if ok else "missing", details="macOS only")

    @staticmethod
    def _p_amd_npu() -> DriverCheckResponse:
        ok = os.path.exists("/dev/accel/accel0") or bool(glob.glob("/sys/class/accel/accel*"))
        return DriverCheckResponse(name="amd_npu", status="available" if ok else "missing",
                                   details="Ryzen AI NPU (amdxdna)" if ok else "no amdxdna accel device")

    @staticmethod
    def _p_rknn() -> DriverCheckResponse:
        ok = os.path.exists("/dev/rknpu") or bool(glob.glob("/sys/class/misc/rknpu*"))
        return DriverCheckResponse(name="rknn", status="available" if ok else "missing",
                                   details="Rockchip NPU" if ok else "no rknpu device")


MI355X_DRIVERS = ("rocm", "amdgpu_kernel", "amd_smi", "hip_runtime", "gfx950", "rccl", "xgmi", "lumen_native")


@dataclass
class EnvironmentReport:
    preset: str
    ready: bool
    drivers: list = field(default_factory=list)
    missing_installable: list = field(default_factory=list)


class EnvironmentChecker:
    @staticmethod
    def check_drivers(names) -> list[DriverCheckResponse]:
        return [DriverChecker.check(n) for n in names]

    @staticmethod
    def check_preset(preset: str) -> EnvironmentReport:
        p = P.get_preset(preset)
        if p is None:
            raise ValueError(f"unknown preset '{preset}'")
        names = list(p.create_config().drivers)
        if preset == "amd_mi355x":
            names = list(dict.fromkeys(names + list(MI355X_DRIVERS)))
        res = EnvironmentChecker.check_drivers(names)
        missing = [d.name for d in res if d.status != "available"]
        installable = [n for n in missing if (DRIVER_YAMLS / f"{n}.yaml").exists() or n == "lumen_native"]
        return EnvironmentReport(preset, not missing, res, installable)


class DependencyInstaller:
    """Install a missing driver: ``micromamba install -f envs/<driver>.yaml`` into the target
    environment (reference), or the in-tree gfx950 build for ``lumen_native``."""

    def __init__(self, env=None):
        self.env = env

    def install(self, driver: str, log: Optional[Callable[[str], None]] = None,
                cancel: Optional[threading.Event] = None) -> str:
        if driver == "lumen_native":
            import sys

            from .installation._proc import run

            root = Path(__file__).resolve().parents[2]
            py = str(self.env.python) if self.env is not None and self.env.exists() else sys.executable
            rc, tail = run([py, "-m", "lumen_amd._build"], log, cancel, cwd=str(root))
            if rc != 0:
                raise RuntimeError(f"native build failed (exit {rc}): {' | '.join(tail[-3:])}")
            return "built gfx950 native libraries"
        yml = DRIVER_YAMLS / f"{driver}.yaml"
        if not yml.exists():
            raise RuntimeError(f"driver '{driver}' is not installable from this control plane "
                               f"(system component: install it with the OS / ROCm installer)")
        if self.env is None:
            raise RuntimeError("driver yaml installs need a micromamba environment")
        rc, tail = self.env.install_file(str(yml), log, cancel)
        if rc != 0:
            raise RuntimeError(f"driver install failed (exit {rc}): {' | '.join(tail[-3:])}")
        return f"installed {driver}"
