"""Loader for the in-tree native libraries.

``load_hip()`` registers ``torch.ops.lumen.*`` from ``_lumen_hip.so``.  On a GPU
host the library is mandatory: if it is missing or fails to load, every GPU op
raises instead of silently falling back to PyTorch (set LUMEN_AUTOBUILD=1 to
build it on first use).  On a CPU-only host the ops use the PyTorch reference
path in :mod:`lumen_amd.ops` and the library is optional.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

_PKG = Path(__file__).resolve().parent
HIP_SO = _PKG / "_lumen_hip.so"
HOST_SO = _PKG / "_lumen_host.so"

_lock = threading.Lock()
_hip_loaded = False
_hip_error: Exception | None = None
_host_lib = None


def _maybe_build() -> None:
    if os.environ.get("LUMEN_AUTOBUILD", "0") == "1":
        from ._build import build

        build()


def load_hip(required: bool = True) -> bool:
    """Load the HIP op library; raise if ``required`` and it cannot be loaded."""
    global _hip_loaded, _hip_error
    if _hip_loaded:
        return True
    with _lock:
        if _hip_loaded:
            return True
        try:
            if not HIP_SO.exists():
                _maybe_build()
            if not HIP_SO.exists():
                raise FileNotFoundError(
                    f"{HIP_SO} not built; run `python -m lumen_amd._build` (or __graft_entry__.build())")
            import torch

            torch.ops.load_library(str(HIP_SO))
            _hip_loaded = True
        except Exception as e:  # pragma: no cover - depends on host
            _hip_error = e
            if required:
                raise RuntimeError(f"lumen_amd native HIP library unavailable: {e}") from e
    return _hip_loaded


def hip_ops():
    """Return ``torch.ops.lumen`` after making sure the library is loaded."""
    load_hip(required=True)
    import torch

    return torch.ops.lumen


def load_host():
    """ctypes handle to the host-only C++ runtime library (or None if not built)."""
    global _host_lib
    if _host_lib is None and HOST_SO.exists():
        _host_lib = ctypes.CDLL(str(HOST_SO))
    return _host_lib


def native_status() -> dict:
    return {
        "hip_so": str(HIP_SO) if HIP_SO.exists() else None,
        "hip_loaded": _hip_loaded,
        "hip_error": repr(_hip_error) if _hip_error else None,
        "host_so": str(HOST_SO) if HOST_SO.exists() else None,
    }
