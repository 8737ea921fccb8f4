"""Post-install verification run INSIDE the target environment (reference
utils/installation/verifier.py: import check via ``micromamba run``).  The probe prints one
JSON line: package import, PyTorch HIP version, GPUs and their gfx arch, native library
status (gfx950 kernels + host runtime), grpc/protobuf versions."""
from __future__ import annotations

import json
import sys
import threading
from dataclasses import dataclass, field
from typing import Callable, Optional

from ._proc import run
from .env_manager import PythonEnvManager

PROBE = r"""
import json, importlib
out = {"ok": True, "errors": []}
def tryimp(m):
    try:
        return importlib.import_module(m)
    except Exception as e:
        out["errors"].append(f"{m}: {e}"); out["ok"] = False
lm = tryimp("lumen_amd")
torch = tryimp("torch")
grpc = tryimp("grpc")
if torch is not None:
    out["torch"] = torch.__version__
    out["hip"] = getattr(torch.version, "hip", None)
    try:
        n = torch.cuda.device_count()
        out["gpus"] = [getattr(torch.cuda.get_device_properties(i), "gcnArchName", "") for i in range(n)]
    except Exception as e:
        out["gpus"] = []
if lm is not None:
    try:
        from lumen_amd._native import HIP_SO, HOST_SO
        out["native"] = {"hip_so": HIP_SO.exists(), "host_so": HOST_SO.exists()}
        if not (HIP_SO.exists() and HOST_SO.exists()):
            out["errors"].append("native libraries not built"); out["ok"] = False
    except Exception as e:
        out["errors"].append(f"native: {e}"); out["ok"] = False
if grpc is not None:
    out["grpc"] = grpc.__version__
print("LUMEN_VERIFY " + json.dumps(out))
"""


@dataclass
class VerifyReport:
    ok: bool
    details: dict = field(default_factory=dict)
    errors: list = field(default_factory=list)


class InstallationVerifier:
    def verify(self, env: Optional[PythonEnvManager], log: Optional[Callable[[str], None]] = None,
               cancel: Optional[threading.Event] = None, timeout: float = 300.0) -> VerifyReport:
        lines: list[str] = []

        def cap(s: str) -> None:
            lines.append(s)
            if log and not s.startswith("LUMEN_VERIFY "):
                log(s)

        if env is None:
            rc, _ = run([sys.executable, "-c", PROBE], cap, cancel, timeout=timeout)
        else:
            rc, _ = env.run_python(["-c", PROBE], cap, cancel, timeout=timeout)
        rep = next((ln for ln in reversed(lines) if ln.startswith("LUMEN_VERIFY ")), None)
        if rep is None:
            return VerifyReport(False, {}, [f"probe failed (exit {rc})"] + lines[-3:])
        d = json.loads(rep[len("LUMEN_VERIFY "):])
        return VerifyReport(bool(d.get("ok")) and rc == 0, d, list(d.get("errors", [])))
