"""pip-install the resolved lumen_amd artefact into an environment (reference
utils/installation/package_installer.py).  The current interpreter counts as an
environment too (``env=None``): then nothing is installed if lumen_amd already imports
from the same tree."""
from __future__ import annotations

import importlib.util
import sys
import threading
from pathlib import Path
from typing import Callable, Optional

from ._proc import run
from .env_manager import PythonEnvManager
from .package_resolver import LumenPackageResolver, PackageSource


class LumenPackageInstaller:
    def __init__(self, resolver: LumenPackageResolver):
        self.resolver = resolver

    def install(self, src: PackageSource, env: Optional[PythonEnvManager], log: Optional[Callable[[str], None]] = None,
                cancel: Optional[threading.Event] = None, offline: bool = True) -> str:
        if env is None:
            spec = importlib.util.find_spec("lumen_amd")
            if spec is not None and src.kind == "source" and Path(spec.origin).resolve().is_relative_to(
                    Path(src.location).resolve()):
                msg = f"lumen_amd already importable from {Path(spec.origin).parent}"
                if log:
                    log(msg)
                return msg
            py = [sys.executable, "-m", "pip"]
            rc, tail = run([*py, *self.resolver.pip_args(src, offline)], log, cancel)
        else:
            rc, tail = env.run_pip(self.resolver.pip_args(src, offline), log, cancel)
        if rc != 0:
            raise RuntimeError(f"pip install failed (exit {rc}): {' | '.join(tail[-3:])}")
        return f"installed {src.kind} {src.location}"
