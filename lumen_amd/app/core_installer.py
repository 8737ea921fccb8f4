"""CoreInstaller (reference lumen-app/src/lumen_app/services/installer.py:32-299): the
installation actions the orchestrator sequences — micromamba, environment, drivers, Lumen
package, native gfx950 build, verification, config save — over the utilities in
:mod:`lumen_amd.app.installation`."""
from __future__ import annotations

import sys
import threading
from pathlib import Path
from typing import Callable, Optional

import yaml

from .env_checker import DependencyInstaller, EnvironmentChecker
from .installation import (EnvSpec, InstallationVerifier, LumenPackageInstaller, LumenPackageResolver,
                           MicromambaInstaller, MicromambaStatus, PythonEnvManager, VerifyReport)
from .installation._proc import run

LogFn = Optional[Callable[[str], None]]


class CoreInstaller:
    def __init__(self, cache_dir: str, env_kind: str = "current", env_name: str = "lumen_env",
                 region: str = "other"):
        self.cache_dir = Path(cache_dir).expanduser()
        self.env_kind = env_kind
        self.mamba = MicromambaInstaller(self.cache_dir, region=region)
        self.env: Optional[PythonEnvManager] = None
        if env_kind != "current":
            self.env = PythonEnvManager(self.cache_dir, EnvSpec(env_name, env_kind))
        self.resolver = LumenPackageResolver(self.cache_dir, region)

    # ---- steps
    def micromamba_ready(self) -> bool:
        return self.mamba.check().status == MicromambaStatus.INSTALLED

    def install_micromamba(self, log: LogFn = None, cancel: Optional[threading.Event] = None, force=False) -> str:
        r = self.mamba.install(log, cancel, force=force)
        if r.status != MicromambaStatus.INSTALLED:
            raise RuntimeError(f"micromamba install failed: {r.message}")
        if self.env is not None:
            self.env.micromamba = r.path
        return f"micromamba {r.version} ({r.path})"

    def check_micromamba(self) -> str:
        r = self.mamba.check()
        if r.status != MicromambaStatus.INSTALLED:
            raise RuntimeError(f"micromamba {r.status.value}: {r.message}")
        if self.env is not None:
            self.env.micromamba = r.path
        return f"micromamba {r.version}"

    def create_environment(self, log: LogFn = None, cancel=None, force=False) -> str:
        if self.env is None:
            return f"using the current interpreter ({sys.executable})"
        self.env.create(log, cancel, force=force)
        return f"environment ready at {self.env.prefix}"

    def missing_drivers(self, preset: str) -> list[str]:
        rep = EnvironmentChecker.check_preset(preset)
        return [d.name for d in rep.drivers if d.status != "available"]

    def install_drivers(self, drivers, log: LogFn = None, cancel=None) -> str:
        inst = DependencyInstaller(self.env)
        return "; ".join(inst.install(d, log, cancel) for d in drivers) or "nothing to install"

    def install_packages(self, preset: str, wheel: Optional[str] = None, log: LogFn = None, cancel=None) -> str:
        src = self.resolver.resolve(preset, wheel, allow_network=False)
        if log:
            log(f"lumen_amd source: {src.kind} {src.location}")
        return LumenPackageInstaller(self.resolver).install(src, self.env, log, cancel, offline=True)

    def build_native(self, log: LogFn = None, cancel=None, force=False) -> str:
        from .._native import HIP_SO, HOST_SO

        if HIP_SO.exists() and HOST_SO.exists() and not force:
            return "native libraries already built"
        root = Path(__file__).resolve().parents[2]
        py = str(self.env.python) if self.env is not None and self.env.exists() else sys.executable
        rc, tail = run([py, "-m", "lumen_amd._build"], log, cancel, cwd=str(root))
        if rc != 0:
            raise RuntimeError(f"native build failed (exit {rc}): {' | '.join(tail[-3:])}")
        return "built _lumen_hip.so (gfx950) and _lumen_host.so"

    def verify(self, log: LogFn = None, cancel=None) -> VerifyReport:
        return InstallationVerifier().verify(self.env, log, cancel)

    def prepare_cache(self) -> str:
        (self.cache_dir / "models").mkdir(parents=True, exist_ok=True)
        return f"cache ready at {self.cache_dir}"

    def save_config(self, config: dict, name: str = "lumen-config.yaml") -> Path:
        p = self.cache_dir / name
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(yaml.safe_dump(config, sort_keys=False))
        return p

    def python_for_server(self) -> str:
        """Interpreter the ServerManager should launch the hub with."""
        return str(self.env.python) if self.env is not None and self.env.exists() else sys.executable
