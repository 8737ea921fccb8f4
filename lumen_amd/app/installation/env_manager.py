"""Isolated Python environments for a Lumen install (reference
utils/installation/env_manager.py: micromamba ``create -f <yaml>`` + ``run pip``).

Two kinds, same interface:

* ``micromamba`` — ``micromamba create -y -p <cache>/envs/<name> -f envs/rocm.yaml``;
* ``venv``       — ``python -m venv --system-site-packages <cache>/envs/<name>``: reuses the
  ROCm PyTorch / RCCL stack already installed on the host (the heavy part of an MI355X
  environment) and needs no network for the base environment.
"""
from __future__ import annotations

import os
import shutil
import sys
import threading
from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Optional, Sequence

from ._proc import run

ENV_YAML_DIR = Path(__file__).resolve().parents[1] / "envs"


@dataclass
class EnvSpec:
    name: str = "lumen_env"
    kind: str = "venv"                 # "venv" | "micromamba"
    yaml: Optional[str] = None         # micromamba: env file (default envs/rocm.yaml)


class PythonEnvManager:
    def __init__(self, cache_dir, spec: EnvSpec, micromamba: Optional[str] = None):
        self.cache_dir = Path(os.path.expanduser(str(cache_dir)))
        self.spec = spec
        self.micromamba = micromamba

    @property
    def prefix(self) -> Path:
        return self.cache_dir / "envs" / self.spec.name

    @property
    def python(self) -> Path:
        if os.name == "nt":
            return self.prefix / ("python.exe" if self.spec.kind == "micromamba" else "Scripts/python.exe")
        return self.prefix / "bin" / "python"

    def exists(self) -> bool:
        return self.python.exists()

    def create(self, log: Optional[Callable[[str], None]] = None, cancel: Optional[threading.Event] = None,
               force: bool = False) -> None:
        if self.exists() and not force:
            if log:
                log(f"environment exists: {self.prefix}")
            return
        if force and self.prefix.exists():
            shutil.rmtree(self.prefix)
        self.prefix.parent.mkdir(parents=True, exist_ok=True)
        if self.spec.kind == "micromamba":
            if not self.micromamba:
                raise RuntimeError("micromamba environment requested but no micromamba binary")
            yml = self.spec.yaml or str(ENV_YAML_DIR / "rocm.yaml")
            rc, tail = run([self.micromamba, "create", "-y", "-p", str(self.prefix), "-f", yml], log, cancel,
                           env=dict(os.environ, MAMBA_ROOT_PREFIX=str(self.cache_dir / "mamba")))
        else:
            # --without-pip: pip comes from the host site-packages (no ensurepip / network needed)
            rc, tail = run([sys.executable, "-m", "venv", "--system-site-packages", "--without-pip", str(self.prefix)],
                           log, cancel)
        if rc != 0 or not self.exists():
            raise RuntimeError(f"environment creation failed (exit {rc}): {' | '.join(tail[-3:])}")

    def run_python(self, args: Sequence[str], log=None, cancel=None, timeout: Optional[float] = None):
        # cwd = the env prefix: a source checkout in the caller's cwd must not shadow the
        # package installed in the environment
        return run([str(self.python), *args], log, cancel, timeout=timeout, env=self._env(), cwd=str(self.prefix))

    def run_pip(self, args: Sequence[str], log=None, cancel=None):
        return run([str(self.python), "-m", "pip", *args], log, cancel, env=self._env(), cwd=str(self.prefix))

    def install_file(self, yml: str, log=None, cancel=None):
        """micromamba install -f <driver yaml> into this env (reference DependencyInstaller)."""
        if self.spec.kind != "micromamba" or not self.micromamba:
            raise RuntimeError("driver yaml installs need a micromamba environment")
        return run([self.micromamba, "install", "-y", "-p", str(self.prefix), "-f", yml], log, cancel)

    def remove(self) -> None:
        if self.prefix.exists():
            shutil.rmtree(self.prefix)

    def _env(self) -> dict:
        env = dict(os.environ)
        env.pop("PYTHONHOME", None)
        env.pop("PYTHONPATH", None)
        env["VIRTUAL_ENV"] = str(self.prefix)
        env["PATH"] = str(self.python.parent) + os.pathsep + env.get("PATH", "")
        return env
