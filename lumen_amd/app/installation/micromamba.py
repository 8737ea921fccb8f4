"""micromamba locate / install / check (reference utils/installation/micromamba_installer.py).

Search order: ``$MAMBA_EXE``, ``<cache_dir>/bin/micromamba``, ``micromamba`` on PATH.
Install downloads the static binary for this platform from the mirror list (official
micro.mamba.pm API, then the GitHub release through CN-friendly proxies) into
``<cache_dir>/bin`` and verifies it with ``micromamba --version``.
"""
from __future__ import annotations

import os
import platform
import shutil
import stat
import subprocess
import tarfile
import tempfile
import threading
import urllib.request
from dataclasses import dataclass
from enum import Enum
from pathlib import Path
from typing import Callable, Optional

from ._proc import Cancelled

MIRRORS = (
    "https://micro.mamba.pm/api/micromamba/{plat}/latest",
    "https://github.com/mamba-org/micromamba-releases/releases/latest/download/micromamba-{plat}",
    "https://gh-proxy.com/https://github.com/mamba-org/micromamba-releases/releases/latest/download/micromamba-{plat}",
)


class MicromambaStatus(Enum):
    INSTALLED = "installed"
    NOT_INSTALLED = "not_installed"
    BROKEN = "broken"


@dataclass
class MicromambaResult:
    status: MicromambaStatus
    path: Optional[str] = None
    version: Optional[str] = None
    message: str = ""


def platform_tag() -> str:
    sysname, mach = platform.system().lower(), platform.machine().lower()
    arch = {"x86_64": "64", "amd64": "64", "aarch64": "aarch64", "arm64": "arm64", "ppc64le": "ppc64le"}.get(mach, mach)
    if sysname == "darwin":
        return f"osx-{'arm64' if arch in ('arm64', 'aarch64') else '64'}"
    if sysname == "windows":
        return "win-64"
    return f"linux-{arch}"


class MicromambaInstaller:
    def __init__(self, cache_dir, mirrors=MIRRORS, timeout: float = 60.0):
        self.cache_dir = Path(os.path.expanduser(str(cache_dir)))
        self.mirrors = tuple(mirrors)
        self.timeout = timeout

    @property
    def local_path(self) -> Path:
        return self.cache_dir / "bin" / ("micromamba.exe" if platform.system() == "Windows" else "micromamba")

    def find(self) -> Optional[str]:
        for cand in (os.environ.get("MAMBA_EXE"), str(self.local_path), shutil.which("micromamba")):
            if cand and Path(cand).is_file() and os.access(cand, os.X_OK):
                return cand
        return None

    def check(self) -> MicromambaResult:
        exe = self.find()
        if exe is None:
            return MicromambaResult(MicromambaStatus.NOT_INSTALLED, message="micromamba not found")
        try:
            out = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=30)
        except (OSError, subprocess.TimeoutExpired) as e:
            return MicromambaResult(MicromambaStatus.BROKEN, exe, message=str(e))
        if out.returncode != 0:
            return MicromambaResult(MicromambaStatus.BROKEN, exe, message=out.stderr.strip()[:200])
        return MicromambaResult(MicromambaStatus.INSTALLED, exe, out.stdout.strip(), "ok")

    def install(self, log: Optional[Callable[[str], None]] = None, cancel: Optional[threading.Event] = None,
                force: bool = False) -> MicromambaResult:
        if not force:
            r = self.check()
            if r.status == MicromambaStatus.INSTALLED:
                return r
        plat = platform_tag()
        self.local_path.parent.mkdir(parents=True, exist_ok=True)
        errors = []
        for m in self.mirrors:
            if cancel is not None and cancel.is_set():
                raise Cancelled()
            url = m.format(plat=plat)
            if log:
                log(f"downloading micromamba from {url}")
            try:
                self._fetch(url)
                r = self.check()
                if r.status == MicromambaStatus.INSTALLED:
                    if log:
                        log(f"micromamba {r.version} at {r.path}")
                    return r
                errors.append(f"{url}: {r.message}")
            except Exception as e:  # noqa: BLE001 - try the next mirror
                errors.append(f"{url}: {e}")
                if log:
                    log(f"  failed: {e}")
        return MicromambaResult(MicromambaStatus.NOT_INSTALLED, message="; ".join(errors) or "no mirrors")

    def _fetch(self, url: str) -> None:
        with tempfile.TemporaryDirectory() as td:
            tmp = Path(td) / "dl"
            with urllib.request.urlopen(url, timeout=self.timeout) as resp, open(tmp, "wb") as f:
                shutil.copyfileobj(resp, f)
            if tarfile.is_tarfile(tmp):   # micro.mamba.pm serves a .tar.bz2 with bin/micromamba
                with tarfile.open(tmp) as tf:
                    member = next((mm for mm in tf.getmembers() if mm.name.endswith("bin/micromamba")), None)
                    if member is None or not member.isfile():
                        raise RuntimeError("archive without bin/micromamba")
                    src = tf.extractfile(member)
                    with open(self.local_path, "wb") as out:
                        shutil.copyfileobj(src, out)
            else:
                shutil.copyfile(tmp, self.local_path)
        self.local_path.chmod(self.local_path.stat().st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
