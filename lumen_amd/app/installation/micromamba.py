"""micromamba locate / install / check (reference utils/installation/micromamba_installer.py).

Search order: ``$MAMBA_EXE``, ``<cache_dir>/bin/micromamba``, ``micromamba`` on PATH.
Install downloads the static binary for this platform from the mamba-org GitHub release
(region ``cn`` also tries the gh-proxy.org mirror, as the reference does), verifies it against
the SHA-256 digest the release publishes next to it (``micromamba-<plat>.sha256``, fetched
from the same host) BEFORE it is made executable, then checks ``micromamba --version``.  A
binary whose digest is missing or differs is deleted and never run.
"""
from __future__ import annotations

import hashlib
import os
import platform
import shutil
import stat
import subprocess
import tempfile
import threading
import urllib.request
from dataclasses import dataclass
from enum import Enum
from pathlib import Path
from typing import Callable, Optional

from ._proc import Cancelled

RELEASE = "https://github.com/mamba-org/micromamba-releases/releases/latest/download/micromamba-{plat}"
CN_PROXY = "https://gh-proxy.org/"          # reference micromamba_installer.py: region == cn only


def mirrors_for(region: str = "other") -> tuple:
    return (RELEASE, CN_PROXY + RELEASE) if region == "cn" else (RELEASE,)


MIRRORS = mirrors_for("other")


def sha256_file(path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def parse_sha256(text: str) -> Optional[str]:
    """The first 64-hex-digit token of a ``.sha256`` sidecar (``<digest>  <name>`` or bare)."""
    for tok in text.replace("*", " ").split():
        t = tok.strip().lower()
        if len(t) == 64 and all(c in "0123456789abcdef" for c in t):
            return t
    return None


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
    def __init__(self, cache_dir, mirrors=None, timeout: float = 60.0, region: str = "other",
                 sha256: Optional[str] = None):
        self.cache_dir = Path(os.path.expanduser(str(cache_dir)))
        self.mirrors = tuple(mirrors) if mirrors is not None else mirrors_for(region)
        self.timeout = timeout
        self.sha256 = sha256.lower() if sha256 else None   # pinned digest (else the release sidecar)

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
        """Download to a temp file, verify its SHA-256, then move it into place + chmod."""
        with tempfile.TemporaryDirectory() as td:
            tmp = Path(td) / "dl"
            with urllib.request.urlopen(url, timeout=self.timeout) as resp, open(tmp, "wb") as f:
                shutil.copyfileobj(resp, f)
            want = self.sha256
            if want is None:
                with urllib.request.urlopen(url + ".sha256", timeout=self.timeout) as resp:
                    want = parse_sha256(resp.read(4096).decode("utf-8", "replace"))
            if want is None:
                raise RuntimeError("no published SHA-256 for the micromamba binary; refusing to install it")
            got = sha256_file(tmp)
            if got != want:
                raise RuntimeError(f"micromamba SHA-256 mismatch: got {got}, expected {want}")
            shutil.copyfile(tmp, self.local_path)
        self.local_path.chmod(self.local_path.stat().st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
