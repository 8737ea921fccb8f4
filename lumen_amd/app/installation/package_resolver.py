"""Where the ``lumen_amd`` package comes from (reference utils/package_resolver.py: GitHub
latest-release wheel lookup for EdwinZhanCN/Lumen, CN mirrors, pip args with extras).

Resolution order:
1. an explicit wheel / directory (``LUMEN_WHEEL`` or the request);
2. a wheel already in ``<cache_dir>/wheels``;
3. this source tree (``pip install <repo root>`` — the gfx950 libraries are built in-tree
   by the native build step, so the tree installs as-is);
4. the latest GitHub release asset (``LUMEN_RELEASE_REPO``); region ``cn`` also tries the
   gh-proxy.org mirror.  A downloaded wheel must match the SHA-256 the release publishes
   (the asset's ``digest`` field, or a ``<wheel>.sha256`` asset) or it is deleted.
"""
from __future__ import annotations

import hashlib
import json
import os
import urllib.request
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional

GITHUB_API = "https://api.github.com/repos/{repo}/releases/latest"
DOWNLOAD_MIRRORS = ("{url}", "https://gh-proxy.org/{url}")     # the proxy only for region == cn
PYPI_MIRRORS = {"cn": "https://mirrors.aliyun.com/pypi/simple/", "other": None}
# preset -> pip extras of the lumen_amd package (reference: cpu/cuda/apple/openvino/rknn/torch)
PRESET_EXTRAS = {"amd_mi355x": ["rocm"], "cpu": ["cpu"]}


@dataclass
class PackageSource:
    kind: str                       # "wheel" | "source" | "release"
    location: str                   # path or URL
    version: Optional[str] = None
    extras: list = field(default_factory=list)
    sha256: Optional[str] = None    # published digest of a release asset

    def pip_target(self) -> str:
        ex = f"[{','.join(self.extras)}]" if self.extras else ""
        return f"{self.location}{ex}"


class LumenPackageResolver:
    def __init__(self, cache_dir, region: str = "other", repo: Optional[str] = None, timeout: float = 20.0):
        self.cache_dir = Path(os.path.expanduser(str(cache_dir)))
        self.region = region
        self.repo = repo or os.environ.get("LUMEN_RELEASE_REPO", "")
        self.timeout = timeout

    @staticmethod
    def source_tree() -> Optional[Path]:
        root = Path(__file__).resolve().parents[3]
        return root if (root / "pyproject.toml").exists() and (root / "lumen_amd").is_dir() else None

    def resolve(self, preset: str, explicit: Optional[str] = None, allow_network: bool = True) -> PackageSource:
        extras = PRESET_EXTRAS.get(preset, [])
        cand = explicit or os.environ.get("LUMEN_WHEEL")
        if cand:
            p = Path(os.path.expanduser(cand))
            if p.is_file() and p.suffix == ".whl":
                return PackageSource("wheel", str(p), _wheel_version(p), extras)
            if p.is_dir() and (p / "pyproject.toml").exists():
                return PackageSource("source", str(p), None, extras)
            raise FileNotFoundError(f"package source not found: {cand}")
        wheels = sorted((self.cache_dir / "wheels").glob("lumen_amd-*.whl"))
        if wheels:
            return PackageSource("wheel", str(wheels[-1]), _wheel_version(wheels[-1]), extras)
        tree = self.source_tree()
        if tree is not None:
            return PackageSource("source", str(tree), None, extras)
        if allow_network and self.repo:
            return self._from_release(extras)
        raise RuntimeError("no lumen_amd package source: no wheel, no source tree, no release repository")

    def _from_release(self, extras) -> PackageSource:
        req = urllib.request.Request(GITHUB_API.format(repo=self.repo), headers={"Accept": "application/vnd.github+json"})
        with urllib.request.urlopen(req, timeout=self.timeout) as r:
            rel = json.load(r)
        assets = rel.get("assets", [])
        for a in assets:
            name = a.get("name", "")
            if name.startswith("lumen_amd-") and name.endswith(".whl"):
                return PackageSource("release", a["browser_download_url"], rel.get("tag_name"), extras,
                                     sha256=self._asset_digest(a, assets))
        raise RuntimeError(f"release {rel.get('tag_name')} of {self.repo} has no lumen_amd wheel")

    def _asset_digest(self, asset: dict, assets: list) -> Optional[str]:
        d = asset.get("digest") or ""
        if d.startswith("sha256:"):
            return d.split(":", 1)[1].lower()
        side = next((a for a in assets if a.get("name") == asset.get("name", "") + ".sha256"), None)
        if side is None:
            return None
        from .micromamba import parse_sha256

        with urllib.request.urlopen(side["browser_download_url"], timeout=self.timeout) as r:
            return parse_sha256(r.read(4096).decode("utf-8", "replace"))

    def download(self, src: PackageSource) -> PackageSource:
        """Fetch a release asset into <cache>/wheels (mirror list)."""
        if src.kind != "release":
            return src
        dst = self.cache_dir / "wheels" / src.location.rsplit("/", 1)[-1]
        dst.parent.mkdir(parents=True, exist_ok=True)
        errs = []
        mirrors = DOWNLOAD_MIRRORS if self.region == "cn" else DOWNLOAD_MIRRORS[:1]
        if not src.sha256:
            raise RuntimeError(f"{src.location}: the release publishes no SHA-256 digest; refusing to install it")
        for m in mirrors:
            try:
                h = hashlib.sha256()
                with urllib.request.urlopen(m.format(url=src.location), timeout=self.timeout) as r, open(dst, "wb") as f:
                    for chunk in iter(lambda: r.read(1 << 20), b""):
                        h.update(chunk)
                        f.write(chunk)
                if h.hexdigest() != src.sha256:
                    dst.unlink(missing_ok=True)
                    raise RuntimeError(f"SHA-256 mismatch: got {h.hexdigest()}, expected {src.sha256}")
                return PackageSource("wheel", str(dst), src.version, src.extras)
            except Exception as e:  # noqa: BLE001
                errs.append(str(e))
        raise RuntimeError(f"download failed: {'; '.join(errs)}")

    def pip_args(self, src: PackageSource, offline: bool = True) -> list[str]:
        """pip install arguments: no dependency resolution against an index when offline (the
        environment's packages come from the env yaml / the host)."""
        args = ["install", "--no-build-isolation"]
        if offline:
            args += ["--no-deps", "--no-index"]
        elif PYPI_MIRRORS.get(self.region):
            args += ["-i", PYPI_MIRRORS[self.region]]
        return args + [src.pip_target()]


def _wheel_version(p: Path) -> Optional[str]:
    parts = p.name.split("-")
    return parts[1] if len(parts) > 2 else None
