"""Control-plane installation stack (reference lumen-app install_orchestrator.py,
installer.py, utils/env_checker.py, utils/installation/*, utils/package_resolver.py):
step planning, cancellation with cache cleanup, micromamba install from a mirror, venv
environments, package resolution and the in-environment verifier."""
import os
import threading
import time
from pathlib import Path

import pytest

from lumen_amd.app.core_installer import CoreInstaller
from lumen_amd.app.env_checker import MI355X_DRIVERS, DependencyInstaller, EnvironmentChecker
from lumen_amd.app.install import InstallOrchestrator, clear_cache_dir, plan_steps
from lumen_amd.app.installation import (EnvSpec, InstallationVerifier, LumenPackageResolver, MicromambaInstaller,
                                        MicromambaStatus, PythonEnvManager)
from lumen_amd.app.schemas import InstallSetupRequest


def _wait(orch, tid, timeout=60):
    t0 = time.time()
    while time.time() - t0 < timeout:
        s = orch.get(tid).snapshot()
        if s.status in ("completed", "failed", "cancelled"):
            return s
        time.sleep(0.02)
    raise AssertionError("task did not finish")


def test_plan_steps(tmp_path):
    req = InstallSetupRequest(preset="cpu", cache_dir=str(tmp_path))
    ids = [s for s, _ in plan_steps(req, CoreInstaller(str(tmp_path)))]
    assert ids == ["check_python", "build_native", "verify_installation", "prepare_cache"]
    req = InstallSetupRequest(preset="cpu", cache_dir=str(tmp_path), env_kind="venv")
    ids = [s for s, _ in plan_steps(req, CoreInstaller(str(tmp_path), "venv"))]
    assert ids == ["check_python", "create_environment", "install_packages", "build_native", "verify_installation",
                   "prepare_cache"]
    req = InstallSetupRequest(preset="cpu", cache_dir=str(tmp_path), env_kind="micromamba")
    ids = [s for s, _ in plan_steps(req, CoreInstaller(str(tmp_path), "micromamba"))]
    assert ids[0] in ("install_micromamba", "check_micromamba") and "create_environment" in ids


def test_cancel_clears_cache(tmp_path, monkeypatch):
    cache = tmp_path / "cache"
    (cache / "models" / "m").mkdir(parents=True)
    (cache / "models" / "m" / "w.bin").write_bytes(b"x" * 10)
    started = threading.Event()

    def slow(self, t, i):
        started.set()
        while not t.cancel.is_set():
            time.sleep(0.01)
        from lumen_amd.app.installation._proc import Cancelled
        raise Cancelled()

    monkeypatch.setattr(InstallOrchestrator, "_do_check_python", slow)
    orch = InstallOrchestrator()
    r = orch.create(InstallSetupRequest(preset="cpu", cache_dir=str(cache)))
    assert started.wait(10)
    snap = orch.cancel(r.task_id)
    assert snap.status == "cancelled" and snap.progress == 0
    assert [s.status for s in snap.steps] == ["cancelled"] * len(snap.steps)
    assert snap.steps[0].message == "Cancelled by user"
    assert cache.is_dir() and list(cache.iterdir()) == []
    assert "cache directory cleared" in snap.current_step


def test_clear_cache_refuses_unsafe(tmp_path):
    assert "Refusing" in clear_cache_dir("/")
    assert "Refusing" in clear_cache_dir(str(Path.home()))
    (tmp_path / "a").mkdir()
    (tmp_path / "b.txt").write_text("x")
    os.symlink(tmp_path / "b.txt", tmp_path / "l")
    assert clear_cache_dir(tmp_path) is None and list(tmp_path.iterdir()) == []


def test_micromamba_install_from_mirror(tmp_path, monkeypatch):
    """The release asset is the bare executable; the installer tries mirrors in order and only
    installs a download whose SHA-256 matches the ``.sha256`` sidecar next to it."""
    import hashlib

    monkeypatch.delenv("MAMBA_EXE", raising=False)
    monkeypatch.setenv("PATH", "/usr/bin:/bin")
    exe = tmp_path / "micromamba-linux-64"
    exe.write_bytes(b"#!/bin/sh\necho 2.0.5\n")
    (tmp_path / "micromamba-linux-64.sha256").write_text(
        f"{hashlib.sha256(exe.read_bytes()).hexdigest()}  micromamba-linux-64\n")
    inst = MicromambaInstaller(tmp_path / "cache", mirrors=("file:///nonexistent/{plat}", f"file://{exe}"))
    assert inst.check().status == MicromambaStatus.NOT_INSTALLED
    logs = []
    r = inst.install(logs.append)
    assert r.status == MicromambaStatus.INSTALLED and r.version == "2.0.5", (r, logs)
    assert Path(r.path) == inst.local_path and any("failed" in x for x in logs)


def test_resolver(tmp_path):
    res = LumenPackageResolver(tmp_path)
    src = res.resolve("amd_mi355x")
    assert src.kind == "source" and Path(src.location, "pyproject.toml").exists() and src.extras == ["rocm"]
    assert res.pip_args(src)[:4] == ["install", "--no-build-isolation", "--no-deps", "--no-index"]
    whl = tmp_path / "wheels" / "lumen_amd-0.2.0-py3-none-any.whl"
    whl.parent.mkdir()
    whl.write_bytes(b"")
    w = res.resolve("cpu")
    assert w.kind == "wheel" and w.version == "0.2.0" and w.pip_target().endswith(".whl[cpu]")
    with pytest.raises(FileNotFoundError):
        res.resolve("cpu", explicit=str(tmp_path / "nope.whl"))


def test_env_checker_mi355x_probes():
    rep = EnvironmentChecker.check_preset("amd_mi355x")
    names = [d.name for d in rep.drivers]
    assert set(MI355X_DRIVERS) <= set(names)
    assert all(d.status in ("available", "missing", "incompatible") and d.details is not None for d in rep.drivers)
    with pytest.raises(RuntimeError, match="system component"):
        DependencyInstaller().install("rocm")
    with pytest.raises(ValueError):
        EnvironmentChecker.check_preset("nope")


def test_verifier_current_interpreter():
    rep = InstallationVerifier().verify(None, timeout=300)
    assert rep.details.get("torch") and "native" in rep.details
    assert rep.ok == (rep.details["native"]["hip_so"] and rep.details["native"]["host_so"])


@pytest.mark.timeout(600)
def test_venv_environment_install_and_verify(tmp_path):
    """A real isolated environment: venv over the host's PyTorch, lumen_amd installed into it
    from this source tree (offline), verified by the probe running inside it."""
    core = CoreInstaller(str(tmp_path), "venv", "lumen_env")
    assert "environment ready" in core.create_environment()
    env = core.env
    assert env.exists() and env.prefix == tmp_path / "envs" / "lumen_env"
    logs = []
    msg = core.install_packages("cpu", log=logs.append)
    assert msg.startswith("installed source"), logs[-5:]
    rep = core.verify()
    assert rep.details.get("torch"), rep
    rc, tail = env.run_python(["-c", "import lumen_amd, sys; print(lumen_amd.__file__)"])
    assert rc == 0 and str(env.prefix) in tail[-1], tail
    assert core.python_for_server() == str(env.python)
