"""Install orchestration (reference lumen-app/src/lumen_app/services/install_orchestrator.py:33-819,
install_task_repository.py).

A setup task plans its steps from the current state (like the reference's
``_plan_installation_steps``), then runs them on a background thread with per-step
progress and logs (``/api/v1/install/tasks/{id}/logs``, ``/ws/install/{id}``):

  [install|check micromamba]  (env_kind = micromamba)
  check Python dependencies   (current interpreter)
  create environment          (venv / micromamba; skipped for the current interpreter)
  install drivers             (only when the preset reports installable missing drivers)
  install Lumen packages      (wheel / this source tree into the environment)
  build gfx950 native libs    (``python -m lumen_amd._build`` in the environment)
  verify installation         (probe script INSIDE the environment)
  prepare cache directory

Cancellation is cooperative: a running child process is terminated, remaining steps are
marked cancelled and — as in the reference (``_handle_cancellation`` / ``_clear_cache_dir``)
— the cache directory's contents are deleted, refusing ``/`` and the home directory.
"""
from __future__ import annotations

import importlib
import shutil
import sys
import threading
import time
import uuid
from pathlib import Path
from typing import Optional

from . import presets as P
from .core_installer import CoreInstaller
from .installation._proc import Cancelled
from .schemas import InstallSetupRequest, InstallStep, InstallTaskResponse

REQUIRED_MODULES = ["torch", "numpy", "grpc", "google.protobuf", "pydantic", "safetensors", "tokenizers", "PIL",
                    "yaml", "jinja2"]

STEP_NAMES = {
    "install_micromamba": "Install micromamba",
    "check_micromamba": "Check micromamba",
    "check_python": "Check Python dependencies",
    "create_environment": "Create environment",
    "install_drivers": "Install drivers",
    "install_packages": "Install Lumen packages",
    "build_native": "Build gfx950 kernels + host runtime",
    "verify_installation": "Verify installation",
    "prepare_cache": "Prepare cache directory",
}


class _Cancelled(Exception):
    pass


def plan_steps(req: InstallSetupRequest, core: CoreInstaller) -> list[tuple[str, str]]:
    steps = []
    if req.env_kind == "micromamba":
        steps.append("check_micromamba" if core.micromamba_ready() and not req.force_reinstall else "install_micromamba")
    steps.append("check_python")
    if req.env_kind != "current":
        steps.append("create_environment")
    try:
        from .env_checker import EnvironmentChecker

        rep = EnvironmentChecker.check_preset(req.preset)
        if rep.missing_installable:
            steps.append("install_drivers")
    except ValueError:
        pass
    if req.env_kind != "current":
        steps.append("install_packages")
    steps += ["build_native", "verify_installation", "prepare_cache"]
    return [(s, STEP_NAMES[s] + (f" '{req.environment_name}'" if s == "create_environment" else "")) for s in steps]


class InstallTask:
    def __init__(self, req: InstallSetupRequest, steps: list[tuple[str, str]]):
        now = time.time()
        self.req = req
        self.id = str(uuid.uuid4())
        self.cancel = threading.Event()
        self.logs: list[str] = []
        self.plan = steps
        self.resp = InstallTaskResponse(task_id=self.id, preset=req.preset, created_at=now, updated_at=now,
                                        steps=[InstallStep(step_id=s, name=n) for s, n in steps])
        self.lock = threading.Lock()

    def log(self, msg: str) -> None:
        with self.lock:
            self.logs.append(f"[{time.strftime('%H:%M:%S')}] {msg}")

    def snapshot(self) -> InstallTaskResponse:
        with self.lock:
            return self.resp.model_copy(deep=True)


def clear_cache_dir(cache_dir) -> Optional[str]:
    """Delete everything under cache_dir, keep the directory; refuse '/' and $HOME
    (reference install_orchestrator.py:746-763).  Returns an error message or None."""
    resolved = Path(cache_dir).expanduser().resolve()
    if resolved in (Path("/"), Path.home().resolve()):
        return f"Refusing to clear unsafe cache directory: {resolved}"
    try:
        resolved.mkdir(parents=True, exist_ok=True)
        for child in resolved.iterdir():
            if child.is_symlink() or child.is_file():
                child.unlink(missing_ok=True)
            else:
                shutil.rmtree(child)
        return None
    except Exception as e:  # noqa: BLE001
        return f"Failed to clear cache directory {resolved}: {e}"


class InstallOrchestrator:
    def __init__(self):
        self.tasks: dict[str, InstallTask] = {}
        self._lock = threading.Lock()

    def create(self, req: InstallSetupRequest) -> InstallTaskResponse:
        if P.get_preset(req.preset) is None:
            raise ValueError(f"unknown preset '{req.preset}'")
        core = CoreInstaller(req.cache_dir, req.env_kind, req.environment_name)
        t = InstallTask(req, plan_steps(req, core))
        t.core = core
        with self._lock:
            self.tasks[t.id] = t
        threading.Thread(target=self._run, args=(t,), daemon=True, name=f"install-{t.id[:8]}").start()
        return t.snapshot()

    def get(self, task_id: str) -> Optional[InstallTask]:
        return self.tasks.get(task_id)

    def list(self) -> list[InstallTaskResponse]:
        return [t.snapshot() for t in self.tasks.values()]

    def cancel(self, task_id: str) -> Optional[InstallTaskResponse]:
        """Request cancellation; the worker finishes it (kills the running child process,
        marks the steps, clears the cache).  A task that already ended is returned as is."""
        t = self.tasks.get(task_id)
        if t is None:
            return None
        with t.lock:
            active = t.resp.status in ("pending", "running")
        if active:
            t.cancel.set()
            ev = getattr(t, "done_event", None)
            if ev is not None:
                ev.wait(timeout=60)
        return t.snapshot()

    # ------------------------------------------------------------------ execution
    def _step(self, t: InstallTask, i: int, status: str, msg: str = "", progress: int = 0):
        with t.lock:
            s = t.resp.steps[i]
            now = time.time()
            if status == "running" and s.started_at is None:
                s.started_at = now
            if status in ("completed", "failed", "skipped"):
                s.completed_at = now
                progress = 100 if status != "failed" else progress
            s.status, s.message, s.progress = status, msg, progress
            t.resp.current_step = s.name
            done = sum(1 for x in t.resp.steps if x.status in ("completed", "skipped"))
            t.resp.progress = int(100 * done / len(t.resp.steps))
            t.resp.updated_at = now
        if msg:
            t.log(f"{s.step_id}: {msg}")

    def _finish_cancel(self, t: InstallTask) -> None:
        t.log("Cancelling installation and clearing cache directory...")
        err = clear_cache_dir(t.req.cache_dir)
        with t.lock:
            now = time.time()
            for s in t.resp.steps:
                if s.status == "running":
                    s.status, s.message = "cancelled", "Cancelled by user"
                    s.completed_at = now
                elif s.status == "pending":
                    s.status, s.message = "cancelled", "Cancelled before execution"
                    s.completed_at = now
                s.progress = 0
            t.resp.status = "cancelled"
            t.resp.progress = 0
            t.resp.completed_at = t.resp.updated_at = now
            t.resp.error = err
            t.resp.current_step = ("Installation cancelled, but cache cleanup failed" if err
                                   else "Installation cancelled and cache directory cleared")
        t.log(err or "Cache directory cleared successfully.")

    def _run(self, t: InstallTask) -> None:
        t.done_event = threading.Event()
        with t.lock:
            t.resp.status = "running"
        try:
            for i, (sid, _) in enumerate(t.plan):
                if t.cancel.is_set():
                    raise _Cancelled()
                self._step(t, i, "running")
                try:
                    getattr(self, f"_do_{sid}")(t, i)
                except Cancelled as e:
                    raise _Cancelled() from e
            with t.lock:
                t.resp.status = "completed"
                t.resp.progress = 100
                t.resp.completed_at = t.resp.updated_at = time.time()
            t.log("setup completed")
        except _Cancelled:
            self._finish_cancel(t)
        except Exception as e:  # noqa: BLE001
            if t.cancel.is_set():
                self._finish_cancel(t)
            else:
                with t.lock:
                    t.resp.status = "failed"
                    t.resp.error = str(e)
                    for s in t.resp.steps:
                        if s.status == "running":
                            s.status = "failed"
                    t.resp.updated_at = time.time()
                t.log(f"failed: {e}")
        finally:
            t.done_event.set()

    # ---- steps
    def _do_install_micromamba(self, t, i):
        self._step(t, i, "completed", t.core.install_micromamba(t.log, t.cancel, force=t.req.force_reinstall))

    def _do_check_micromamba(self, t, i):
        self._step(t, i, "completed", t.core.check_micromamba())

    def _do_check_python(self, t, i):
        missing = []
        for m in REQUIRED_MODULES:
            try:
                importlib.import_module(m)
            except Exception:  # noqa: BLE001
                missing.append(m)
        if missing:
            raise RuntimeError(f"missing python modules: {missing}")
        self._step(t, i, "completed", f"python {sys.version.split()[0]}; all {len(REQUIRED_MODULES)} modules present")

    def _do_create_environment(self, t, i):
        self._step(t, i, "completed", t.core.create_environment(t.log, t.cancel, force=t.req.force_reinstall))

    def _do_install_drivers(self, t, i):
        from .env_checker import EnvironmentChecker

        rep = EnvironmentChecker.check_preset(t.req.preset)
        self._step(t, i, "completed", t.core.install_drivers(rep.missing_installable, t.log, t.cancel))

    def _do_install_packages(self, t, i):
        self._step(t, i, "completed", t.core.install_packages(t.req.preset, t.req.wheel, t.log, t.cancel))

    def _do_build_native(self, t, i):
        msg = t.core.build_native(t.log, t.cancel, force=t.req.force_reinstall)
        self._step(t, i, "skipped" if msg.startswith("native libraries already") else "completed", msg)

    def _do_verify_installation(self, t, i):
        rep = t.core.verify(t.log, t.cancel)
        if not rep.ok:
            raise RuntimeError(f"verification failed: {rep.errors}")
        d = rep.details
        self._step(t, i, "completed", f"torch {d.get('torch')} (HIP {d.get('hip')}), GPUs {d.get('gpus')}, "
                                      f"native {d.get('native')}")

    def _do_prepare_cache(self, t, i):
        self._step(t, i, "completed", t.core.prepare_cache())
