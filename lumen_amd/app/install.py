"""One-click setup tasks (reference lumen-app/src/lumen_app/services/install_orchestrator.py,
installer.py, install_task_repository.py).

The reference installs micromamba, creates a conda env and pip-installs the packages.
The MI355X build runs from the current interpreter, so a setup task verifies the
Python dependencies, checks the preset's drivers (ROCm / HIP / gfx950), builds the
native gfx950 kernel + host runtime libraries (``python -m lumen_amd._build`` in a
child process, output streamed into the task log) and prepares the cache directory.
Tasks run on a background thread, report per-step progress, can be cancelled and
keep their logs for ``/api/v1/install/tasks/{id}/logs`` and ``/ws/install/{id}``.
"""
from __future__ import annotations

import importlib
import os
import subprocess
import sys
import threading
import time
import uuid
from pathlib import Path
from typing import Optional

from . import presets as P
from .hardware import check_driver
from .schemas import InstallSetupRequest, InstallStep, InstallTaskResponse

REQUIRED_MODULES = ["torch", "numpy", "grpc", "google.protobuf", "pydantic", "safetensors", "tokenizers", "PIL",
                    "yaml", "jinja2"]


class _Cancelled(Exception):
    pass


class InstallTask:
    def __init__(self, req: InstallSetupRequest):
        now = time.time()
        self.req = req
        self.id = str(uuid.uuid4())
        self.cancel = threading.Event()
        self.logs: list[str] = []
        self.resp = InstallTaskResponse(task_id=self.id, preset=req.preset, created_at=now, updated_at=now,
                                        steps=[InstallStep(step_id=s, name=n) for s, n in STEPS])
        self.lock = threading.Lock()

    def log(self, msg: str) -> None:
        with self.lock:
            self.logs.append(f"[{time.strftime('%H:%M:%S')}] {msg}")

    def snapshot(self) -> InstallTaskResponse:
        with self.lock:
            return self.resp.model_copy(deep=True)


STEPS = [("check_python", "Check Python dependencies"), ("check_drivers", "Check drivers"),
         ("build_native", "Build gfx950 kernels + host runtime"), ("prepare_cache", "Prepare cache directory")]


class InstallOrchestrator:
    def __init__(self):
        self.tasks: dict[str, InstallTask] = {}
        self._lock = threading.Lock()

    def create(self, req: InstallSetupRequest) -> InstallTaskResponse:
        if P.get_preset(req.preset) is None:
            raise ValueError(f"unknown preset '{req.preset}'")
        t = InstallTask(req)
        with self._lock:
            self.tasks[t.id] = t
        threading.Thread(target=self._run, args=(t,), daemon=True, name=f"install-{t.id[:8]}").start()
        return t.snapshot()

    def get(self, task_id: str) -> Optional[InstallTask]:
        return self.tasks.get(task_id)

    def list(self) -> list[InstallTaskResponse]:
        return [t.snapshot() for t in self.tasks.values()]

    def cancel(self, task_id: str) -> Optional[InstallTaskResponse]:
        t = self.tasks.get(task_id)
        if t is None:
            return None
        t.cancel.set()
        with t.lock:
            if t.resp.status in ("pending", "running"):
                t.resp.status = "cancelled"
                for s in t.resp.steps:
                    if s.status in ("pending", "running"):
                        s.status = "cancelled"
                t.resp.updated_at = time.time()
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

    def _run(self, t: InstallTask) -> None:
        with t.lock:
            t.resp.status = "running"
        try:
            for i, (sid, _) in enumerate(STEPS):
                if t.cancel.is_set():
                    raise _Cancelled()
                self._step(t, i, "running")
                getattr(self, f"_do_{sid}")(t, i)
            with t.lock:
                t.resp.status = "completed"
                t.resp.progress = 100
                t.resp.completed_at = t.resp.updated_at = time.time()
            t.log("setup completed")
        except _Cancelled:
            t.log("cancelled")
        except Exception as e:  # noqa: BLE001
            with t.lock:
                t.resp.status = "failed"
                t.resp.error = str(e)
                for s in t.resp.steps:
                    if s.status == "running":
                        s.status = "failed"
                t.resp.updated_at = time.time()
            t.log(f"failed: {e}")

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

    def _do_check_drivers(self, t, i):
        dc = P.get_preset(t.req.preset).create_config()
        res = [check_driver(d) for d in dc.drivers if d != "lumen_native"]
        bad = [f"{d.name}: {d.status} ({d.details})" for d in res if d.status != "available"]
        if bad:
            raise RuntimeError("; ".join(bad))
        self._step(t, i, "completed", ", ".join(f"{d.name} ok" for d in res) or "no drivers required")

    def _do_build_native(self, t, i):
        from .._native import HIP_SO, HOST_SO

        if HIP_SO.exists() and HOST_SO.exists() and not t.req.force_reinstall:
            self._step(t, i, "skipped", "native libraries already built")
            return
        root = Path(__file__).resolve().parents[2]
        p = subprocess.Popen([sys.executable, "-m", "lumen_amd._build"], cwd=str(root), stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, start_new_session=True)
        for raw in iter(p.stdout.readline, b""):
            t.log(raw.decode("utf-8", "replace").rstrip())
            if t.cancel.is_set():
                p.terminate()
                p.wait(timeout=30)
                raise _Cancelled()
        rc = p.wait()
        if rc != 0:
            raise RuntimeError(f"native build failed (exit {rc})")
        self._step(t, i, "completed", "built _lumen_hip.so (gfx950) and _lumen_host.so")

    def _do_prepare_cache(self, t, i):
        root = Path(os.path.expanduser(t.req.cache_dir))
        (root / "models").mkdir(parents=True, exist_ok=True)
        self._step(t, i, "completed", f"cache ready at {root}")
