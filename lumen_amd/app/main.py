"""lumen-app control plane (FastAPI): config generation, hardware detection, setup
tasks, hub server lifecycle, log websockets, SPA static files.

Endpoint paths, request and response shapes follow SURVEY §A.1 (reference
lumen-app/src/lumen_app/main.py:70-92, api/{config,hardware,install,server}.py,
websockets/logs.py).  Run: ``lumen-app`` / ``python -m lumen_amd.app.main --port 8000``.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import queue
import shutil
import time
from pathlib import Path
from typing import Optional

import yaml
from fastapi import APIRouter, FastAPI, HTTPException, WebSocket, WebSocketDisconnect
from fastapi.responses import FileResponse, HTMLResponse, JSONResponse

from .. import __version__
from ..resources.config import LumenConfig
from ..resources.validator import load_and_validate_config, structural_errors
from . import presets as P
from .hardware import check_driver, free_space_gb, hardware_info, preset_response, recommend
from .install import InstallOrchestrator
from .schemas import (CheckInstallationPathResponse, ConfigRequest, ConfigResponse, DriverCheckResponse,
                      HardwarePresetResponse, InstallLogsResponse, InstallSetupRequest, InstallStatusResponse,
                      InstallTaskListResponse, InstallTaskResponse, PathRequest, ServerLogs, ServerRestartRequest,
                      ServerStartRequest, ServerStatus, ServerStopRequest, ServiceStatus)
from .server_manager import ServerManager

STATIC_DIR = Path(os.environ.get("LUMEN_WEB_DIR", Path(__file__).parent / "static"))


class AppState:
    def __init__(self):
        self.config: Optional[LumenConfig] = None
        self.config_path: Optional[str] = None
        self.preset: Optional[str] = None
        self.server = ServerManager()
        self.installs = InstallOrchestrator()

    def set_config(self, cfg: LumenConfig, path: str, preset: Optional[str] = None):
        self.config, self.config_path = cfg, path
        if preset:
            self.preset = preset


def _dump_yaml(cfg: LumenConfig) -> str:
    return yaml.safe_dump(cfg.model_dump(mode="json", exclude_none=True), sort_keys=False)


def create_app(state: Optional[AppState] = None) -> FastAPI:
    st = state or AppState()
    app = FastAPI(title="Lumen (MI355X)", version=__version__)
    app.state.lumen = st

    @app.get("/health")
    def health():
        return {"status": "ok", "version": "0.1.0"}

    @app.get("/metrics")
    def metrics():
        from fastapi.responses import Response

        from ..runtime.metrics import exposition

        return Response(exposition(), media_type="text/plain; version=0.0.4")

    # ------------------------------------------------------------------ config
    cfg = APIRouter(prefix="/api/v1/config")

    @cfg.post("/generate", response_model=ConfigResponse)
    def generate(req: ConfigRequest):
        p = P.get_preset(req.preset)
        if p is None:
            raise HTTPException(status_code=400, detail=f"Unknown preset: {req.preset}")
        try:
            c = P.Config(req.cache_dir, p.create_config(), req.region, req.service_name, req.port)
            if req.config_type == "minimal":
                lc = c.minimal()
            elif req.config_type == "light_weight":
                lc = c.light_weight(req.clip_model if req.clip_model in ("MobileCLIP2-S2", "CN-CLIP_ViT-B-16") else None)
            elif req.config_type == "basic":
                lc = c.basic(req.clip_model if req.clip_model in ("MobileCLIP2-S4", "CN-CLIP_ViT-L-14") else None)
            else:
                lc = c.brave()
            root = Path(req.cache_dir).expanduser()
            root.mkdir(parents=True, exist_ok=True)
            path = root / "lumen-config.yaml"
            path.write_text(_dump_yaml(lc), encoding="utf-8")
            st.set_config(lc, str(path), p.name)
            warnings = []
            if not preset_response(p).ready:
                warnings.append(f"preset {p.name} is not ready on this machine (missing drivers)")
            return ConfigResponse(success=True, preset=req.preset, config_path=str(path),
                                  config_content=lc.model_dump(mode="json"),
                                  message=f"Configuration generated successfully at {path}", warnings=warnings)
        except HTTPException:
            raise
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=500, detail=f"Failed to generate configuration: {e}")

    @cfg.get("/current")
    def current():
        lc = st.config
        if lc is None:
            return {"loaded": False, "message": "No configuration loaded"}
        device = None
        for sc in lc.services.values():
            if sc.enabled and sc.backend_settings:
                b = sc.backend_settings
                m = next(iter(sc.models.values()), None)
                device = {"runtime": m.runtime.value if m else "onnx", "batch_size": b.batch_size or 1,
                          "precision": (m.precision if m and m.precision else "fp32"),
                          "rknn_device": m.rknn_device if m else None, "onnx_providers": b.onnx_providers or []}
                break
        return {"loaded": True, "config_path": st.config_path, "cache_dir": lc.metadata.cache_dir,
                "region": lc.metadata.region.value, "port": lc.server.port,
                "service_name": lc.server.mdns.service_name if lc.server.mdns else "lumen-server",
                "env_name": "lumen_env", "device": device}

    @cfg.post("/validate")
    def validate(body: dict):
        errs = structural_errors(body)
        if not errs:
            try:
                LumenConfig.model_validate(body)
            except Exception as e:  # noqa: BLE001
                errs = [str(e)]
        return {"valid": not errs, "errors": errs, "warnings": []}

    @cfg.post("/validate-path")
    def validate_path(req: dict):
        s = (req or {}).get("path", "")
        if not s:
            return {"valid": False, "exists": False, "writable": False, "error": "path must not be empty"}
        p = Path(s).expanduser()
        exists = p.exists()
        error = warning = None
        if exists:
            writable = os.access(p, os.W_OK)
            if not writable:
                error = f"no write permission: {p}"
        elif p.parent.exists():
            writable = os.access(p.parent, os.W_OK)
            if not writable:
                error = f"cannot create directory under {p.parent}"
        else:
            writable = False
            error = f"parent directory does not exist: {p.parent}"
        free = free_space_gb(str(p))
        if free < 10:
            warning = f"only {free:.1f} GB free (>= 10 GB recommended)"
        return {"valid": bool(writable and free >= 10 and error is None), "exists": exists, "writable": writable,
                "free_space_gb": round(free, 2), "error": error, "warning": warning}

    @cfg.post("/load")
    def load(config_path: str):
        p = Path(config_path).expanduser()
        if not p.exists():
            raise HTTPException(status_code=404, detail=f"config not found: {p}")
        try:
            lc = load_and_validate_config(str(p))
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=400, detail=f"invalid config: {e}")
        st.set_config(lc, str(p))
        return {"loaded": True, "config_path": str(p), "cache_dir": lc.metadata.cache_dir,
                "region": lc.metadata.region.value, "port": lc.server.port,
                "service_name": lc.server.mdns.service_name if lc.server.mdns else "lumen-server",
                "env_name": "lumen_env"}

    @cfg.get("/yaml")
    def get_yaml():
        if st.config is None:
            return {"loaded": False, "yaml": "", "cache_dir": None}
        text = Path(st.config_path).read_text() if st.config_path and Path(st.config_path).exists() \
            else _dump_yaml(st.config)
        return {"loaded": True, "yaml": text, "cache_dir": st.config.metadata.cache_dir}

    app.include_router(cfg)

    # ------------------------------------------------------------------ hardware
    hw = APIRouter(prefix="/api/v1/hardware")

    @hw.get("/info")
    def info():
        return hardware_info()

    @hw.get("/presets", response_model=list[HardwarePresetResponse])
    def list_presets():
        return [preset_response(P.PRESETS[n], check=False) for n in P.detection_order()]

    @hw.get("/presets/{name}/check", response_model=list[DriverCheckResponse])
    def check(name: str):
        p = P.get_preset(name)
        if p is None:
            raise HTTPException(status_code=404, detail=f"Unknown preset: {name}")
        return [check_driver(d) for d in p.create_config().drivers]

    @hw.post("/detect")
    def detect():
        pres = [preset_response(P.PRESETS[n]) for n in P.detection_order()]
        rec = next((p.name for p in pres if p.ready), "cpu")
        return {"recommended_preset": rec,
                "detailed_status": [{"preset": p.name, "availability": p.availability, "ready": p.ready,
                                     "drivers": [d.model_dump() for d in p.drivers]} for p in pres]}

    app.include_router(hw)

    # ------------------------------------------------------------------ install
    ins = APIRouter(prefix="/api/v1/install")

    def _status(cache_dir: str, preset: Optional[str] = None) -> InstallStatusResponse:
        from .._native import HIP_SO, HOST_SO

        built = HIP_SO.exists() and HOST_SO.exists()
        preset = preset or st.preset or recommend()
        p = P.get_preset(preset) or P.PRESETS["cpu"]
        drivers = {d: check_driver(d).status for d in p.create_config().drivers}
        missing = [k for k, v in drivers.items() if v != "available"]
        if not built:
            missing.append("lumen_native")
        return InstallStatusResponse(micromamba_installed=False, micromamba_path=None, environment_exists=built,
                                     environment_name="lumen_env" if built else None,
                                     environment_path=str(HIP_SO.parent) if built else None, drivers_checked=True,
                                     drivers=drivers, ready_for_preset=p.name if not missing else None,
                                     missing_components=sorted(set(missing)))

    @ins.get("/check-path", response_model=CheckInstallationPathResponse)
    def check_path(path: str):
        root = Path(path).expanduser()
        has_cfg = (root / "lumen-config.yaml").exists()
        s = _status(str(root))
        ss = ServiceStatus(micromamba=True, environment=s.environment_exists, config=has_cfg,
                           drivers=not [m for m in s.missing_components if m != "lumen_native"])
        ready = has_cfg and ss.environment and ss.drivers
        action = "start_existing" if ready else ("repair" if has_cfg else "configure_new")
        return CheckInstallationPathResponse(has_existing_service=has_cfg, service_status=ss, ready_to_start=ready,
                                             recommended_action=action,
                                             message="ready to start" if ready else "configuration or setup required")

    @ins.get("/status", response_model=InstallStatusResponse)
    def status(cache_dir: str = "~/.lumen"):
        return _status(cache_dir)

    @ins.post("/setup", response_model=InstallTaskResponse)
    def setup(req: InstallSetupRequest):
        try:
            return st.installs.create(req)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))

    @ins.get("/tasks", response_model=InstallTaskListResponse)
    def tasks():
        t = st.installs.list()
        return InstallTaskListResponse(tasks=t, total=len(t))

    @ins.get("/tasks/{task_id}", response_model=InstallTaskResponse)
    def task(task_id: str):
        t = st.installs.get(task_id)
        if t is None:
            raise HTTPException(status_code=404, detail="task not found")
        return t.snapshot()

    @ins.post("/tasks/{task_id}/cancel", response_model=InstallTaskResponse)
    def cancel(task_id: str):
        r = st.installs.cancel(task_id)
        if r is None:
            raise HTTPException(status_code=404, detail="task not found")
        return r

    @ins.get("/tasks/{task_id}/logs", response_model=InstallLogsResponse)
    def task_logs(task_id: str, tail: int = 100):
        t = st.installs.get(task_id)
        if t is None:
            raise HTTPException(status_code=404, detail="task not found")
        with t.lock:
            logs = list(t.logs)
        return InstallLogsResponse(task_id=task_id, logs=logs[-tail:] if tail > 0 else logs, total_lines=len(logs))

    app.include_router(ins)

    # ------------------------------------------------------------------ server
    srv = APIRouter(prefix="/api/v1/server")

    @srv.get("/status", response_model=ServerStatus)
    def server_status():
        return st.server.status(check_health=True)

    @srv.post("/start", response_model=ServerStatus)
    def server_start(req: ServerStartRequest):
        path = req.config_path or st.config_path
        if not path:
            raise HTTPException(status_code=400, detail="no configuration loaded; generate or load one first")
        if st.server.running:
            raise HTTPException(status_code=409, detail="server already running")
        try:
            return st.server.start(path, req.port, req.host, req.environment)
        except FileNotFoundError as e:
            raise HTTPException(status_code=404, detail=str(e))
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=500, detail=f"failed to start server: {e}")

    @srv.post("/stop", response_model=ServerStatus)
    def server_stop(req: Optional[ServerStopRequest] = None):
        req = req or ServerStopRequest()
        return st.server.stop(force=req.force, timeout=req.timeout)

    @srv.post("/restart", response_model=ServerStatus)
    def server_restart(req: ServerRestartRequest):
        st.server.stop(force=req.force, timeout=req.timeout)
        path = req.config_path or st.server.config_path or st.config_path
        if not path:
            raise HTTPException(status_code=400, detail="no configuration to restart with")
        return st.server.start(path, req.port, req.host, req.environment)

    @srv.get("/logs", response_model=ServerLogs)
    def server_logs(lines: int = 100):
        return st.server.logs(lines)

    app.include_router(srv)

    # ------------------------------------------------------------------ websockets
    @app.websocket("/ws/logs")
    async def ws_logs(ws: WebSocket):
        await ws.accept()
        q: "queue.Queue[str]" = queue.Queue(maxsize=10000)
        st.server.subscribe(q)
        await ws.send_json({"type": "connected", "message": "log stream connected", "timestamp": time.time()})
        try:
            last = time.time()
            while True:
                sent = False
                while True:
                    try:
                        line = q.get_nowait()
                    except queue.Empty:
                        break
                    await ws.send_json({"type": "log", "message": line, "timestamp": time.time()})
                    sent = True
                if time.time() - last > 15:
                    await ws.send_json({"type": "heartbeat", "timestamp": time.time()})
                    last = time.time()
                await asyncio.sleep(0.05 if sent else 0.2)
        except WebSocketDisconnect:
            pass
        except Exception as e:  # noqa: BLE001
            try:
                await ws.send_json({"type": "error", "message": str(e)})
            except Exception:
                pass
        finally:
            st.server.unsubscribe(q)

    @app.websocket("/ws/install/{task_id}")
    async def ws_install(ws: WebSocket, task_id: str):
        await ws.accept()
        t = st.installs.get(task_id)
        if t is None:
            await ws.send_json({"type": "error", "message": "task not found"})
            await ws.close()
            return
        try:
            last = None
            while True:
                snap = t.snapshot()
                if snap.updated_at != last:
                    await ws.send_json({"type": "status", "task": snap.model_dump()})
                    last = snap.updated_at
                if snap.status in ("completed", "failed", "cancelled"):
                    await ws.send_json({"type": "complete" if snap.status == "completed" else "error",
                                        "task": snap.model_dump(), "message": snap.error or snap.status})
                    break
                await asyncio.sleep(0.2)
        except WebSocketDisconnect:
            return
        await ws.close()

    # ------------------------------------------------------------------ SPA
    @app.get("/{full_path:path}")
    def spa(full_path: str):
        if full_path.startswith("api/") or full_path.startswith("ws/"):
            raise HTTPException(status_code=404, detail="not found")
        f = (STATIC_DIR / full_path).resolve()
        if full_path and f.is_file() and STATIC_DIR.resolve() in f.parents:
            return FileResponse(str(f))
        idx = STATIC_DIR / "index.html"
        if idx.exists():
            return FileResponse(str(idx))
        return HTMLResponse("<html><body><h1>Lumen (MI355X)</h1><p>API at /api/v1, docs at /docs</p></body></html>")

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="lumen-app")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_app(), host=a.host, port=a.port, log_level="info")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
