"""Lifecycle of the hub gRPC server process (reference
lumen-app/src/lumen_app/services/server_manager.py:89-390).

The reference spawns ``micromamba run -p <env> python -m lumen.server --config ...``;
here the hub runs from the same interpreter (``python -m lumen_amd.hub.server``) as a
child in its own process group, with stdout/stderr captured line by line into a ring
buffer that feeds ``/api/v1/server/logs`` and the ``/ws/logs`` websocket.  Health is
the gRPC ``Health`` RPC.  Stop sends SIGTERM to the child's process group (only ever
the group this manager created), escalating to SIGKILL after ``timeout`` or when
``force`` is set.
"""
from __future__ import annotations

import collections
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Optional

from .schemas import ServerLogs, ServerStatus


class ServerManager:
    def __init__(self, max_lines: int = 5000):
        self._proc: Optional[subprocess.Popen] = None
        self._lock = threading.Lock()
        self._logs: collections.deque = collections.deque(maxlen=max_lines)
        self._total = 0
        self._read_mark = 0
        self._started: Optional[float] = None
        self.port = 50051
        self.host = "0.0.0.0"
        self.config_path: Optional[str] = None
        self.environment = "lumen_env"
        self.service_name = "lumen-ai"
        self.last_error: Optional[str] = None
        self._listeners: list = []

    # ------------------------------------------------------------------ logs
    def _append(self, line: str) -> None:
        with self._lock:
            self._logs.append(line)
            self._total += 1
            listeners = list(self._listeners)
        for q in listeners:
            try:
                q.put_nowait(line)
            except Exception:
                pass

    def subscribe(self, q) -> None:
        with self._lock:
            self._listeners.append(q)

    def unsubscribe(self, q) -> None:
        with self._lock:
            if q in self._listeners:
                self._listeners.remove(q)

    def _pump(self, stream) -> None:
        for raw in iter(stream.readline, b""):
            self._append(raw.decode("utf-8", "replace").rstrip("\n"))
        stream.close()

    def logs(self, lines: int = 100) -> ServerLogs:
        with self._lock:
            data = list(self._logs)[-lines:] if lines > 0 else list(self._logs)
            new = self._total - self._read_mark
            self._read_mark = self._total
            return ServerLogs(logs=data, total_lines=self._total, new_lines=new)

    # ------------------------------------------------------------------ lifecycle
    @property
    def running(self) -> bool:
        return self._proc is not None and self._proc.poll() is None

    def start(self, config_path: str, port: Optional[int] = None, host: Optional[str] = None,
              environment: str = "lumen_env", extra_env: Optional[dict] = None) -> ServerStatus:
        if self.running:
            raise RuntimeError(f"server already running (pid {self._proc.pid})")
        if not config_path or not os.path.exists(os.path.expanduser(config_path)):
            raise FileNotFoundError(f"config not found: {config_path}")
        self.config_path = os.path.expanduser(config_path)
        self.environment = environment
        try:
            import yaml

            cfg = yaml.safe_load(open(self.config_path)) or {}
            srv = cfg.get("server", {}) or {}
            self.port = int(port or srv.get("port", 50051))
            self.host = host or srv.get("host", "0.0.0.0") or "0.0.0.0"
            self.service_name = ((srv.get("mdns") or {}).get("service_name")) or self.service_name
        except Exception:
            self.port = int(port or 50051)
        cmd = [sys.executable, "-m", "lumen_amd.hub.server", "--config", self.config_path, "--port", str(self.port)]
        env = dict(os.environ)
        env.update(extra_env or {})
        self._append(f"[lumen-app] starting: {' '.join(cmd)}")
        self._proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env,
                                      start_new_session=True)
        threading.Thread(target=self._pump, args=(self._proc.stdout,), daemon=True).start()
        self._started = time.time()
        self.last_error = None
        return self.status()

    def stop(self, force: bool = False, timeout: int = 30) -> ServerStatus:
        p = self._proc
        if p is None or p.poll() is not None:
            return self.status()
        try:
            pgid = os.getpgid(p.pid)
        except ProcessLookupError:
            pgid = None
        sig = signal.SIGKILL if force else signal.SIGTERM
        if pgid is not None and pgid == p.pid:
            os.killpg(pgid, sig)
        else:
            p.send_signal(sig)
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            if pgid is not None and pgid == p.pid:
                os.killpg(pgid, signal.SIGKILL)
            else:
                p.kill()
            p.wait(timeout=10)
        self._append(f"[lumen-app] server stopped (exit {p.returncode})")
        self._started = None
        return self.status()

    def health(self, timeout: float = 1.0) -> str:
        if not self.running:
            return "unknown"
        try:
            import grpc

            from ..proto import ml_service as pb

            host = "127.0.0.1" if self.host in ("0.0.0.0", "::", "") else self.host
            with grpc.insecure_channel(f"{host}:{self.port}") as ch:
                pb.InferenceStub(ch).Health(pb.Empty(), timeout=timeout)
            return "healthy"
        except Exception as e:  # noqa: BLE001
            self.last_error = str(e)[:200]
            return "unhealthy"

    def status(self, check_health: bool = False) -> ServerStatus:
        run = self.running
        if self._proc is not None and not run and self._proc.returncode not in (0, None, -15, -9):
            self.last_error = self.last_error or f"server exited with code {self._proc.returncode}"
        return ServerStatus(running=run, pid=self._proc.pid if run else None, port=self.port, host=self.host,
                            uptime_seconds=(time.time() - self._started) if run and self._started else None,
                            service_name=self.service_name, config_path=self.config_path,
                            environment=self.environment, health=self.health() if (check_health and run) else
                            ("unknown" if run else "unknown"), last_error=self.last_error)
