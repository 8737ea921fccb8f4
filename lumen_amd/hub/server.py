"""``lumen`` hub server and the per-package single-service servers.

Flow (reference src/lumen/server.py:188-385 and packages/*/server.py):
load + validate the LumenConfig -> check the deployment mode -> resolve /
download every enabled model (offline-first; ``LUMEN_SYNTHETIC=1`` materialises
random-init models) -> build every service through its ``from_config`` and
*initialise* it (the reference hub never does) -> HubRouter ->
gRPC server on ``host:port`` (fixes the reference's ``"0.0.0.0::{port}"`` bind,
Q3) -> log the readiness line the control plane waits for
("Lumen Hub service listening on ...") -> optional mDNS -> SIGINT/SIGTERM ->
``server.stop(grace=5)``.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import socket
import sys
import threading
import uuid
from concurrent import futures
from typing import Optional

import grpc

from .. import __version__
from ..proto import ml_service as pb
from ..resources.config import LumenConfig
from ..resources.downloader import Downloader
from ..resources.validator import load_and_validate_config
from ..utils.logging import setup_logging
from .loader import ServiceLoader
from .router import HubRouter

log = logging.getLogger("lumen.server")


class AppService:
    """Instantiate + initialise every enabled service (reference src/lumen/service.py:12-49)."""

    def __init__(self, services: list, names: list[str]):
        self.services = services
        self.names = names

    @classmethod
    def from_app_config(cls, config: LumenConfig, initialize: bool = True) -> "AppService":
        """Each enabled service is built and initialised under its GPU set
        (runtime/placement.py: disjoint GPUs per service, DP workers per GPU)."""
        from ..runtime import placement

        services, names = [], []
        enabled = config.enabled_services()
        plan = placement.plan_from_env(list(enabled))
        for name, svc_cfg in enabled.items():
            cls_ = ServiceLoader.get_class(svc_cfg.import_info.registry_class)
            with placement.use(plan.get(name)):
                svc = cls_.from_config(svc_cfg, config.cache_path())
                if initialize and hasattr(svc, "initialize"):
                    svc.initialize()
            services.append(svc)
            names.append(name)
        app = cls(services, names)
        app.placement = plan
        return app

    def close(self):
        for s in self.services:
            try:
                s.close()
            except Exception:  # pragma: no cover
                pass


def handle_download_results(results: dict) -> None:
    failed = {k: r for k, r in results.items() if not r.success}
    for k, r in results.items():
        if r.success:
            log.info("model ready: %s -> %s%s", k, r.model_path, " (synthetic)" if r.synthetic else "")
    if failed:
        for k, r in failed.items():
            log.error("model %s failed: %s", k, r.error)
        raise SystemExit(1)


def setup_mdns(port: int, mdns_cfg) -> tuple:
    """Advertise ``_lumen._tcp.local.`` when zeroconf is importable (optional dependency)."""
    try:
        from zeroconf import ServiceInfo, Zeroconf  # type: ignore
    except Exception:
        log.warning("zeroconf not installed; mDNS advertisement disabled")
        return None, None
    ip = os.getenv("ADVERTISE_IP")
    if not ip:
        try:
            s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            s.connect(("8.8.8.8", 80))
            ip = s.getsockname()[0]
            s.close()
        except Exception:
            ip = "127.0.0.1"
    props = {"uuid": os.getenv("SERVICE_UUID", str(uuid.uuid4())), "status": os.getenv("SERVICE_STATUS", "ready"),
             "version": os.getenv("SERVICE_VERSION", "1.0.0")}
    stype = "_lumen._tcp.local."
    name = (getattr(mdns_cfg, "service_name", None) or "Lumen-Hub")
    info = ServiceInfo(type_=stype, name=f"{name}.{stype}", addresses=[socket.inet_aton(ip)], port=port,
                       properties=props, server=f"{socket.gethostname()}.local.")
    zc = Zeroconf()
    zc.register_service(info)
    log.info("mDNS: advertised %s at %s:%d", name, ip, port)
    return zc, info


def build_server(servicer, host: str, port: int, max_workers: int = 16):
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_receive_message_length", 64 * 1024 * 1024),
                                  ("grpc.max_send_message_length", 64 * 1024 * 1024)])
    if isinstance(servicer, HubRouter):
        servicer.attach_to_server(server)
    else:
        pb.add_InferenceServicer_to_server(servicer, server)
    bound = server.add_insecure_port(f"{host}:{port}")
    if bound == 0:
        raise RuntimeError(f"cannot bind {host}:{port}")
    return server, bound


def serve(config_path: str, port_override: Optional[int] = None, mode: str = "hub",
          stop_event: Optional[threading.Event] = None) -> None:
    config = load_and_validate_config(config_path)
    if config.deployment.mode != mode:
        log.error("this server runs deployment.mode=%s; config has %s", mode, config.deployment.mode)
        raise SystemExit(1)
    handle_download_results(Downloader(config).download_all())
    app = AppService.from_app_config(config)
    if mode == "single":
        target = config.deployment.service
        idx = app.names.index(target) if target in app.names else 0
        servicer = app.services[idx]
    else:
        servicer = HubRouter(app.services)
    host = config.server.host or "0.0.0.0"
    port = port_override or config.server.port
    server, bound = build_server(servicer, host, port)
    server.start()
    from ..runtime.metrics import start_metrics_server

    mport = start_metrics_server()
    if mport:
        log.info("Prometheus metrics on :%d/metrics", mport)
    kind = "Hub" if mode == "hub" else "single-service"
    log.info("🚀 Lumen %s service listening on %s:%d", kind, host, bound)
    print(f"Lumen {kind} service listening on {host}:{bound}", flush=True)
    for name, svc in zip(app.names, app.services):
        try:
            cap = svc.build_capability()
            log.info("  %s: %s", name, [t.name for t in cap.tasks])
        except Exception as e:  # pragma: no cover
            log.warning("  %s: capability probe failed: %s", name, e)
    zc = info = None
    mdns = config.server.mdns
    if mdns is not None and mdns.enabled:
        zc, info = setup_mdns(bound, mdns)
    done = stop_event or threading.Event()

    def _stop(signum, frame):
        log.info("signal %s: shutting down", signum)
        done.set()

    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGINT, _stop)
        signal.signal(signal.SIGTERM, _stop)
    done.wait()
    if zc is not None:
        try:
            zc.unregister_service(info)
            zc.close()
        except Exception:  # pragma: no cover
            pass
    server.stop(grace=5).wait()
    app.close()


def main(argv=None, mode: str = "hub", prog: str = "lumen") -> int:
    ap = argparse.ArgumentParser(prog=prog, description="Lumen MI355X inference server")
    ap.add_argument("--config", required=True, help="path to lumen-config.yaml")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--log-level", default="INFO", choices=["DEBUG", "INFO", "WARNING", "ERROR"])
    ap.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    args = ap.parse_args(argv)
    setup_logging(args.log_level)
    try:
        serve(args.config, args.port, mode=mode)
    except SystemExit as e:
        return int(e.code or 0)
    return 0


def main_single(argv=None) -> int:
    return main(argv, mode="single", prog="lumen-service")


if __name__ == "__main__":
    sys.exit(main())
