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
    def from_app_config(cls, config: LumenConfig, initialize: bool = True, proxies: Optional[dict] = None,
                        only=None) -> "AppService":
        """Each enabled service is built and initialised under its GPU set
        (runtime/placement.py: disjoint GPUs per service, DP workers per GPU).  In a serving front
        end (parallel/engine.py) a service whose engines are attached finds them through
        ``remote_scope`` and loads no model here; a service in ``proxies`` (name -> address) is a
        :class:`~lumen_amd.hub.proxy.ProxyService` to the serving parent.  ``only``: build just
        these services (the parent's share of a mixed topology)."""
        from ..parallel.engine import remote_scope
        from ..runtime import placement

        services, names = [], []
        enabled = config.enabled_services()
        plan = placement.plan_from_env(list(enabled))
        for name, svc_cfg in enabled.items():
            if only is not None and name not in only:
                continue
            if proxies and name in proxies:
                from .proxy import ProxyService

                services.append(ProxyService(proxies[name], name))
                names.append(name)
                continue
            cls_ = ServiceLoader.get_class(svc_cfg.import_info.registry_class)
            with placement.use(plan.get(name)), remote_scope(name):
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


def build_server(servicer, host: str, port: int, max_workers: int = 16, reuse_port: bool = False):
    opts = [("grpc.max_receive_message_length", 64 * 1024 * 1024),
            ("grpc.max_send_message_length", 64 * 1024 * 1024)]
    if reuse_port:   # several replica processes accept on one port; the kernel spreads the connections
        opts.append(("grpc.so_reuseport", 1))
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=opts)
    if isinstance(servicer, HubRouter):
        servicer.attach_to_server(server)
    else:
        pb.add_InferenceServicer_to_server(servicer, server)
    bound = server.add_insecure_port(f"{host}:{port}")
    if bound == 0:
        raise RuntimeError(f"cannot bind {host}:{port}")
    return server, bound


def _replica_main(config_path: str, port: int, mode: str, stop_event, ready_q, idx: int, parent_pid: int) -> None:
    """A replica process of :func:`serve` (spawned before any GPU use): same config, same port.
    ``stop_event`` is the parent's shared stop; ``parent_pid`` the pid to outlive-check against
    (a plain ``getppid() == 1`` test misfires when the parent itself is PID 1 in a container)."""
    setup_logging(os.environ.get("LUMEN_LOG_LEVEL", "INFO"))
    serve(config_path, port, mode=mode, stop_event=stop_event, procs=1, replica=idx, ready_q=ready_q,
          parent_pid=parent_pid)


def _frontend_main(config_path: str, port: int, mode: str, stop_event, ready_q, idx: int, parent_pid: int,
                   specs: dict, proxies: Optional[dict] = None) -> None:
    """A serving front-end process (spawned before any GPU use): the services of the config with
    their GPU work forwarded to the engine processes (or, for ``proxies``, whole requests to the
    serving parent), gRPC on the shared port (SO_REUSEPORT)."""
    setup_logging(os.environ.get("LUMEN_LOG_LEVEL", "INFO"))
    from ..parallel.engine import attach_frontend

    from ..utils.sampler import maybe_start

    attach_frontend(specs)
    stop_sampler = maybe_start(f"frontend{idx}")   # LUMEN_SAMPLE_DIR: stack samples of every thread
    try:
        serve(config_path, port, mode=mode, stop_event=stop_event, procs=1, replica=idx, ready_q=ready_q,
              parent_pid=parent_pid, frontends=0, proxies=proxies)
    finally:
        stop_sampler()


def engine_devices() -> list[str]:
    """One engine per visible GPU (LUMEN_ENGINE_DEVICES=cuda:0,cuda:1,... to choose), else one CPU engine."""
    env = os.environ.get("LUMEN_ENGINE_DEVICES")
    if env:
        return [d.strip() for d in env.split(",") if d.strip()]
    try:
        import torch

        n = torch.cuda.device_count()   # counts without initialising the GPU in this process
    except Exception:  # noqa: BLE001
        n = 0
    return [f"cuda:{i}" for i in range(n)] or ["cpu"]


def serve_frontends(config_path: str, port: int, frontends: int, mode: str = "hub",
                    stop_event: Optional[threading.Event] = None, ready_q=None, devices=None) -> bool:
    """Engine/front-end topology: one GPU engine process per device holding the models, and
    ``frontends`` gRPC front-end processes sharing ``port``.  A service that cannot run on engines
    (``engine_spec()`` None: a tensor-parallel VLM) is served by THIS process on a private local
    socket, and the front ends proxy its tasks there (hub/proxy.py): a mixed topology, never an
    all-or-nothing fallback.  Returns False (nothing started) only when no service can use engines."""
    import multiprocessing as mp
    import tempfile

    from ..parallel.engine import EngineSet

    config = load_and_validate_config(config_path)
    handle_download_results(Downloader(config).download_all())
    specs, local = {}, []
    exclude = {x.strip() for x in os.environ.get("LUMEN_ENGINE_EXCLUDE", "").split(",") if x.strip()}
    for name, svc_cfg in config.enabled_services().items():
        cls_ = ServiceLoader.get_class(svc_cfg.import_info.registry_class)
        svc = cls_.from_config(svc_cfg, config.cache_path())   # not initialised: no model, no GPU
        spec = svc.engine_spec() if hasattr(svc, "engine_spec") and name not in exclude else None
        try:
            svc.close()
        except Exception:  # noqa: BLE001
            pass
        if spec is None:
            log.warning("service %s cannot run on GPU engines: served by the parent process, proxied by the "
                        "front ends", name)
            local.append(name)
        else:
            specs[name] = spec
    if not specs:
        log.warning("no service of this config can run on GPU engines: serving in-process instead")
        return False
    devs = list(devices or engine_devices())
    log.info("starting %d GPU engine(s) on %s for %s", len(devs), devs, list(specs))
    # batch loops per (engine, service): one runs its GPU work while the other assembles / decodes the
    # next merged batch (LUMEN_ENGINE_THREADS); a popped batch lingers LUMEN_ENGINE_LINGER_US for more
    # front-end batches -- with 3 loops and 1.5 ms the engine ran 320 batches/s of 6.5 images, every
    # loop busy on per-batch overhead (profiles/r4_serve_fe_v1.txt)
    engines = EngineSet(specs, devs, threads_per_service=int(os.environ.get("LUMEN_ENGINE_THREADS", "3")),
                        linger_us=int(os.environ.get("LUMEN_ENGINE_LINGER_US", "5000")))
    ctx = mp.get_context("spawn")
    stop = ctx.Event()
    rq = ready_q if ready_q is not None else ctx.Queue()
    addr = f"unix:{tempfile.gettempdir()}/lumen-hub-{os.getpid()}-{uuid.uuid4().hex[:8]}.sock" if local else None
    proxies = {name: addr for name in local}
    # front ends first: they are spawned before this process initialises any GPU (a spawned child
    # must not start from a GPU-initialised parent); their proxies wait for the local server
    procs = [ctx.Process(target=_frontend_main, args=(config_path, port, mode, stop, rq, i + 1, os.getpid(),
                                                      engines.frontend_specs(), proxies), daemon=False)
             for i in range(frontends)]
    for p in procs:
        p.start()
    local_app = local_server = None
    if local:
        local_app = AppService.from_app_config(config, only=set(local))
        local_server = grpc.server(futures.ThreadPoolExecutor(max_workers=64),
                                   options=[("grpc.max_receive_message_length", 64 * 1024 * 1024),
                                            ("grpc.max_send_message_length", 64 * 1024 * 1024)])
        HubRouter(local_app.services).attach_to_server(local_server)
        if local_server.add_insecure_port(addr) == 0:
            raise RuntimeError(f"cannot bind {addr}")
        local_server.start()
        log.info("parent serves %s on %s for the front ends", local, addr)
    if ready_q is None:
        for _ in procs:
            rq.get(timeout=900)
    log.info("Lumen front ends: %d process(es) on :%d over %d engine(s)", frontends, port, len(devs))
    print(f"Lumen Hub service listening on {config.server.host or '0.0.0.0'}:{port} "
          f"({frontends} front ends, {len(devs)} engines)", flush=True)
    done = stop_event or threading.Event()

    def _stop(signum, frame):
        log.info("signal %s: shutting down", signum)
        done.set()

    if threading.current_thread() is threading.main_thread() and stop_event is None:
        signal.signal(signal.SIGINT, _stop)
        signal.signal(signal.SIGTERM, _stop)
    while not done.wait(0.5):
        pass
    stop.set()
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    if local_server is not None:
        local_server.stop(grace=2)
        local_app.close()
        try:
            os.unlink(addr[len("unix:"):])
        except OSError:
            pass
    engines.close()
    return True


def _pid_alive(pid: int) -> bool:
    if os.getppid() != pid:        # re-parented: the original parent exited
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:       # pragma: no cover - exists, other owner
        return True
    return True


def start_replicas(config_path: str, port: int, n: int, mode: str = "hub", ready_q=None):
    """Spawn ``n`` replica server processes of ``config_path`` on ``port`` (SO_REUSEPORT).  Python
    gRPC serving is bound by one interpreter's lock (~0.7k one-image streams/s per process on the
    CLIP path, r3_serve_clip_256c_dp2_v1.log); replicas multiply that, each with its own models and
    batchers on the GPU(s).  Must run before this process initialises the GPU.  Returns
    (processes, stop event)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    stop = ctx.Event()
    procs = [ctx.Process(target=_replica_main, args=(config_path, port, mode, stop, ready_q, i + 1, os.getpid()),
                         daemon=False)
             for i in range(n)]
    for p in procs:
        p.start()
    return procs, stop


def serve(config_path: str, port_override: Optional[int] = None, mode: str = "hub",
          stop_event: Optional[threading.Event] = None, procs: Optional[int] = None, replica: int = 0,
          ready_q=None, parent_pid: Optional[int] = None, frontends: Optional[int] = None,
          proxies: Optional[dict] = None) -> None:
    """Run the server.  ``frontends`` > 0 (or LUMEN_FRONTENDS): GPU engine processes + that many
    front-end processes on one port (:func:`serve_frontends`).  ``procs`` > 1 (or LUMEN_HUB_PROCS):
    this process plus procs - 1 spawned full replicas accept on the same port (SO_REUSEPORT; a
    fixed port is required)."""
    config = load_and_validate_config(config_path)
    if config.deployment.mode != mode:
        log.error("this server runs deployment.mode=%s; config has %s", mode, config.deployment.mode)
        raise SystemExit(1)
    nfront = int(frontends if frontends is not None else os.environ.get("LUMEN_FRONTENDS", "0"))
    if nfront > 0 and replica == 0:
        port0 = port_override or config.server.port
        if not port0:
            raise SystemExit("front-end processes need a fixed server.port")
        if serve_frontends(config_path, port0, nfront, mode, stop_event=stop_event):
            return
    nproc = int(procs if procs is not None else os.environ.get("LUMEN_HUB_PROCS", "1"))
    if replica == 0:
        handle_download_results(Downloader(config).download_all())
    reps, rep_stop = [], None
    if nproc > 1 and replica == 0:
        port0 = port_override or config.server.port
        if not port0:
            raise SystemExit("LUMEN_HUB_PROCS > 1 needs a fixed server.port")
        reps, rep_stop = start_replicas(config_path, port0, nproc - 1, mode)
    app = AppService.from_app_config(config, proxies=proxies)
    if mode == "single":
        target = config.deployment.service
        idx = app.names.index(target) if target in app.names else 0
        servicer = app.services[idx]
    else:
        servicer = HubRouter(app.services)
    host = config.server.host or "0.0.0.0"
    port = port_override or config.server.port
    multi = nproc > 1 or replica > 0
    server, bound = build_server(servicer, host, port, reuse_port=multi)
    server.start()
    if ready_q is not None:
        ready_q.put((replica, bound))
    from ..runtime.metrics import start_metrics_server

    mport = start_metrics_server() if replica == 0 else None
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
    if mdns is not None and mdns.enabled and replica == 0:
        zc, info = setup_mdns(bound, mdns)
    # a replica's own signals stop only that replica (a local event); the parent's shared event
    # (stop_event) stops them all
    done = threading.Event() if replica > 0 or stop_event is None else stop_event
    shared = stop_event if replica > 0 else None

    def _stop(signum, frame):
        log.info("signal %s: shutting down", signum)
        done.set()

    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGINT, _stop)
        signal.signal(signal.SIGTERM, _stop)
    while not done.wait(0.5):
        if shared is not None and shared.is_set():
            break
        if replica > 0 and parent_pid is not None and not _pid_alive(parent_pid):   # parent gone
            break
    if rep_stop is not None:
        rep_stop.set()
        for p in reps:
            p.join(timeout=30)
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
    ap.add_argument("--procs", type=int, default=None,
                    help="server replica processes on the one port (default LUMEN_HUB_PROCS or 1)")
    ap.add_argument("--frontends", type=int, default=None,
                    help="front-end processes over one GPU engine per device (default LUMEN_FRONTENDS or 0: "
                         "in-process serving)")
    ap.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    args = ap.parse_args(argv)
    setup_logging(args.log_level)
    try:
        serve(args.config, args.port, mode=mode, procs=args.procs, frontends=args.frontends)
    except SystemExit as e:
        return int(e.code or 0)
    return 0


def main_single(argv=None) -> int:
    return main(argv, mode="single", prog="lumen-service")


if __name__ == "__main__":
    sys.exit(main())
