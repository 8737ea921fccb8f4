"""Serving-path benchmark: the real gRPC hub, end to end.

Starts a hub in this process on 127.0.0.1:<free port> with ONE service (synthetic,
random-init model of the named architecture written into a temp cache by the downloader),
then drives it with C concurrent gRPC clients.  Each client thread owns a channel and sends
requests back to back, one ``Infer`` stream per request carrying one JPEG (the reference's
client pattern: ``src/lumen/server.py:232-235`` serves them on a 10-thread pool, batch 1).
Everything the service does is inside the measured latency: gRPC transport, chunk
reassembly, JPEG decode, the dynamic batcher (``LUMEN_MAX_BATCH`` / ``LUMEN_MAX_WAIT_MS``),
the DP worker pool and its shared-memory rings (``--dp``), the GPU kernels and the JSON
response.  Reports images/s over the timed window and per-request p50 / p99 latency.

    # BASELINE config 1: CPU ViT-B/32 single-image latency through the service
    python tools/serve_bench.py --service clip --model CLIP-ViT-B-32 --device cpu --clients 1 --seconds 20
    # CLIP ViT-L/14 serving on one GPU, 64 concurrent clients
    python tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda --clients 64
    # face detect + embed (SCRFD-10G + IResNet-100) through the service
    python tools/serve_bench.py --service face --model antelopev2 --device cuda --clients 32
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TASKS = {"clip": "clip_image_embed", "face": "face_detect_and_embed", "ocr": "ocr"}
REGISTRY = {"clip": ("lumen_clip", "lumen_clip.general_clip.GeneralCLIPService"),
            "face": ("lumen_face", "lumen_face.general_face.GeneralFaceService"),
            "ocr": ("lumen_ocr", "lumen_ocr.general_ocr.GeneralOcrService")}


def _config(service: str, model: str, device: str, batch: int, cache: str, runtime: str):
    from lumen_amd.resources.config import LumenConfig

    pkg, reg = REGISTRY[service]
    mc = {"model": model, "runtime": runtime}
    if service == "clip":
        mc["dataset"] = "ImageNet_1k"
    d = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": cache},
         "deployment": {"mode": "hub", "services": [service]},
         "server": {"port": 50051, "host": "127.0.0.1"},
         "services": {service: {"enabled": True, "package": pkg,
                                "import_info": {"registry_class": reg,
                                                "add_to_server": f"{pkg}.proto.ml_service_pb2_grpc."
                                                                 "add_InferenceServicer_to_server"},
                                "backend_settings": {"device": device, "batch_size": batch},
                                "models": {"general": mc}}}}
    return LumenConfig.model_validate(d)


def _images(n: int, side: int, kind: str, seed: int = 0) -> list[bytes]:
    from lumen_amd.utils.image import encode_jpeg

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        if kind == "noise":
            a = rng.integers(0, 256, (side, side * 4 // 3, 3), dtype=np.uint8)
        else:   # photo-like: smooth gradients + a few blobs (compresses like a real photo)
            h, w = side, side * 4 // 3
            y, x = np.mgrid[0:h, 0:w].astype(np.float32)
            a = np.stack([(x / w * 255 + i * 7) % 256, (y / h * 255 + i * 13) % 256,
                          ((x + y) / (h + w) * 255) % 256], -1)
            for _ in range(6):
                cy, cx, r = rng.integers(0, h), rng.integers(0, w), rng.integers(h // 16, h // 4)
                m = (y - cy) ** 2 + (x - cx) ** 2 < r * r
                a[m] = rng.integers(0, 256, 3)
            a = a.astype(np.uint8)
        out.append(encode_jpeg(a))
    return out


def _client_proc(plan_q, res_q, task: str, imgs: list, nthreads: int, pid: int, per_stream: int = 1) -> None:
    """One client process: ``nthreads`` threads, each with its own channel, sending one-image
    ``Infer`` streams back to back; requests that start and finish inside [t_on, t_off] count."""
    import grpc

    from lumen_amd.proto import ml_service as pb

    port, t_on, t_off = plan_q.get()
    lock = threading.Lock()
    acc = {"lat": [], "errors": 0, "n": 0, "meta": {}}

    def run(ci: int):
        # a connection per simulated client, as distinct clients have: gRPC otherwise shares one subchannel
        # (one TCP connection) among a process's channels to a target, and SO_REUSEPORT then spreads only
        # 6 connections over the front ends (measured: 3 of 8 front ends at 100 % CPU, 5 at 15 %)
        ch = grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_send_message_length", 64 << 20),
                                                                ("grpc.max_receive_message_length", 64 << 20),
                                                                ("grpc.use_local_subchannel_pool", 1)])
        stub = pb.InferenceStub(ch)
        k = ci
        try:
            while time.time() < t_off:
                reqs = []
                for _ in range(per_stream):
                    reqs.append(pb.InferRequest(correlation_id=f"{pid}-{ci}-{k}", task=task,
                                                payload=imgs[k % len(imgs)], payload_mime="image/jpeg"))
                    k += 1
                t_w, t = time.time(), time.perf_counter()
                rs = list(stub.Infer(iter(reqs), timeout=300))
                dt = time.perf_counter() - t
                ok = len(rs) == per_stream and not any(r.HasField("error") for r in rs)
                with lock:
                    if not ok:
                        acc["errors"] += 1
                    elif t_w >= t_on and t_w + dt <= t_off:
                        acc["lat"].append(dt)
                        acc["n"] += per_stream
                        for key, v in rs[0].meta.items():      # server-side stage times of this request
                            if key.startswith("t_") or key in ("duration_ms", "batch_size"):
                                try:
                                    acc["meta"].setdefault(key, []).append(float(v))
                                except ValueError:
                                    pass
        finally:
            ch.close()

    ths = [threading.Thread(target=run, args=(i,), daemon=True) for i in range(nthreads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    res_q.put(acc)


def _client_proc_aio(plan_q, res_q, task: str, imgs: list, nthreads: int, pid: int, per_stream: int = 1) -> None:
    """--aio form of :func:`_client_proc`: the clients on one grpc.aio event loop (a channel per 16
    clients).  Measured no cheaper per request than the threaded sync stubs (8 aio processes 2346
    vs 12 sync 2891 img/s against 10 front ends, profiles/r4_serve_fe_v1.txt)."""
    import asyncio

    import grpc

    from lumen_amd.proto import ml_service as pb

    port, t_on, t_off = plan_q.get()
    acc = {"lat": [], "errors": 0, "n": 0, "meta": {}}
    opts = [("grpc.max_send_message_length", 64 << 20), ("grpc.max_receive_message_length", 64 << 20)]

    async def one(stub, ci: int):
        k = ci
        while time.time() < t_off:
            reqs = []
            for _ in range(per_stream):
                reqs.append(pb.InferRequest(correlation_id=f"{pid}-{ci}-{k}", task=task,
                                            payload=imgs[k % len(imgs)], payload_mime="image/jpeg"))
                k += 1
            t_w, t = time.time(), time.perf_counter()
            try:
                rs = [r async for r in stub.Infer(iter(reqs), timeout=300)]
            except grpc.aio.AioRpcError:
                rs = []
            dt = time.perf_counter() - t
            ok = len(rs) == per_stream and not any(r.HasField("error") for r in rs)
            if not ok:
                acc["errors"] += 1
            elif t_w >= t_on and t_w + dt <= t_off:
                acc["lat"].append(dt)
                acc["n"] += per_stream
                for key, v in rs[0].meta.items():      # server-side stage times of this request
                    if key.startswith("t_") or key in ("duration_ms", "batch_size"):
                        try:
                            acc["meta"].setdefault(key, []).append(float(v))
                        except ValueError:
                            pass

    async def run():
        chans = [grpc.aio.insecure_channel(f"127.0.0.1:{port}", options=opts)
                 for _ in range(max(1, -(-nthreads // 16)))]
        stubs = [pb.InferenceStub(c) for c in chans]
        await asyncio.gather(*(one(stubs[i % len(stubs)], i) for i in range(nthreads)))
        for c in chans:
            await c.close()

    asyncio.run(run())
    res_q.put(acc)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--service", choices=sorted(TASKS), default="clip")
    ap.add_argument("--model", default="CLIP-ViT-L-14")
    ap.add_argument("--runtime", default="torch")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dp", type=int, default=1, help="DP worker processes (LUMEN_DP_SIZE); 1 = in-process")
    ap.add_argument("--batch", type=int, default=128, help="backend_settings.batch_size (dynamic batcher cap)")
    ap.add_argument("--max-wait-ms", type=float, default=None, help="LUMEN_MAX_WAIT_MS")
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=20.0, help="timed window after the warm-up")
    ap.add_argument("--warmup", type=float, default=5.0)
    ap.add_argument("--image-side", type=int, default=384, help="JPEG height (width = 4/3 height)")
    ap.add_argument("--image-kind", choices=["photo", "noise"], default="photo")
    ap.add_argument("--server-threads", type=int, default=None)
    ap.add_argument("--client-procs", type=int, default=4, help="client processes (threads spread over them)")
    ap.add_argument("--procs", type=int, default=1, help="hub replica processes on one port (LUMEN_HUB_PROCS)")
    ap.add_argument("--frontends", type=int, default=0,
                    help="front-end processes over one GPU engine per device (LUMEN_FRONTENDS); 0 = in-process")
    ap.add_argument("--aio", action="store_true", help="grpc.aio client processes instead of threaded sync stubs")
    ap.add_argument("--per-stream", type=int, default=1,
                    help="images per Infer stream (the service handles a stream's requests concurrently); "
                         "latency is then per stream")
    args = ap.parse_args()

    os.environ["LUMEN_SYNTHETIC"] = "1"
    if args.dp > 1:
        os.environ["LUMEN_DP_SIZE"] = str(args.dp)
    if args.max_wait_ms is not None:
        os.environ["LUMEN_MAX_WAIT_MS"] = str(args.max_wait_ms)
    os.environ.setdefault("LUMEN_MAX_BATCH", str(args.batch))

    import grpc

    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server
    from lumen_amd.proto import ml_service as pb
    from lumen_amd.resources.downloader import Downloader

    # client processes first, before this process touches the GPU (they only speak gRPC): remote-like
    # clients that do not share the server's GIL
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    nproc = max(1, min(args.client_procs, args.clients))
    plan_q, res_q = ctx.Queue(), ctx.Queue()
    task = TASKS[args.service]
    imgs = _images(16, args.image_side, args.image_kind)
    procs = [ctx.Process(target=_client_proc_aio if args.aio else _client_proc, args=(plan_q, res_q, task, imgs, args.clients * (i + 1) // nproc -
                                                    args.clients * i // nproc, i, args.per_stream), daemon=True)
             for i in range(nproc)]
    for pr in procs:
        pr.start()

    cache = tempfile.mkdtemp(prefix="lumen_serve_bench_")
    cfg = _config(args.service, args.model, args.device, args.batch, cache, args.runtime)
    t0 = time.perf_counter()
    res = Downloader(cfg).download_all()
    assert all(r.success for r in res.values()), {k: r.error for k, r in res.items()}
    reps, rep_stop = [], None
    fe_thread = fe_stop = None
    if args.frontends > 0:
        # engine / front-end topology (parallel/engine.py): one GPU engine process per device + K
        # gRPC front-end processes on one port; this process only supervises and drives clients
        import socket

        from lumen_amd.hub.server import serve_frontends

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cfg_path = os.path.join(cache, "lumen-config.json")
        d = cfg.model_dump(mode="json", exclude_none=True)
        d["server"]["port"] = port
        with open(cfg_path, "w") as f:
            json.dump(d, f)
        ready = ctx.Queue()
        fe_stop = threading.Event()
        fe_thread = threading.Thread(target=serve_frontends, args=(cfg_path, port, args.frontends),
                                     kwargs={"stop_event": fe_stop, "ready_q": ready}, daemon=True)
        fe_thread.start()
        for _ in range(args.frontends):
            ready.get(timeout=900)
        app = server = None
    elif args.procs > 1:
        # hub replica processes on one port (hub/server.py start_replicas, SO_REUSEPORT); this process
        # only drives the clients
        import socket

        from lumen_amd.hub.server import start_replicas

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cfg_path = os.path.join(cache, "lumen-config.json")
        d = cfg.model_dump(mode="json", exclude_none=True)
        d["server"]["port"] = port
        with open(cfg_path, "w") as f:
            json.dump(d, f)
        ready = ctx.Queue()
        reps, rep_stop = start_replicas(cfg_path, port, args.procs, ready_q=ready)
        for _ in reps:
            ready.get(timeout=600)
        app = server = None
    else:
        app = AppService.from_app_config(cfg)
        threads = args.server_threads or max(16, args.clients + 4)
        server, port = build_server(HubRouter(app.services), "127.0.0.1", 0, max_workers=threads)
        server.start()
    load_s = time.perf_counter() - t0
    t_on = time.time() + args.warmup
    t_off = t_on + args.seconds
    for _ in procs:
        plan_q.put((port, t_on, t_off))
    lat, errors, n, smeta = [], 0, 0, {}
    for _ in procs:
        r = res_q.get(timeout=args.warmup + args.seconds + 600)
        lat += r["lat"]
        errors += r["errors"]
        n += r["n"]
        for k, v in r["meta"].items():
            smeta.setdefault(k, []).extend(v)
    for pr in procs:
        pr.join(timeout=60)
    el = args.seconds
    if server is not None:
        server.stop(0)
        app.close()
    if fe_stop is not None:
        fe_stop.set()
        fe_thread.join(timeout=120)
    if rep_stop is not None:
        rep_stop.set()
        for pr in reps:
            pr.join(timeout=60)
    la = np.asarray(lat) * 1e3 if lat else np.zeros(1)
    out = {"metric": f"serving {task} images/s", "value": round(n / el, 2), "unit": "images/s",
           "client_processes": nproc,
           "p50_ms": round(float(np.percentile(la, 50)), 2), "p99_ms": round(float(np.percentile(la, 99)), 2),
           "mean_ms": round(float(la.mean()), 2), "requests": n, "seconds": round(el, 2), "errors": errors,
           "clients": args.clients, "service": args.service, "model": args.model, "device": args.device,
           "dp_workers": args.dp, "hub_processes": args.procs, "frontends": args.frontends, "images_per_stream": args.per_stream, "batch_cap": args.batch, "max_wait_ms": os.environ.get("LUMEN_MAX_WAIT_MS"),
           "image": f"{args.image_kind} JPEG {args.image_side * 4 // 3}x{args.image_side}, "
                    f"{int(np.mean([len(b) for b in imgs]) / 1024)} KiB mean",
           "load_s": round(load_s, 1),
           "server_stage_ms_p50": {k: round(float(np.median(v)), 2) for k, v in sorted(smeta.items())},
           "data": "synthetic (random-init weights of the named architecture, generated JPEGs)",
           "path": ("gRPC Infer stream -> front-end process (service, decode, batcher) -> shm channel -> "
                    "GPU engine process (cross-front-end batch)") if args.frontends > 0 else
                   "gRPC Infer stream -> hub router -> service -> dynamic batcher -> "
                   + ("GPU worker pool (shm rings)" if args.dp > 1 else "in-process backend")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
