"""Engine / front-end serving topology (parallel/engine.py, parallel/shm_channel.py) on CPU:
several front-end processes share ONE engine's batches through the shared-memory channel,
results come back to the right caller, an engine crash fails only the requests it held and
the supervisor respawns it; the full gRPC hub with 2 front ends over a CPU engine answers like
the in-process hub."""
import json
import multiprocessing as mp
import os
import socket
import threading
import time

import numpy as np
import pytest

from lumen_amd.parallel.engine import EngineSet, RemotePool, attach_frontend, current_remote, remote_scope
from lumen_amd.parallel.shm_channel import ChannelGroup, ShmChannel
from lumen_amd.parallel.worker_pool import WorkerLostError, WorkerTaskError


def echo_engine(device, delay_s: float = 0.0):
    """Engine factory: kind "sum" -> scaled row sums, "slow" -> sleeps, "boom" -> raises."""
    def fn(kind, items):
        if kind == "boom":
            raise ValueError("requested failure")
        if kind == "crash":
            os._exit(3)
        if kind == "slow":      # occupies the batch loop while the front ends queue work
            time.sleep(2.0)
        elif delay_s:
            time.sleep(delay_s)
        return [float(np.asarray(x).sum()) * 2.0 for x in items]
    return fn


def _frontend(specs, q, n, start_ev, ready_q=None):
    attach_frontend(specs)
    with remote_scope("echo"):
        pool = current_remote()
    if ready_q is not None:
        ready_q.put(os.getpid())
    start_ev.wait(60)
    outs = []
    futs = [pool.submit("sum", [np.full(4, i, np.float32), np.full(2, i + 1, np.float32)]) for i in range(n)]
    for i, f in enumerate(futs):
        outs.append((i, f.result(60)))
    q.put((os.getpid(), outs))


def test_channel_round_trip_in_process():
    ch = ShmChannel.create("t", ["a"], nslots=4, slot_bytes=1 << 12, result_bytes=1 << 10)
    stop = threading.Event()

    def eng():
        ch.engine_start()
        while not stop.is_set():
            for s in ch.pop_batch(4, wait_ms=50, linger_us=200):
                _k, arr, meta = ch.request(s)
                ch.complete(s, np.asarray([arr.sum() * meta.get("k", 1)], np.float32))

    t = threading.Thread(target=eng, daemon=True)
    t.start()
    try:
        res = [float(ch.call("a", np.full(8, i, np.int32), meta={"k": 3})[0]) for i in range(20)]
        assert res == [24.0 * i for i in range(20)]
        big = np.zeros(ch.slot_bytes + 1, np.uint8)
        with pytest.raises(ValueError):
            ch.call("a", big)
        assert ch.depth() == 0
    finally:
        stop.set()
        t.join(5)
        ch.close()


def test_abandoned_slots_are_reclaimed():
    """A front end that times out abandons its slot: one abandoned while QUEUED is freed when the
    engine pops it, one abandoned while RUNNING is freed at completion, so timeouts under load
    never drain the slot pool."""
    from lumen_amd.parallel.shm_channel import EngineUnavailable

    ch = ShmChannel.create("ab", ["a"], nslots=2, slot_bytes=1 << 12, result_bytes=1 << 10)
    try:
        ch.engine_start()
        # abandoned while queued (no engine popping): both slots time out
        for _ in range(2):
            with pytest.raises(EngineUnavailable):
                ch.call("a", np.zeros(4, np.int32), timeout=0.05)
        assert ch.depth() == 2
        assert ch.pop_batch(4, wait_ms=10) == []        # the engine frees both instead of running them
        assert ch.depth() == 0
        # abandoned while running: the engine completes after the front end gave up
        popped = []

        def slow_engine():
            while not popped:
                popped.extend(ch.pop_batch(1, wait_ms=50))
            time.sleep(0.3)
            ch.complete(popped[0], np.ones(1, np.float32))

        t = threading.Thread(target=slow_engine, daemon=True)
        t.start()
        with pytest.raises(EngineUnavailable):
            ch.call("a", np.zeros(4, np.int32), timeout=0.1)
        t.join(5)
        assert ch.depth() == 0
        # every slot is usable again
        stop = threading.Event()

        def eng():
            while not stop.is_set():
                for s in ch.pop_batch(2, wait_ms=20):
                    ch.complete(s, np.asarray([7.0], np.float32))

        t = threading.Thread(target=eng, daemon=True)
        t.start()
        for _ in range(6):
            assert float(ch.call("a", np.zeros(2, np.int32), timeout=5)[0]) == 7.0
        stop.set()
        t.join(5)
    finally:
        ch.close()


def test_two_frontends_share_one_engines_batches():
    # one batch loop, 0.3 s per batch: while the first batch runs, both front ends queue theirs
    es = EngineSet({"echo": ("tests.test_frontends_cpu:echo_engine", {"delay_s": 0.3})}, ["cpu"], nslots=32,
                   slot_bytes=1 << 16, result_bytes=1 << 14, threads_per_service=1)
    try:
        ctx = mp.get_context("spawn")
        q, start, ready = ctx.Queue(), ctx.Event(), ctx.Queue()
        ps = [ctx.Process(target=_frontend, args=(es.frontend_specs(), q, 12, start, ready)) for _ in range(2)]
        for p in ps:
            p.start()
        pool = RemotePool(ChannelGroup([ShmChannel.attach(s) for s in es.frontend_specs()["echo"]]))
        for _ in ps:                # both front ends attached (spawned imports can take seconds)
            ready.get(timeout=120)
        blocker = pool.submit("slow", [np.zeros(1, np.float32)])   # the batch loop sleeps 2 s ...
        time.sleep(0.2)
        start.set()                                                 # ... while both front ends queue
        got = [q.get(timeout=120) for _ in ps]
        for p in ps:
            p.join(30)
        blocker.result(30)
        assert len({pid for pid, _ in got}) == 2
        for _pid, outs in got:
            assert [o for _, o in outs] == [[8.0 * i, 4.0 * (i + 1)] for i in range(12)]
        st = pool.submit("__stats__", [None]).result(30)[0]
        assert st["items"] == 49 and st["max_frontends_per_batch"] >= 2 and st["shared_batches"] >= 1
        with pytest.raises(WorkerTaskError, match="requested failure"):
            pool.submit("boom", [1]).result(30)
        pool.close()
    finally:
        es.close()


def test_engine_crash_fails_inflight_and_respawns():
    es = EngineSet({"echo": ("tests.test_frontends_cpu:echo_engine", {})}, ["cpu"], nslots=8,
                   slot_bytes=1 << 14, result_bytes=1 << 12)
    try:
        pool = RemotePool(ChannelGroup([ShmChannel.attach(s) for s in es.frontend_specs()["echo"]]), timeout_s=60)
        assert pool.submit("sum", [np.ones(3)]).result(30) == [6.0]
        with pytest.raises(WorkerLostError):
            pool.submit("crash", [1]).result(60)
        t0 = time.time()
        while True:       # the supervisor respawns the engine on the same channel
            try:
                assert pool.submit("sum", [np.ones(2)]).result(30) == [4.0]
                break
            except WorkerLostError:
                assert time.time() - t0 < 120
                time.sleep(0.5)
        assert es.restarts >= 1
        pool.close()
    finally:
        es.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_grpc_hub_two_frontends_over_cpu_engine(tmp_path):
    import grpc
    import yaml

    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server, serve_frontends
    from lumen_amd.proto import ml_service as pb
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.utils.image import encode_jpeg

    write_clip_model(tmp_path / "models" / "clip-tiny", "clip-tiny", preset="tiny", dataset="ImageNet_1k",
                     n_labels=20)
    port = _free_port()
    d = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(tmp_path)},
         "deployment": {"mode": "hub", "services": ["clip"]},
         "server": {"port": port, "host": "127.0.0.1"},
         "services": {"clip": {"enabled": True, "package": "lumen_clip",
                               "import_info": {"registry_class": "lumen_clip.general_clip.clip_service.GeneralCLIPService",
                                               "add_to_server": "lumen_clip.proto.ml_service_pb2_grpc."
                                                                "add_InferenceServicer_to_server"},
                               "backend_settings": {"device": "cpu", "batch_size": 4},
                               "models": {"general": {"model": "clip-tiny", "runtime": "torch",
                                                      "dataset": "ImageNet_1k"}}}}}
    cfg_path = tmp_path / "cfg.yaml"
    cfg_path.write_text(yaml.safe_dump(d))
    imgs = [encode_jpeg(np.random.default_rng(i).integers(0, 255, (40, 48, 3), dtype=np.uint8)) for i in range(6)]
    # in-process reference
    app = AppService.from_app_config(config_from_dict(d))
    server, rport = build_server(HubRouter(app.services), "127.0.0.1", 0)
    server.start()

    def embed(p, payload, task="clip_image_embed"):
        with grpc.insecure_channel(f"127.0.0.1:{p}") as ch:
            rs = list(pb.InferenceStub(ch).Infer(iter([pb.InferRequest(correlation_id="x", task=task, payload=payload,
                                                                          payload_mime="image/jpeg")]), timeout=120))
        assert len(rs) == 1 and not rs[0].HasField("error"), rs[0].error
        return rs[0]

    ref = [json.loads(embed(rport, b).result)["vector"] for b in imgs]
    ref_cls = json.loads(embed(rport, imgs[0], "clip_classify").result)
    server.stop(0)
    app.close()
    stop = threading.Event()
    ready = mp.get_context("spawn").Queue()
    th = threading.Thread(target=serve_frontends, args=(str(cfg_path), port, 2), kwargs={"stop_event": stop,
                                                                                        "ready_q": ready,
                                                                                        "devices": ["cpu"]})
    th.start()
    try:
        for _ in range(2):
            ready.get(timeout=300)
        out = [None] * len(imgs)

        def worker(i):
            out[i] = json.loads(embed(port, imgs[i]).result)["vector"]

        ts = [threading.Thread(target=worker, args=(i,)) for i in range(len(imgs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        for a, b in zip(out, ref):
            assert np.allclose(a, b, atol=2e-4)
        cls = json.loads(embed(port, imgs[0], "clip_classify").result)
        assert [x["label"] for x in cls["labels"]] == [x["label"] for x in ref_cls["labels"]]
    finally:
        stop.set()
        th.join(120)
