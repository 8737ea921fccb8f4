"""Token streaming from a VLM engine process (VERDICT r5 missing #1 / ADVICE r5 medium 3).

* the shared-memory channel's streaming slots (csrc/host/shm_channel.cpp lumen_ch_partial /
  lumen_ch_wait_partial): partial records reach the front end while the slot still runs, the final
  result lands after the log, an abandoned stream makes the engine's next append fail;
* a VLM served on an engine behind 2 gRPC front ends (hub/server.py serve_frontends): the
  ``vlm_generate_stream`` chunks arrive while the engine is still generating (first chunk well
  before the last), the streamed text equals the in-process answer, and a generation completes on
  its own slot (services/vlm/backend.py:engine_worker ``solo_kinds``).

Reference behaviour: the reference backend streams tokens from its generator
(/root/reference/packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:358-418).
"""
import json
import multiprocessing as mp
import pickle
import socket
import threading
import time

import numpy as np
import pytest
import yaml

from lumen_amd.parallel.shm_channel import EngineUnavailable, ShmChannel


def test_channel_partials_arrive_before_completion():
    ch = ShmChannel.create("st", ["a"], nslots=2, slot_bytes=1 << 12, result_bytes=1 << 12)
    ch.engine_start()
    log = []

    def eng():
        s = ch.pop_batch(1, wait_ms=2000)[0]
        for i in range(5):
            assert ch.partial(s, pickle.dumps(("tok", i))) == 0
            log.append(("sent", i, time.perf_counter()))
            time.sleep(0.05)
        ch.complete(s, np.asarray([42.0], np.float32))

    t = threading.Thread(target=eng, daemon=True)
    t.start()
    try:
        got = []
        for tag, val in ch.call_stream("a", np.zeros(4, np.int32), timeout=10):
            got.append((tag, pickle.loads(val) if tag == "partial" else val, time.perf_counter()))
        t.join(5)
        assert [g[1] for g in got[:-1]] == [("tok", i) for i in range(5)]
        assert got[-1][0] == "result" and float(got[-1][1][0]) == 42.0
        # partial i reached the front end before partial i + 1 was even produced
        sent = [x[2] for x in log]
        for i in range(4):
            assert got[i][2] < sent[i + 1]
        assert ch.depth() == 0
    finally:
        ch.close()


def test_channel_abandoned_stream_stops_the_producer():
    ch = ShmChannel.create("sa", ["a"], nslots=1, slot_bytes=1 << 12, result_bytes=256)
    ch.engine_start()
    rcs = []
    first = threading.Event()

    def eng():
        s = ch.pop_batch(1, wait_ms=2000)[0]
        for i in range(200):
            rc = ch.partial(s, b"x" * 8)
            rcs.append(rc)
            if i == 0:
                first.set()
            if rc == -2:
                break
            time.sleep(0.01)
        ch.complete(s, np.ones(1, np.float32))

    t = threading.Thread(target=eng, daemon=True)
    t.start()
    try:
        it = ch.call_stream("a", np.zeros(2, np.int32), timeout=10)
        assert next(it)[0] == "partial"
        it.close()                        # the client went away
        t.join(10)
        assert rcs[-1] == -2              # the engine saw the abandonment and stopped
        assert -1 in rcs or len(rcs) < 200
        # the slot was returned: a new call gets it
        def eng2():
            s = ch.pop_batch(1, wait_ms=2000)[0]
            ch.complete(s, np.full(1, 7.0, np.float32))
        t2 = threading.Thread(target=eng2, daemon=True)
        t2.start()
        assert float(ch.call("a", np.zeros(2, np.int32), timeout=5)[0]) == 7.0
        t2.join(5)
        with pytest.raises(EngineUnavailable):   # nobody pops: per-record timeout
            list(ch.call_stream("a", np.zeros(2, np.int32), timeout=0.1))
    finally:
        ch.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def vlm_cache(tmp_path_factory):
    from lumen_amd.models.vlm import write_vlm_model

    c = tmp_path_factory.mktemp("vlmcache")
    write_vlm_model(c / "models" / "fastvlm-tiny", "fastvlm-tiny")
    return c


def _stream(port, payload, meta):
    import grpc

    from lumen_amd.proto import ml_service as pb

    t0 = time.perf_counter()
    out = []
    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        for r in pb.InferenceStub(ch).Infer(iter([pb.InferRequest(correlation_id="s", task="vlm_generate_stream",
                                                                 payload=payload, payload_mime="image/jpeg",
                                                                 meta=meta)]), timeout=300):
            assert not r.HasField("error"), r.error
            out.append((time.perf_counter() - t0, r))
    return out


def test_vlm_engine_streams_tokens_through_two_frontends(tmp_path, vlm_cache, monkeypatch):
    engine_stream_check(tmp_path, vlm_cache, monkeypatch, "cpu", 32)


def engine_stream_check(tmp_path, vlm_cache, monkeypatch, device: str, new_tokens: int):
    """Shared with tests/test_frontends_gpu.py (device cuda:0)."""
    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server, serve_frontends
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.utils.image import encode_jpeg

    port = _free_port()
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(vlm_cache)},
           "deployment": {"mode": "hub", "services": ["vlm"]},
           "server": {"port": port, "host": "127.0.0.1"},
           "services": {"vlm": {"enabled": True, "package": "lumen_vlm",
                                "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                                                "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc."
                                                                 "add_InferenceServicer_to_server"},
                                "backend_settings": {"device": "cuda" if device != "cpu" else "cpu",
                                                     "batch_size": 4},
                                "models": {"general": {"model": "fastvlm-tiny", "runtime": "onnx"}}}}}
    img = encode_jpeg(np.random.default_rng(3).integers(0, 255, (48, 64, 3), dtype=np.uint8))
    meta = {"prompt": "Describe the picture.", "max_new_tokens": str(new_tokens)}
    # in-process reference (same greedy decode)
    app = AppService.from_app_config(config_from_dict(cfg))
    server, rport = build_server(HubRouter(app.services), "127.0.0.1", 0)
    server.start()
    try:
        ref = _stream(rport, img, meta)
    finally:
        server.stop(0)
        app.close()
    ref_final = json.loads(ref[-1][1].result)

    cfg_path = tmp_path / "cfg.yaml"
    cfg_path.write_text(yaml.safe_dump(cfg))
    monkeypatch.setenv("LUMEN_ENGINE_EXCLUDE", "")
    stop = threading.Event()
    ready = mp.get_context("spawn").Queue()
    th = threading.Thread(target=serve_frontends, args=(str(cfg_path), port, 2),
                          kwargs={"stop_event": stop, "ready_q": ready, "devices": [device]})
    th.start()
    try:
        for _ in range(2):
            ready.get(timeout=600)
        _stream(port, img, {"prompt": "warm", "max_new_tokens": "2"})   # engine warm-up
        got = _stream(port, img, meta)
        chunks = [(t, r) for t, r in got if not r.is_final]
        final = got[-1][1]
        assert final.is_final and len(chunks) >= 2, len(chunks)
        d = json.loads(final.result)
        assert d["generated_tokens"] == new_tokens == ref_final["generated_tokens"]
        # the streamed text equals the in-process stream's, chunk for chunk
        assert "".join(r.result.decode() for _, r in chunks) == d["text"] == ref_final["text"]
        assert [r.result for _, r in chunks] == [r.result for _, r in ref[:-1]]
        # chunks arrive while the engine still generates: first chunk well before the end
        t_first, t_total = chunks[0][0], got[-1][0]
        assert t_first < 0.5 * t_total, (t_first, t_total)
        # several concurrent streams through both front ends, each its own slot
        outs = [None] * 4

        def worker(i):
            outs[i] = _stream(port, img, meta)

        ws = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
        for w in ws:
            w.start()
        for w in ws:
            w.join(300)
        for o in outs:
            assert json.loads(o[-1][1].result)["text"] == ref_final["text"]
    finally:
        stop.set()
        th.join(180)
