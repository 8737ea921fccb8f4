"""A hub.example-shaped config (SmartCLIP = general CLIP + BioCLIP, face, OCR, VLM; reference
/root/reference/src/lumen/server.py:232-235 serves all of them from one process) through the engine
/ front-end topology with 4 front ends (hub/server.py:serve_frontends):

* SmartCLIP's two towers share one engine (parallel.engine.multi_worker, ``general:`` / ``bio:``
  kinds), BioCLIP's TreeOfLife bank held by the engine and queried by broadcast;
* face and OCR batches run on the engine;
* the VLM is excluded from the engines (``LUMEN_ENGINE_EXCLUDE=vlm``, what a tensor-parallel VLM
  does by itself) and served by the parent, the front ends proxying its tasks (hub/proxy.py) --
  the mixed topology instead of the r4 all-or-nothing fallback;

every task answers like the in-process hub.  A second test runs the VLM itself on an engine
(services/vlm/backend.py:engine_worker)."""
import json
import multiprocessing as mp
import socket
import threading

import numpy as np
import pytest
import yaml

from lumen_amd.utils.image import encode_jpeg


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _svc(registry, models, device="cpu", batch=4):
    pkg = registry.split(".")[0]
    return {"enabled": True, "package": pkg,
            "import_info": {"registry_class": registry,
                            "add_to_server": f"{pkg}.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
            "backend_settings": {"device": device, "batch_size": batch}, "models": models}


def _config(cache, port, services):
    return {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(cache)},
            "deployment": {"mode": "hub", "services": list(services)},
            "server": {"port": port, "host": "127.0.0.1"}, "services": services}


ALL = {
    "clip": ("lumen_clip.unified_smartclip.SmartCLIPService",
             {"general": {"model": "clip-tiny", "runtime": "torch", "dataset": "ImageNet_1k"},
              "bioclip": {"model": "bioclip-tiny", "runtime": "torch", "dataset": "TreeOfLife-10M"}}),
    "face": ("lumen_face.general_face.GeneralFaceService", {"general": {"model": "buffalo_tiny", "runtime": "onnx"}}),
    "ocr": ("lumen_ocr.general_ocr.GeneralOcrService", {"general": {"model": "ppocr-tiny", "runtime": "onnx"}}),
    "vlm": ("lumen_vlm.fastvlm.GeneralFastVLMService", {"general": {"model": "fastvlm-tiny", "runtime": "onnx"}}),
}


@pytest.fixture(scope="module")
def cache(tmp_path_factory):
    from lumen_amd.models.face import write_face_model
    from lumen_amd.models.ocr import write_ocr_model
    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.resources.synthetic import write_clip_model

    c = tmp_path_factory.mktemp("cache")
    write_clip_model(c / "models" / "clip-tiny", "clip-tiny", preset="tiny", dataset="ImageNet_1k", n_labels=40)
    write_clip_model(c / "models" / "bioclip-tiny", "bioclip-tiny", preset="tiny", dataset="TreeOfLife-10M",
                     n_labels=60, bio=True)
    write_face_model(c / "models" / "buffalo_tiny", "buffalo_tiny")
    write_ocr_model(c / "models" / "ppocr-tiny", "ppocr-tiny")
    write_vlm_model(c / "models" / "fastvlm-tiny", "fastvlm-tiny")
    return c


def _img(seed, h=64, w=80):
    return encode_jpeg(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


LOW = {"detection_confidence_threshold": "0.0", "face_size_min": "0", "nms_threshold": "0.3", "max_faces": "3"}
REQS = [("smartclip_image_embed", _img(1), "image/jpeg", {}),
        ("smartclip_text_embed", b"a cat", "text/plain", {}),
        ("smartclip_classify", _img(2), "image/jpeg", {"topk": "3"}),
        ("smartclip_bioclassify", _img(3), "image/jpeg", {"topk": "4"}),
        ("face_detect_and_embed", _img(4, 96, 128), "image/jpeg", LOW),
        ("ocr", _img(5, 96, 160), "image/jpeg", {}),
        ("vlm_generate", _img(6), "image/jpeg", {"prompt": "Describe.", "max_new_tokens": "5"}),
        ("vlm_generate_stream", _img(7), "image/jpeg", {"prompt": "Hi.", "max_new_tokens": "4"})]


def _call(port, task, payload, mime, meta):
    import grpc

    from lumen_amd.proto import ml_service as pb

    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        rs = list(pb.InferenceStub(ch).Infer(iter([pb.InferRequest(correlation_id="x", task=task, payload=payload,
                                                                   payload_mime=mime, meta=meta)]), timeout=300))
    assert len(rs) == 1 and not rs[0].HasField("error"), (task, rs[0].error)
    return json.loads(rs[0].result)


def _cos(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def _same(task, got, ref, score_atol=1e-4, box_atol=1e-3, emb_cos=0.9999):
    if "vector" in ref:
        assert _cos(got["vector"], ref["vector"]) > 0.9999, task
    elif "labels" in ref:
        assert [x["label"] for x in got["labels"]] == [x["label"] for x in ref["labels"]], task
        np.testing.assert_allclose([x["score"] for x in got["labels"]], [x["score"] for x in ref["labels"]],
                                   atol=score_atol)
    elif "faces" in ref:
        assert got["count"] == ref["count"] > 0, task
        for fa, fb in zip(got["faces"], ref["faces"]):
            np.testing.assert_allclose(fa["bbox"], fb["bbox"], atol=box_atol)
            assert _cos(fa["embedding"], fb["embedding"]) > emb_cos
    elif "items" in ref:
        assert got["count"] == ref["count"], task
        assert [i["text"] for i in got["items"]] == [i["text"] for i in ref["items"]], task
    else:                                      # text generation (greedy): identical text
        assert got["text"] == ref["text"] and got["finish_reason"] == ref["finish_reason"], task


def _reference(cfg_dict, tasks=None):
    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server
    from lumen_amd.resources.validator import config_from_dict

    app = AppService.from_app_config(config_from_dict(cfg_dict))
    server, rport = build_server(HubRouter(app.services), "127.0.0.1", 0)
    server.start()
    try:
        return {t: _call(rport, t, p, m, meta) for t, p, m, meta in REQS if tasks is None or t in tasks}, app
    finally:
        server.stop(0)


def _serve(tmp_path, cfg_dict, nfe, tasks, monkeypatch, exclude="", devices=("cpu",)):
    from lumen_amd.hub.server import serve_frontends

    cfg_path = tmp_path / "cfg.yaml"
    cfg_path.write_text(yaml.safe_dump(cfg_dict))
    monkeypatch.setenv("LUMEN_ENGINE_EXCLUDE", exclude)
    stop = threading.Event()
    ready = mp.get_context("spawn").Queue()
    started = []
    th = threading.Thread(target=lambda: started.append(serve_frontends(
        str(cfg_path), cfg_dict["server"]["port"], nfe, stop_event=stop, ready_q=ready, devices=list(devices))))
    th.start()
    try:
        for _ in range(nfe):
            ready.get(timeout=600)
        out = {}

        def worker(t, p, m, meta):
            out[t] = _call(cfg_dict["server"]["port"], t, p, m, meta)

        ths = [threading.Thread(target=worker, args=r) for r in REQS if r[0] in tasks]
        for t in ths:
            t.start()
        for t in ths:
            t.join(300)
        return out
    finally:
        stop.set()
        th.join(180)
        assert started == [True]


def test_hub_example_shaped_config_through_four_frontends(tmp_path, cache, monkeypatch):
    port = _free_port()
    cfg = _config(cache, port, {k: _svc(*v) for k, v in ALL.items()})
    ref, app = _reference(cfg)
    try:
        # the engine spec of every engine-capable service, SmartCLIP's as one multi-model engine
        specs = {n: s.engine_spec() for n, s in zip(app.names, app.services)}
        assert specs["clip"][0] == "lumen_amd.parallel.engine:multi_worker"
        assert set(specs["clip"][1]["parts"]) == {"general", "bio"}
        assert specs["clip"][1]["parts"]["bio"][1]["shard_bank"] is True
        assert all(specs[n] is not None for n in ("face", "ocr", "vlm"))
    finally:
        app.close()
    got = _serve(tmp_path, cfg, 4, [r[0] for r in REQS], monkeypatch, exclude="vlm")
    assert set(got) == {r[0] for r in REQS}
    for t, _, _, _ in REQS:
        _same(t, got[t], ref[t])


def test_vlm_on_engine(tmp_path, cache, monkeypatch):
    port = _free_port()
    cfg = _config(cache, port, {"vlm": _svc(*ALL["vlm"])})
    tasks = ["vlm_generate", "vlm_generate_stream"]
    ref, app = _reference(cfg, tasks)
    app.close()
    got = _serve(tmp_path, cfg, 1, tasks, monkeypatch)
    for t in tasks:
        _same(t, got[t], ref[t])
