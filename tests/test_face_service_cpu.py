"""GeneralFaceService on the CPU reference path (synthetic tiny SCRFD + IResNet pack)."""
import json

import grpc
import numpy as np
import pytest

from lumen_amd.hub.router import HubRouter
from lumen_amd.hub.server import build_server
from lumen_amd.models.face import write_face_model
from lumen_amd.proto import ml_service as pb
from lumen_amd.resources.validator import config_from_dict
from lumen_amd.services.face import GeneralFaceService
from lumen_amd.services.face.backend import crop_minv, letterbox_geom
from lumen_amd.utils.image import encode_jpeg


def _svc_cfg(cache):
    return {
        "metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(cache)},
        "deployment": {"mode": "single", "service": "face"},
        "server": {"port": 50552, "host": "127.0.0.1"},
        "services": {"face": {"enabled": True, "package": "lumen_face",
                              "import_info": {"registry_class": "lumen_face.general_face.GeneralFaceService",
                                              "add_to_server": "lumen_face.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                              "backend_settings": {"device": "cpu"},
                              "models": {"general": {"model": "buffalo_tiny", "runtime": "onnx"}}}},
    }


@pytest.fixture(scope="module")
def face(tmp_path_factory):
    cache = tmp_path_factory.mktemp("cache")
    write_face_model(cache / "models" / "buffalo_tiny", "buffalo_tiny")
    cfg = config_from_dict(_svc_cfg(cache))
    svc = GeneralFaceService.from_config(cfg.services["face"], cache)
    svc.initialize()
    yield svc
    svc.close()


def _img(h=96, w=160, seed=0):
    return encode_jpeg(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


LOW = {"detection_confidence_threshold": "0.0", "face_size_min": "0", "nms_threshold": "0.3"}


def test_detect(face):
    res, mime, meta = face.handle("face_detect", _img(), "image/jpeg", LOW)
    d = json.loads(res)
    assert mime == "application/json;schema=face_v1"
    assert d["count"] == len(d["faces"]) == int(meta["face_count"]) > 0
    for f in d["faces"]:
        x1, y1, x2, y2 = f["bbox"]
        assert 0 <= x1 <= x2 <= 160 and 0 <= y1 <= y2 <= 96
        assert 0.0 <= f["confidence"] <= 1.0 and len(f["landmarks"]) == 10
    confs = [f["confidence"] for f in d["faces"]]
    assert confs == sorted(confs, reverse=True)
    # default thresholds: random-init logits are biased low -> no faces
    res, _, meta = face.handle("face_detect", _img(), "image/jpeg", {})
    assert json.loads(res)["count"] == 0 and meta["face_count"] == "0"


def test_embed_and_detect_embed(face):
    res, mime, meta = face.handle("face_embed", _img(112, 112, 3), "image/jpeg", {})
    d = json.loads(res)
    assert mime.endswith("embedding_v1") and d["dim"] == 64 and abs(np.linalg.norm(d["vector"]) - 1) < 1e-3
    lm = json.dumps([{"x": 40, "y": 50}, {"x": 72, "y": 50}, {"x": 56, "y": 70}, {"x": 42, "y": 90},
                     {"x": 70, "y": 90}])
    d2 = json.loads(face.handle("face_embed", _img(112, 112, 3), "image/jpeg", {"landmarks": lm})[0])
    assert d2["dim"] == 64 and d2["vector"] != d["vector"]
    res, _, meta = face.handle("face_detect_and_embed", _img(), "image/jpeg", dict(LOW, max_faces="3"))
    d = json.loads(res)
    assert d["count"] == 3 and all(len(f["embedding"]) == 64 for f in d["faces"])


def test_grpc_unknown_task_is_internal(face):
    router = HubRouter([face])
    server, port = build_server(router, "127.0.0.1", 0)
    server.start()
    try:
        stub = pb.InferenceStub(grpc.insecure_channel(f"127.0.0.1:{port}"))
        r = list(stub.Infer(iter([pb.InferRequest(correlation_id="x", task="face_detect", payload=_img(),
                                                  payload_mime="image/jpeg", meta=LOW)])))[0]
        assert not r.HasField("error") and "processing_time_ms" in r.meta
        assert set(face.registry.list_task_names()) == {"face_detect", "face_embed", "face_detect_and_embed"}
        r = list(face.Infer(iter([pb.InferRequest(correlation_id="y", task="nope", payload=b"x")]), None))[0]
        assert r.error.code == pb.ERROR_CODE_INTERNAL
        cap = face.build_capability()
        assert cap.service_name == "face-general" and cap.extra["face_embedding_dim"] == "64"
    finally:
        server.stop(0)


def test_geometry_helpers():
    g, s = letterbox_geom(480, 640, 0, 640)
    assert (g.dw, g.dh) == (640, 480) and s == 1.0
    g, s = letterbox_geom(1000, 500, 0, 640)
    assert (g.dw, g.dh) == (320, 640) and abs(s - 0.64) < 1e-9
    m = crop_minv((10, 20, 122, 132), 112)
    assert np.allclose(m[:2, :2], np.eye(2)) and np.allclose(m[:2, 2], [10, 20])
