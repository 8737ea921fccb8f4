"""End to end on the MI355X: the control plane's generated ``light_weight`` configuration
(OCR PP-OCRv5 + general CLIP MobileCLIP2-S2 + face buffalo_l, preset amd_mi355x) with
synthetic (random-init, real-architecture) models -> downloader -> hub AppService ->
in-process gRPC server -> one request per service."""
import json

import grpc
import numpy as np
import pytest

from lumen_amd.utils.image import encode_jpeg

pytestmark = pytest.mark.gpu


def test_generated_light_weight_config_serves_on_gpu(tmp_path, monkeypatch):
    from lumen_amd.app import presets as P
    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server
    from lumen_amd.proto import ml_service as pb
    from lumen_amd.resources.config import Region
    from lumen_amd.resources.downloader import Downloader

    monkeypatch.setenv("LUMEN_SYNTHETIC", "1")
    c = P.Config(str(tmp_path), P.get_preset("amd_mi355x").create_config(), Region.other, "lumen-ai", 0)
    cfg = c.light_weight()
    assert set(cfg.enabled_services()) == {"ocr", "clip", "face"}
    results = Downloader(cfg).download_all()
    assert all(r.success for r in results.values()), {k: r.error for k, r in results.items()}
    app = AppService.from_app_config(cfg)
    server, port = build_server(HubRouter(app.services), "127.0.0.1", 0)
    server.start()
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    stub = pb.InferenceStub(ch)
    img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (360, 480, 3), dtype=np.uint8))

    def call(task, payload=img, mime="image/jpeg", meta=None):
        rs = list(stub.Infer(iter([pb.InferRequest(correlation_id=task, task=task, payload=payload,
                                                   payload_mime=mime, meta=meta or {})]), timeout=120))
        assert len(rs) == 1 and not rs[0].HasField("error"), rs[0].error
        return rs[0]

    try:
        r = call("clip_image_embed")
        body = json.loads(r.result)
        vec = np.asarray(body["vector"] if "vector" in body else body["embedding"], np.float32)
        assert vec.shape == (512,) and abs(float(np.linalg.norm(vec)) - 1) < 1e-2     # MobileCLIP2-S2: 512-d
        call("clip_text_embed", b"a photo of a cat", "text/plain")
        call("ocr")
        call("face_detect")
    finally:
        ch.close()
        server.stop(0)
        app.close()
