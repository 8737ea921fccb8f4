"""OCR models, crop geometry and GeneralOcrService on the CPU reference path."""
import json

import numpy as np
import pytest
import torch

from lumen_amd.models.ocr import DBNET_PRESETS, REC_PRESETS, DBNet, SVTRRecognizer, write_ocr_model
from lumen_amd.ops import vision
from lumen_amd.proto import ml_service as pb
from lumen_amd.resources.validator import config_from_dict
from lumen_amd.services.ocr import GeneralOcrService
from lumen_amd.services.ocr.backend import crop_map, det_resize_shape, sorted_boxes
from lumen_amd.utils.image import encode_png


def test_det_resize_shape():
    assert det_resize_shape(100, 200, 960) == (96, 192)
    assert det_resize_shape(2000, 1000, 960) == (960, 480)
    assert det_resize_shape(10, 10, 960) == (32, 32)


def test_sorted_boxes_reading_order():
    b = [np.array([[50, 12], [90, 12], [90, 30], [50, 30]]), np.array([[5, 10], [40, 10], [40, 30], [5, 30]]),
         np.array([[5, 60], [40, 60], [40, 80], [5, 80]])]
    out = sorted_boxes(b)
    assert [int(x[0][0]) for x in out] == [5, 50, 5]


def _rgb(h, w, seed=0):
    return np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8)


def _smooth(h, w):
    y, x = np.mgrid[0:h, 0:w]
    return np.stack([(x * 2) % 256, (y * 3) % 256, (x + y) % 256], -1).astype(np.uint8)


def test_crop_map_axis_aligned_and_rotated():
    img = _smooth(80, 120)
    # axis-aligned 60x24 crop at (10, 20): resized to height 48 -> width 120, scale 0.5
    box = np.array([[10, 20], [70, 20], [70, 44], [10, 44]], np.float32)
    minv, rw = crop_map(box, 48)
    assert rw == 120
    src = minv @ np.array([0.0, 0.0, 1.0])
    assert np.allclose(src[:2] / src[2], [10 + 0.25 - 0.5 + 0.0, 20 - 0.25], atol=1e-4)
    # tall crop 10 wide x 40 high -> np.rot90 (CCW) -> 40 x 10 -> height 48 -> width 192
    box = np.array([[30, 5], [40, 5], [40, 45], [30, 45]], np.float32)
    minv, rw = crop_map(box, 48)
    assert rw == 192
    out = vision.warp_batch([img], [0], minv[None], (48, rw), swap_rb=False, scale=1.0, mean=0.0, std=1.0,
                            replicate=True)[0, :, :, :3].float().numpy()
    rot = np.rot90(img[5:45, 30:40]).astype(np.float64)        # [10, 40, 3]
    ys = (np.arange(48) + 0.5) * 10 / 48 - 0.5
    xs = (np.arange(192) + 0.5) * 40 / 192 - 0.5
    y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
    fy, fx = ys - y0, xs - x0
    cy = lambda v: np.clip(v, 0, 9)
    cx = lambda v: np.clip(v, 0, 39)
    ref = ((1 - fy)[:, None, None] * ((1 - fx)[None, :, None] * rot[cy(y0)][:, cx(x0)] + fx[None, :, None] * rot[cy(y0)][:, cx(x0 + 1)])
           + fy[:, None, None] * ((1 - fx)[None, :, None] * rot[cy(y0 + 1)][:, cx(x0)] + fx[None, :, None] * rot[cy(y0 + 1)][:, cx(x0 + 1)]))
    inner = (slice(6, 42), slice(6, 186))
    assert np.abs(out[inner] - np.rint(ref[inner])).max() <= 1.0


def test_models_shapes():
    g = torch.Generator().manual_seed(0)
    d = DBNet(DBNET_PRESETS["tiny"])
    d.random_init(g)
    p = d(torch.randn(2, 64, 96, 8))
    assert p.shape == (2, 64, 96) and float(p.min()) >= 0 and float(p.max()) <= 1
    r = SVTRRecognizer(REC_PRESETS["tiny"])
    r.random_init(g)
    lg = r(torch.randn(3, 48, 96, 8), valid_w=[96, 60, 20])
    assert lg.shape[:2] == (3, 12) and lg.shape[2] >= REC_PRESETS["tiny"].num_classes
    assert float(lg[..., REC_PRESETS["tiny"].num_classes:].max()) < -1e8


def _cfg(cache, device="cpu"):
    return {
        "metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(cache)},
        "deployment": {"mode": "single", "service": "ocr"},
        "server": {"port": 50554, "host": "127.0.0.1"},
        "services": {"ocr": {"enabled": True, "package": "lumen_ocr",
                             "import_info": {"registry_class": "lumen_ocr.general_ocr.GeneralOcrService",
                                             "add_to_server": "lumen_ocr.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                             "backend_settings": {"device": device},
                             "models": {"general": {"model": "ppocr-tiny", "runtime": "onnx"}}}},
    }


@pytest.fixture(scope="module")
def ocr(tmp_path_factory):
    cache = tmp_path_factory.mktemp("cache")
    write_ocr_model(cache / "models" / "ppocr-tiny", "ppocr-tiny")
    cfg = config_from_dict(_cfg(cache))
    svc = GeneralOcrService.from_config(cfg.services["ocr"], cache)
    yield svc
    svc.close()


def test_ocr_service(ocr):
    img = encode_png(_rgb(70, 150))
    # lazy init on first Infer; empty task -> "ocr"
    meta = {"detection_threshold": "0.0", "ocr.box_thresh": "0.0", "recognition_threshold": "0.0"}
    r = list(ocr.Infer(iter([pb.InferRequest(correlation_id="a", payload=img, payload_mime="image/png", meta=meta)]),
                       None))[0]
    assert not r.HasField("error"), r.error
    assert r.result_schema == "ocr_v1" and "duration_ms" in r.meta
    for k in ("t_decode_ms", "t_det_forward_ms", "t_db_post_ms", "t_rec_forward_ms", "t_ctc_ms", "t_queue_ms"):
        assert float(r.meta[k]) >= 0.0, (k, dict(r.meta))
    d = json.loads(r.result)
    assert d["model_id"] == "ppocr-tiny_onnx" and d["count"] == len(d["items"]) >= 1
    for it in d["items"]:
        assert len(it["box"]) == 4 and 0 <= it["confidence"] <= 1
        assert all(0 <= x <= 150 and 0 <= y <= 70 for x, y in it["box"])
    # default thresholds on a blank image -> nothing
    d = json.loads(ocr.handle("ocr", encode_png(np.zeros((40, 40, 3), np.uint8)), "image/png",
                              {"detection_threshold": "0.999"})[0])
    assert d["count"] == 0
    r = list(ocr.Infer(iter([pb.InferRequest(correlation_id="b", task="nope", payload=img)]), None))[0]
    assert r.error.code == pb.ERROR_CODE_INTERNAL
    cap = ocr.build_capability()
    assert cap.service_name == "ocr" and [t.name for t in cap.tasks] == ["ocr"]
