"""OCR models / service on the MI355X path vs the fp32 CPU reference."""
import json

import numpy as np
import pytest
import torch

from lumen_amd.models.ocr import DBNET_PRESETS, REC_PRESETS, DBNet, SVTRRecognizer, write_ocr_model
from lumen_amd.resources.validator import config_from_dict
from lumen_amd.services.ocr import GeneralOcrService
from lumen_amd.utils.image import encode_png

pytestmark = pytest.mark.gpu


def test_dbnet_mobile_full_size():
    g = torch.Generator().manual_seed(0)
    m = DBNet(DBNET_PRESETS["mobile"])
    m.random_init(g)
    x = torch.randn(2, 320, 480, 8, generator=g)
    x[..., 3:] = 0
    ref = m(x)
    got = m.to("cuda")(x.to("cuda", torch.bfloat16)).cpu()
    assert got.shape == ref.shape == (2, 320, 480)
    assert (got - ref).abs().max().item() < 0.05
    assert ((got > 0.3) == (ref > 0.3)).float().mean().item() > 0.98


@pytest.mark.parametrize("C", [16, 32])
def test_db_head_up_fused_vs_fp32(C):
    """csrc/conv.hip db_head_up (up1 + ReLU + shuffle + up2 + sigmoid in one MFMA pass) against the
    fp32 CPU path of the same head tail; 7 x 9 pixels per image: a partial 16-pixel group and groups
    that span image rows and images."""
    from lumen_amd.models.ocr import ConvT2
    from lumen_amd.ops import cnn

    g = torch.Generator().manual_seed(C)
    up1 = ConvT2(C, C, act="relu")
    up2 = ConvT2(C, 1, act="sigmoid", out_dtype=torch.float32)
    up1.random_init(g)
    up2.random_init(g)
    up1.g.b.data[:4 * C] = torch.randn(4 * C, generator=g) * 0.1
    up2.g.b.data[:4] = torch.randn(4, generator=g) * 0.1
    N, H4, W4 = 3, 7, 9
    h = torch.randn(N, H4, W4, C, generator=g).bfloat16()
    y = up2.gemm(up1(h.float()))
    ref = y.view(N, 2 * H4, 2 * W4, 2, 2).permute(0, 1, 3, 2, 4).reshape(N, 4 * H4, 4 * W4).float()
    dev = torch.device("cuda")
    w1 = up1.g.w[:4 * C, :C].to(dev, torch.bfloat16).contiguous()
    b1 = up1.g.b[:4 * C].to(dev, torch.float32).contiguous()
    w2p = cnn.db_head_pack_up2(up2.g.w[:4, :C]).to(dev)
    b2 = up2.g.b[:4].to(dev, torch.float32).contiguous()
    got = cnn.db_head_up(h.to(dev), w1, b1, w2p, b2).cpu()
    assert got.shape == ref.shape
    # bf16 up1 output (as in the unfused GPU path) vs fp32: sigmoid outputs agree to ~1e-2
    assert (got - ref).abs().max().item() < 2e-2


def test_svtr_mobile():
    g = torch.Generator().manual_seed(1)
    m = SVTRRecognizer(REC_PRESETS["mobile"])
    m.random_init(g)
    x = torch.randn(6, 48, 320, 8, generator=g)
    x[..., 3:] = 0
    vw = [320, 300, 200, 96, 64, 33]
    ref = m(x, valid_w=vw)
    got = m.to("cuda")(x.to("cuda", torch.bfloat16), valid_w=vw).cpu()
    C = REC_PRESETS["mobile"].num_classes
    a, b = got[..., :C].flatten(0, 1), ref[..., :C].flatten(0, 1)
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert cos.min().item() > 0.99


def _cfg(cache, device):
    return {
        "metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(cache)},
        "deployment": {"mode": "single", "service": "ocr"},
        "server": {"port": 50555, "host": "127.0.0.1"},
        "services": {"ocr": {"enabled": True, "package": "lumen_ocr",
                             "import_info": {"registry_class": "lumen_ocr.general_ocr.GeneralOcrService",
                                             "add_to_server": "lumen_ocr.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                             "backend_settings": {"device": device},
                             "models": {"general": {"model": "ppocr-tiny", "runtime": "onnx"}}}},
    }


def test_ocr_service_gpu_vs_cpu(tmp_path):
    write_ocr_model(tmp_path / "models" / "ppocr-tiny", "ppocr-tiny")
    svcs = {d: GeneralOcrService.from_config(config_from_dict(_cfg(tmp_path, d)).services["ocr"], tmp_path)
            for d in ("cpu", "cuda")}
    try:
        img = encode_png(np.random.default_rng(0).integers(0, 255, (90, 200, 3), dtype=np.uint8))
        meta = {"detection_threshold": "0.0", "ocr.box_thresh": "0.0", "recognition_threshold": "0.0"}
        dc = json.loads(svcs["cpu"].handle("ocr", img, "image/png", meta)[0])
        dg = json.loads(svcs["cuda"].handle("ocr", img, "image/png", meta)[0])
        assert dg["count"] == dc["count"] >= 1
        for a, b in zip(dc["items"], dg["items"]):
            assert np.abs(np.array(a["box"]) - np.array(b["box"])).max() <= 2
            assert abs(a["confidence"] - b["confidence"]) < 0.05
    finally:
        for s in svcs.values():
            s.close()


def test_ocr_engine_device_jpeg_matches_host_decode(tmp_path):
    """The OCR engine's merged batch of encoded images takes the device JPEG path (host entropy
    decode + one GPU reconstruction; detector and crop warps read the device buffer): same boxes and
    texts as the host-decoded arrays; an undecodable payload fails alone."""
    from lumen_amd.services.ocr.backend import InvalidInputError, OcrParams, dp_worker
    from lumen_amd.utils.image import decode_rgb, encode_jpeg

    write_ocr_model(tmp_path / "models" / "ppocr-tiny", "ppocr-tiny")
    svc = GeneralOcrService.from_config(config_from_dict(_cfg(tmp_path, "cuda")).services["ocr"], tmp_path)
    try:
        svc.manager.initialize()
        fn = dp_worker("cuda", svc.manager.resources)
        rng = np.random.default_rng(5)
        jpegs = [encode_jpeg(rng.integers(0, 255, (90 + 8 * k, 200 - 6 * k, 3), dtype=np.uint8)) for k in range(3)]
        p = OcrParams(det_thresh=0.0, box_thresh=0.0, rec_thresh=0.0)
        dev = fn("ocr", [(j, p) for j in jpegs] + [(b"not an image", p)])
        host = fn("ocr", [(decode_rgb(j), p) for j in jpegs])
        assert isinstance(dev[3], InvalidInputError)
        for d, h in zip(dev[:3], host):
            assert len(d) == len(h) >= 1
            for a, b in zip(d, h):
                assert np.abs(np.array(a.box) - np.array(b.box)).max() <= 2
                assert a.text == b.text
    finally:
        svc.close()
