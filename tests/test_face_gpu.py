"""Face models and service on the MI355X path vs the fp32 CPU reference."""
import json

import numpy as np
import pytest
import torch

from lumen_amd.models.face import IRESNET_PRESETS, SCRFD, SCRFD_PRESETS, IResNet, write_face_model
from lumen_amd.resources.validator import config_from_dict
from lumen_amd.services.face import GeneralFaceService
from lumen_amd.utils.image import encode_jpeg

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.float().flatten(1), b.float().flatten(1)
    return torch.nn.functional.cosine_similarity(a, b, dim=1)


def test_iresnet50_full_size():
    g = torch.Generator().manual_seed(0)
    m = IResNet(IRESNET_PRESETS["r50"])
    m.random_init(g)
    x = torch.randn(4, 112, 112, 8, generator=g)
    x[..., 3:] = 0
    ref = m(x)
    got = m.to("cuda")(x.to("cuda", torch.bfloat16)).cpu()
    assert got.shape == (4, 512)
    assert _cos(got, ref).min() > 0.99


def test_scrfd_10g_full_size():
    g = torch.Generator().manual_seed(1)
    m = SCRFD(SCRFD_PRESETS["10g"])
    m.random_init(g)
    x = torch.randn(1, 640, 640, 8, generator=g)
    x[..., 3:] = 0
    ref = m(x)
    got = m.to("cuda")(x.to("cuda", torch.bfloat16))
    for r, o in zip(ref, got):
        assert o.shape == r.shape
        assert _cos(o.cpu(), r).min() > 0.99


def _cfg(cache, device):
    return {
        "metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(cache)},
        "deployment": {"mode": "single", "service": "face"},
        "server": {"port": 50553, "host": "127.0.0.1"},
        "services": {"face": {"enabled": True, "package": "lumen_face",
                              "import_info": {"registry_class": "lumen_face.general_face.GeneralFaceService",
                                              "add_to_server": "lumen_face.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                              "backend_settings": {"device": device},
                              "models": {"general": {"model": "buffalo_tiny", "runtime": "onnx"}}}},
    }


def test_face_service_gpu_vs_cpu(tmp_path):
    write_face_model(tmp_path / "models" / "buffalo_tiny", "buffalo_tiny")
    svcs = {}
    for dev in ("cpu", "cuda"):
        cfg = config_from_dict(_cfg(tmp_path, dev))
        svcs[dev] = GeneralFaceService.from_config(cfg.services["face"], tmp_path)
        svcs[dev].initialize()
    try:
        rng = np.random.default_rng(0)
        img = encode_jpeg(rng.integers(0, 255, (96, 160, 3), dtype=np.uint8))
        face = encode_jpeg(rng.integers(0, 255, (130, 120, 3), dtype=np.uint8))
        lm = json.dumps([{"x": 40, "y": 50}, {"x": 72, "y": 50}, {"x": 56, "y": 70}, {"x": 42, "y": 90},
                         {"x": 70, "y": 90}])
        for meta in ({}, {"landmarks": lm}):
            a = np.array(json.loads(svcs["cpu"].handle("face_embed", face, "image/jpeg", meta)[0])["vector"])
            b = np.array(json.loads(svcs["cuda"].handle("face_embed", face, "image/jpeg", meta)[0])["vector"])
            assert float(a @ b) > 0.98
        low = {"detection_confidence_threshold": "0.0", "face_size_min": "0", "nms_threshold": "0.3"}
        dc = json.loads(svcs["cpu"].handle("face_detect", img, "image/jpeg", low)[0])
        dg = json.loads(svcs["cuda"].handle("face_detect", img, "image/jpeg", low)[0])
        assert dg["count"] > 0 and abs(dg["count"] - dc["count"]) <= max(2, dc["count"] // 5)
        bc, bg = np.array(dc["faces"][0]["bbox"]), np.array(dg["faces"][0]["bbox"])
        assert np.abs(bc - bg).max() < 4.0
        de = json.loads(svcs["cuda"].handle("face_detect_and_embed", img, "image/jpeg", dict(low, max_faces="4"))[0])
        assert de["count"] == 4 and all(abs(np.linalg.norm(f["embedding"]) - 1) < 1e-2 for f in de["faces"])
    finally:
        for s in svcs.values():
            s.close()


def test_reference_alignment_warp_gpu_matches_cpu():
    """LUMEN_FACE_ALIGN=reference geometry (crop sources, constant / replicate borders mixed
    in one batch) gives the same recogniser input on the GPU warp kernel as on the CPU path."""
    import numpy as np
    import torch

    from lumen_amd.services.face.backend import MI355XFaceBackend

    class _Res:
        extra = {"face_align": "reference"}

    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (180, 200, 3)).astype(np.uint8)
    items = [((30.5, 20.2, 150.9, 170.1), [(70, 80), (110, 78), (90, 105), (75, 135), (108, 133)]),
             ((10, 10, 60, 70), None), ((40, 30, 190, 175), [(90, 90), (140, 92), (115, 120), (95, 150), (135, 149)])]
    outs = {}
    for dev in ("cpu", "cuda"):
        b = MI355XFaceBackend(_Res(), device=dev)
        b.device = torch.device(dev)
        srcs, minvs, reps = [], [], []
        for bb, lm in items:
            s, m, r = b._reference_crop(img, lm, bb)
            srcs.append(s)
            minvs.append(m)
            reps.append(r)
        outs[dev] = b.warp_faces(srcs, list(range(len(srcs))), np.stack(minvs), reps)[..., :3].float().cpu()
    d = (outs["cpu"] - outs["cuda"]).abs()
    assert d.max().item() < 3 / 255 and d.mean().item() < 1e-3


def test_face_engine_device_jpeg_matches_pillow(tmp_path, monkeypatch):
    """The face engine's batched device JPEG path (host entropy decode + one GPU reconstruction,
    pixels never leave the device) detects and embeds like the Pillow path; an undecodable
    payload fails alone."""
    from lumen_amd.services.face.backend import DetParams, InvalidInputError, dp_worker

    write_face_model(tmp_path / "models" / "buffalo_tiny", "buffalo_tiny")
    cfg = config_from_dict(_cfg(tmp_path, "cuda"))
    svc = GeneralFaceService.from_config(cfg.services["face"], tmp_path)
    svc.initialize()
    try:
        fn = dp_worker("cuda", svc.backend.resources)
        rng = np.random.default_rng(7)
        jpegs = [encode_jpeg(rng.integers(0, 255, (96 + 8 * k, 160 - 4 * k, 3), dtype=np.uint8)) for k in range(3)]
        items = [(j, DetParams(0.0, 0.3, 0, 10000), 4) for j in jpegs] + [(b"not an image", DetParams(), 4)]
        monkeypatch.setenv("LUMEN_FACE_DEVICE_JPEG", "1")
        dev = fn("det_emb", items)
        monkeypatch.setenv("LUMEN_FACE_DEVICE_JPEG", "0")
        host = fn("det_emb", items)
        assert isinstance(dev[3], InvalidInputError) and isinstance(host[3], InvalidInputError)
        for d, h in zip(dev[:3], host[:3]):
            assert len(d) > 0 and abs(len(d) - len(h)) <= 1
            assert np.abs(np.array(d[0][0].bbox) - np.array(h[0][0].bbox)).max() < 4.0
            assert float(np.dot(d[0][1], h[0][1])) > 0.95
    finally:
        svc.close()


def test_pipelined_detect_embed_matches_sync(tmp_path):
    """Two detector batches in flight (detect_launch x2, detect_finish, the async batch embedding
    queued behind the second detector) give the synchronous detect_and_embed_images result."""
    from lumen_amd.services.face.backend import DetParams

    write_face_model(tmp_path / "models" / "buffalo_tiny", "buffalo_tiny")
    cfg = config_from_dict(_cfg(tmp_path, "cuda"))
    svc = GeneralFaceService.from_config(cfg.services["face"], tmp_path)
    svc.initialize()
    try:
        be = svc.backend
        rng = np.random.default_rng(11)
        batches = [[rng.integers(0, 255, (96 + 8 * k, 160 - 4 * k, 3), dtype=np.uint8) for k in range(3)]
                   for _ in range(2)]
        p = [DetParams(0.0, 0.3, 0, 10000)] * 3
        ref = [be.detect_and_embed_images(b, p, 4) for b in batches]
        st = [be.detect_launch(b, p) for b in batches]
        got = []
        for b, s in zip(batches, st):
            h = be.embed_batch_detections_async(b, be.detect_finish(s), [4] * len(b))
            got.append(be.embed_batch_detections_wait(h))
        for g_, r_ in zip(got, ref):
            for gi, ri in zip(g_, r_):
                assert len(gi) == len(ri) > 0
                for (fg, eg), (fr, er) in zip(gi, ri):
                    assert np.abs(np.array(fg.bbox) - np.array(fr.bbox)).max() < 1e-3
                    assert float(np.dot(eg, er)) > 0.999
    finally:
        svc.close()
