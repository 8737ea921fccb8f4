"""Multi-GPU serving topology on CPU workers: face / OCR data-parallel worker pools give the
same results as the single-process backends (reference hot loops: face_service.py:516-574,
ocr onnxrt_backend.py:150-632), the shared-memory result ring, concurrent dispatchers, and
the hub's per-service GPU placement plan."""
import json
import threading

import numpy as np
import pytest

from lumen_amd.parallel.worker_pool import GPUWorkerPool
from lumen_amd.runtime import placement
from lumen_amd.runtime.batcher import DynamicBatcher
from lumen_amd.utils.image import encode_jpeg, encode_png


# ----------------------------------------------------------------------------- placement
def test_placement_plan_auto_and_spec():
    p = placement.plan(["clip", "face", "ocr", "vlm"], 8)
    assert sorted(i for v in p.values() for i in v) == list(range(8))           # disjoint, all used
    assert all(len(v) >= 1 for v in p.values()) and len(p["clip"]) >= len(p["ocr"])
    assert placement.plan(["clip", "face"], 1) == {"clip": [0], "face": [0]}     # shared
    assert placement.plan(["clip"], 0) == {"clip": []}
    p = placement.plan(["clip", "face", "ocr"], 8, "face=4,5;clip=0-3")
    assert p["face"] == [4, 5] and p["clip"] == [0, 1, 2, 3] and p["ocr"] == [6, 7]
    with pytest.raises(ValueError):
        placement.plan(["clip"], 4, "clip=5")
    with pytest.raises(ValueError):
        placement.parse_spec("clip")


def test_placement_resolve(monkeypatch):
    monkeypatch.delenv("LUMEN_DP_SIZE", raising=False)
    assert placement.resolve(None) == (None, [])
    assert placement.resolve("cpu", 2) == ("cpu", ["cpu", "cpu"])
    with placement.use([4, 5, 6]):
        assert placement.current() == (4, 5, 6)
        assert placement.resolve(None) == ("cuda:4", ["cuda:4", "cuda:5", "cuda:6"])
        assert placement.resolve(None, 1) == ("cuda:4", [])
        assert placement.resolve("cuda:7") == ("cuda:7", [])       # explicit device wins
    assert placement.current() is None


# ----------------------------------------------------------------------------- pool transport
def _rows_factory(device, dim=4096):
    def fn(kind, items):
        if kind == "blobs":      # inputs through the shared-memory input ring
            return [np.full(dim, float(len(b) + b[0]), np.float32) for b in items]
        if kind == "small":
            return [np.full(3, float(x), np.float32) for x in items]
        return [np.full(dim, float(x), np.float32) for x in items]
    return fn


def test_shm_result_ring_round_trip():
    pool = GPUWorkerPool("tests.test_dp_serving_cpu:_rows_factory", ["cpu"], shm_slots=2, shm_slot_bytes=1 << 20)
    try:
        futs = [pool.submit("rows", list(range(i, i + 16))) for i in range(0, 160, 16)]   # > slots in flight
        for i, f in zip(range(0, 160, 16), futs):
            r = f.result(60)
            assert len(r) == 16 and all(r[k][0] == i + k and r[k].shape == (4096,) for k in range(16))
        assert pool.stats["shm_results"] == 10
        small = pool.submit("small", [1, 2]).result(60)                                    # below threshold
        assert [float(x[0]) for x in small] == [1.0, 2.0] and pool.stats["shm_results"] == 10
    finally:
        pool.close()


def test_batcher_concurrency_keeps_batches_in_flight():
    active, peak, lock = [0], [0], threading.Lock()
    gate = threading.Event()

    def fn(items):
        with lock:
            active[0] += 1
            peak[0] = max(peak[0], active[0])
        gate.wait(5)
        with lock:
            active[0] -= 1
        return [x * 2 for x in items]

    b = DynamicBatcher(fn, max_batch=2, max_wait_ms=1, name="t", concurrency=3)
    try:
        futs = [b.submit(i) for i in range(6)]
        threading.Timer(0.5, gate.set).start()
        assert [f.result(10) for f in futs] == [2 * i for i in range(6)]
        assert peak[0] >= 2
    finally:
        b.close()


# ----------------------------------------------------------------------------- face DP
def _face_svc(cache, monkeypatch, dp):
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.face import GeneralFaceService
    from tests.test_face_service_cpu import _svc_cfg

    if dp > 1:
        monkeypatch.setenv("LUMEN_DP_SIZE", str(dp))
    else:
        monkeypatch.delenv("LUMEN_DP_SIZE", raising=False)
    cfg = config_from_dict(_svc_cfg(cache))
    svc = GeneralFaceService.from_config(cfg.services["face"], cache)
    svc.initialize()
    return svc


def _cos(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


LOW = {"detection_confidence_threshold": "0.0", "face_size_min": "0", "nms_threshold": "0.3", "max_faces": "4"}


def test_face_dp2_matches_single_process(tmp_path, monkeypatch):
    from lumen_amd.models.face import write_face_model

    write_face_model(tmp_path / "models" / "buffalo_tiny", "buffalo_tiny")
    imgs = [encode_jpeg(np.random.default_rng(s).integers(0, 255, (96, 128 + 8 * s, 3), dtype=np.uint8))
            for s in range(4)]
    crop = encode_jpeg(np.random.default_rng(9).integers(0, 255, (112, 112, 3), dtype=np.uint8))

    def run(svc):
        out = [json.loads(svc.handle("face_detect_and_embed", im, "image/jpeg", LOW)[0]) for im in imgs]
        out.append(json.loads(svc.handle("face_detect", imgs[0], "image/jpeg", LOW)[0]))
        out.append(json.loads(svc.handle("face_embed", crop, "image/jpeg", {})[0]))
        return out

    single = _face_svc(tmp_path, monkeypatch, 1)
    try:
        ref = run(single)
    finally:
        single.close()
    dp = _face_svc(tmp_path, monkeypatch, 2)
    try:
        assert dp.backend._pool is not None and dp.backend._pool.size == 2
        # concurrent requests from several threads: batches spread over both workers
        got: list = [None] * 8
        ths = [threading.Thread(target=lambda k=k: got.__setitem__(k, run(dp))) for k in range(8)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
        assert dp.backend.get_info().extra["dp_workers"] == "2"
        with pytest.raises(Exception):
            dp.handle("face_detect", b"not a jpeg", "image/jpeg", LOW)
    finally:
        dp.close()
    for g in got:
        assert g is not None and len(g) == len(ref)
        for a, b in zip(g, ref):
            if "faces" in a:
                assert a["count"] == b["count"] > 0
                for fa, fb in zip(a["faces"], b["faces"]):
                    np.testing.assert_allclose(fa["bbox"], fb["bbox"], atol=1e-4)
                    if fa.get("embedding") is not None:      # fp32 CPU convs batch differently: cosine, not bits
                        assert _cos(fa["embedding"], fb["embedding"]) > 0.99999
            else:
                assert _cos(a["vector"], b["vector"]) > 0.99999


# ----------------------------------------------------------------------------- OCR DP
def test_ocr_dp2_matches_single_process(tmp_path, monkeypatch):
    from lumen_amd.models.ocr import write_ocr_model
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.ocr.service import GeneralOcrService
    from tests.test_ocr_cpu import _cfg, _rgb

    write_ocr_model(tmp_path / "models" / "ppocr-tiny", "ppocr-tiny")
    meta = {"detection_threshold": "0.0", "ocr.box_thresh": "0.0", "recognition_threshold": "0.0"}
    imgs = [encode_png(_rgb(70, 150, s)) for s in range(3)]

    def build(dp):
        if dp > 1:
            monkeypatch.setenv("LUMEN_DP_SIZE", str(dp))
        else:
            monkeypatch.delenv("LUMEN_DP_SIZE", raising=False)
        cfg = config_from_dict(_cfg(tmp_path))
        svc = GeneralOcrService.from_config(cfg.services["ocr"], tmp_path)
        svc.initialize()
        return svc

    single = build(1)
    try:
        ref = [json.loads(single.handle("ocr", im, "image/png", meta)[0]) for im in imgs]
    finally:
        single.close()
    dp = build(2)
    try:
        assert dp.manager.backend._pool is not None and dp.manager.backend._pool.size == 2
        got: list = [None] * len(imgs)
        ths = [threading.Thread(target=lambda k=k: got.__setitem__(
            k, json.loads(dp.handle("ocr", imgs[k], "image/png", meta)[0]))) for k in range(len(imgs))]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
    finally:
        dp.close()
    for a, b in zip(got, ref):
        assert a["count"] == b["count"] >= 1
        for ia, ib in zip(a["items"], b["items"]):
            assert ia["box"] == ib["box"] and ia["text"] == ib["text"]
            assert abs(ia["confidence"] - ib["confidence"]) < 1e-5


def test_shm_input_ring_round_trip_and_fallback():
    pool = GPUWorkerPool("tests.test_dp_serving_cpu:_rows_factory", ["cpu"], shm_slots=2, shm_slot_bytes=1 << 16)
    try:
        batches = [[bytes([i % 251]) * (100 + 37 * k) for k in range(8)] for i in range(12)]   # > slots in flight
        futs = [pool.submit("blobs", b) for b in batches]
        for b, f in zip(batches, futs):
            r = f.result(60)
            assert [float(x[0]) for x in r] == [float(len(x) + x[0]) for x in b]
        assert pool.stats["shm_inputs"] == 12
        big = [bytes([7]) * 40000, bytes([9]) * 40000]               # > one slot: pickled
        assert [float(x[0]) for x in pool.submit("blobs", big).result(60)] == [40007.0, 40009.0]
        assert pool.stats["shm_inputs"] == 12
    finally:
        pool.close()


def test_stale_ring_descriptor_is_dropped():
    """A result descriptor from a previous spawn of the worker (its ring is gone) is dropped
    without touching the new ring's semaphore, and the collector keeps running."""
    pool = GPUWorkerPool("tests.test_dp_serving_cpu:_rows_factory", ["cpu"], shm_slots=2, shm_slot_bytes=1 << 20)
    try:
        w = pool.workers[0]
        pool._handle("okshm", 0, 12345, (w.gen - 1, 0, (4, 4096), "<f4"))
        assert pool.stats["stale_dropped"] == 1
        pool._outq.put(("okshm", 0, 999, "garbage"))                  # malformed: logged, not fatal
        r = pool.submit("rows", list(range(16))).result(60)
        assert len(r) == 16 and r[3][0] == 3.0
    finally:
        pool.close()


# ----------------------------------------------------------------------------- SPMD face DP (RCCL path, gloo here)
def _face_backend_cpu(cache):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.face.backend import MI355XFaceBackend

    res = load_model_resources(cache, ModelConfig(model="buffalo_tiny", runtime=Runtime.onnx))
    be = MI355XFaceBackend(res, device="cpu")
    be.initialize()
    return be


def _spmd_images():
    from lumen_amd.utils.image import decode_rgb

    return [decode_rgb(encode_jpeg(np.random.default_rng(s).integers(0, 255, (96, 120 + 8 * s, 3), dtype=np.uint8)))
            for s in range(5)]


def _spmd_face_rank(rank, world, port, cache, q):
    import os

    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from lumen_amd.parallel import Communicator, destroy, init_distributed
    from lumen_amd.services.face.backend import DetParams
    from lumen_amd.services.face.spmd import SPMDFaceRunner

    st = init_distributed(tp_size=1, device=torch.device("cpu"), timeout_s=120)
    try:
        be = _face_backend_cpu(cache)
        imgs = _spmd_images()
        run = SPMDFaceRunner(be, Communicator(st.dp_group, ipc=False), torch.device("cpu"))
        out = run.run(imgs, [DetParams(0.0, 0.3, 0, 10000)] * len(imgs), max_faces=4)
        q.put((rank, [[(f.bbox, f.confidence, f.landmarks, e.tolist()) for f, e in faces] for faces in out]))
        be.close()
    finally:
        destroy()


def test_spmd_face_world2_matches_single_process(tmp_path):
    """Each of 2 gloo ranks detects + embeds its shard of 5 images; one all-gather of the packed
    (bbox, confidence, landmarks, embedding) rows gives every rank the single-process result."""
    import multiprocessing as mp

    from lumen_amd.models.face import write_face_model
    from lumen_amd.services.face.backend import DetParams
    from tests.test_parallel_cpu import _port

    write_face_model(tmp_path / "models" / "buffalo_tiny", "buffalo_tiny")
    be = _face_backend_cpu(tmp_path)
    imgs = _spmd_images()
    ref = be.detect_and_embed_images(imgs, [DetParams(0.0, 0.3, 0, 10000)] * len(imgs), max_faces=4)
    be.close()
    assert sum(len(f) for f in ref) > 0
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_spmd_face_rank, args=(r, 2, port, tmp_path, qq)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(qq.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    for rank in (0, 1):
        got = res[rank]
        assert [len(f) for f in got] == [len(f) for f in ref]
        for gf, rf in zip(got, ref):
            for (bb, conf, lm, emb), (f, e) in zip(gf, rf):
                np.testing.assert_allclose(bb, f.bbox, atol=1e-3)
                assert abs(conf - f.confidence) < 1e-5
                np.testing.assert_allclose(np.asarray(lm).ravel(), np.asarray(f.landmarks).ravel(), atol=1e-3)
                assert _cos(emb, e) > 0.99999


# ----------------------------------------------------------------------------- SPMD OCR DP (RCCL path, gloo here)
def _ocr_backend_cpu(cache):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.ocr.backend import MI355XOcrBackend

    res = load_model_resources(cache, ModelConfig(model="ppocr-tiny", runtime=Runtime.onnx))
    be = MI355XOcrBackend(res, device="cpu")
    be.initialize()
    return be


def _ocr_images():
    from tests.test_ocr_cpu import _rgb

    return [_rgb(70, 150 + 10 * s, s) for s in range(5)]


_OCR_P = dict(det_thresh=0.0, rec_thresh=0.0, box_thresh=0.0)


def _spmd_ocr_rank(rank, world, port, cache, q):
    import os

    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from lumen_amd.parallel import Communicator, destroy, init_distributed
    from lumen_amd.services.ocr.backend import OcrParams
    from lumen_amd.services.ocr.spmd import SPMDOcrRunner

    st = init_distributed(tp_size=1, device=torch.device("cpu"), timeout_s=120)
    try:
        be = _ocr_backend_cpu(cache)
        imgs = _ocr_images()
        run = SPMDOcrRunner(be, Communicator(st.dp_group, ipc=False), torch.device("cpu"))
        out = run.run(imgs, [OcrParams(**_OCR_P)] * len(imgs))
        q.put((rank, [[(r.box, r.text, r.confidence) for r in lines] for lines in out]))
        be.close()
    finally:
        destroy()


def test_spmd_ocr_pack_roundtrip():
    """Packed OCR rows (box, confidence, code points) survive pack -> unpack exactly, including
    non-ASCII text and images without lines."""
    from lumen_amd.services.ocr.backend import OcrResult
    from lumen_amd.services.ocr.spmd import pack_lines, unpack_lines

    res = [[OcrResult(box=[(1, 2), (30, 2), (30, 9), (1, 9)], text="ab中文", confidence=0.75)], [],
           [OcrResult(box=[(0, 0), (5, 0), (5, 5), (0, 5)], text="", confidence=0.5),
            OcrResult(box=[(7, 8), (9, 8), (9, 12), (7, 12)], text="\U0001F600x", confidence=1.0)]]
    rows, counts = pack_lines(res, 4, 2, 4)
    back = unpack_lines(rows.numpy(), counts.numpy())
    assert back[3] == [] and [[(r.box, r.text, r.confidence) for r in ls] for ls in back[:3]] == \
        [[(r.box, r.text, r.confidence) for r in ls] for ls in res]


def test_spmd_ocr_world2_matches_single_process(tmp_path):
    """Each of 2 gloo ranks runs detect + recognise on its shard of 5 images; one all-gather of
    the packed (box, confidence, code point) rows gives every rank the single-process result."""
    import multiprocessing as mp

    from lumen_amd.models.ocr import write_ocr_model
    from lumen_amd.services.ocr.backend import OcrParams
    from tests.test_parallel_cpu import _port

    write_ocr_model(tmp_path / "models" / "ppocr-tiny", "ppocr-tiny")
    be = _ocr_backend_cpu(tmp_path)
    imgs = _ocr_images()
    ref = be._predict_batch([(im, OcrParams(**_OCR_P)) for im in imgs])
    be.close()
    assert sum(len(ls) for ls in ref) > 0
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_spmd_ocr_rank, args=(r, 2, port, tmp_path, qq)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(qq.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    want = [[(r.box, r.text, r.confidence) for r in ls] for ls in ref]
    for rank in (0, 1):
        got = res[rank]
        assert [len(ls) for ls in got] == [len(ls) for ls in want]
        for gl, wl in zip(got, want):
            for (gb, gt, gc), (wb, wt, wc) in zip(gl, wl):
                assert list(map(tuple, gb)) == list(map(tuple, wb)), (gb, wb)
                assert gt == wt, (gt, wt)
                assert abs(gc - wc) < 1e-4, (gc, wc)   # fp32 recogniser over a different batch
