"""The engine / front-end serving topology on the GPU (hub/server.py:serve_frontends,
parallel/engine.py:EngineSet): a hub.example-shaped config (SmartCLIP = general CLIP + BioCLIP on
one engine, face, OCR, the VLM) served by 2 front-end processes over ONE engine process on
cuda:0 answers every task like the in-process hub on the same GPU (embeddings cos > 0.9999, same
labels / boxes / texts; label scores within 3e-3 -- the bf16 tower's batch composition moves
softmax(100 cos) by a few 1e-4).  Reference: /root/reference/src/lumen/server.py:232-235 serves all of
them from one process."""
import pytest

from test_frontends_all_cpu import ALL, REQS, _config, _free_port, _reference, _same, _serve, _svc

pytestmark = pytest.mark.gpu


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


def test_engine_set_on_gpu_answers_like_in_process_hub(tmp_path, cache, monkeypatch):
    # both sides decode face JPEGs with Pillow (the engine's batched device decode is covered by
    # tests/test_face_gpu.py): the random-init detector moves boxes by ~0.5 px on IDCT rounding
    monkeypatch.setenv("LUMEN_FACE_DEVICE_JPEG", "0")
    port = _free_port()
    cfg = _config(cache, port, {k: _svc(*v, device="cuda") for k, v in ALL.items()})
    ref, app = _reference(cfg)
    app.close()
    got = _serve(tmp_path, cfg, 2, [r[0] for r in REQS], monkeypatch, devices=["cuda:0"])
    assert set(got) == {r[0] for r in REQS}
    for t, _, _, _ in REQS:
        # bf16 tower: batch composition moves the softmax(100 cos) scores by a few 1e-4
        _same(t, got[t], ref[t], score_atol=3e-3, box_atol=0.05, emb_cos=0.999)


def test_vlm_engine_streams_tokens_on_gpu(tmp_path, cache, monkeypatch):
    """The VLM on a GPU engine behind 2 front ends streams: chunks arrive while the engine still
    generates (first chunk < 50 % of the request time), text equal to the in-process stream."""
    from test_vlm_stream_cpu import engine_stream_check

    engine_stream_check(tmp_path, cache, monkeypatch, "cuda:0", 128)
