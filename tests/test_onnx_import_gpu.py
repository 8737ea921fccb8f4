"""ONNX-pack CLIP on the MI355X path: the imported weights run the same HIP kernels and give
the same embeddings as the safetensors pack of the same model (CPU twin: test_onnx_import_cpu)."""
import numpy as np
import pytest

from tests.test_onnx_import_cpu import _write_clip_onnx

pytestmark = pytest.mark.gpu


def test_clip_onnx_pack_gpu_matches_safetensors(tmp_path):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.services.clip.backend import create_backend
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    src = tmp_path / "models" / "clip-b"
    write_clip_model(src, "clip-b", preset="tiny", dataset=None)
    settings = type("S", (), {"device": "cuda", "batch_size": 8})()
    imgs = [encode_jpeg(np.random.default_rng(i).integers(0, 255, (64, 80, 3), dtype=np.uint8)) for i in range(5)]

    def embed(rt):
        res = ResourceLoader.load_model_resources(tmp_path, ModelConfig(model="clip-b", runtime=rt))
        b = create_backend(settings, res, rt.value)
        b.initialize()
        try:
            assert b.device.type == "cuda"
            b.model.center_crop = False   # same preprocessor on both runtimes (torch's crop is tested apart)
            return b.image_batch_to_vectors(imgs), b.text_batch_to_vectors(["a cat", "two dogs", "x"])
        finally:
            b.close()

    ref_i, ref_t = embed(Runtime.torch)
    _write_clip_onnx(src)
    (src / "model.safetensors").unlink()
    got_i, got_t = embed(Runtime.onnx)
    np.testing.assert_array_equal(got_i, ref_i)       # same bf16 weights, same kernels: bitwise
    np.testing.assert_array_equal(got_t, ref_t)
