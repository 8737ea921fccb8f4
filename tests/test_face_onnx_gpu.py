"""InsightFace-layout ONNX face pack on the MI355X graph executor vs the CPU path."""
import numpy as np
import pytest

from test_face_onnx_cpu import S, write_pack

pytestmark = pytest.mark.gpu


def test_onnx_face_pack_gpu_matches_cpu(tmp_path):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.face.backend import DetParams, MI355XFaceBackend

    write_pack(tmp_path / "models" / "buffalo_onnx")
    res = load_model_resources(tmp_path, ModelConfig(model="buffalo_onnx", runtime=Runtime.onnx))
    rng = np.random.default_rng(5)
    img = rng.integers(0, 255, (S, S, 3), dtype=np.uint8)
    crop = rng.integers(0, 255, (112, 112, 3), dtype=np.uint8)
    out = {}
    for dev in ("cpu", "cuda"):
        be = MI355XFaceBackend(res, device=dev)
        be.initialize()
        try:
            faces = be.detect_images([img], [DetParams(conf=0.5, nms=1.0, size_min=0.0, size_max=1e9)])[0]
            out[dev] = (faces, be.face_to_embedding(cropped_face_array=crop))
        finally:
            be.close()
    (fc, ec), (fg, eg) = out["cpu"], out["cuda"]
    assert abs(len(fg) - len(fc)) <= max(2, len(fc) // 10)
    assert float(np.dot(ec, eg)) > 0.99
