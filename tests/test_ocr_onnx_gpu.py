"""PP-OCR-layout ONNX pack on the MI355X graph executor vs the CPU path."""
import numpy as np
import pytest

from test_ocr_onnx_cpu import run_backend

pytestmark = pytest.mark.gpu


def test_onnx_ocr_pack_gpu_matches_cpu(tmp_path):
    bc, tc = run_backend(tmp_path, "cpu")
    bg, tg = run_backend(tmp_path, "cuda")
    assert len(bg) == len(bc) == 1
    assert np.abs(np.asarray(bg[0]) - np.asarray(bc[0])).max() <= 3
    assert tg[0][0] == tc[0][0] or abs(tg[0][1] - tc[0][1]) < 0.05
