"""A reference-style PP-OCR ONNX pack (detection / recognition ONNX + ppocr_keys, no native
safetensors) served by the OCR backend through the MI355X ONNX graph executor.  Synthetic
graphs: the detector is a fixed 1x1 conv + sigmoid (bright pixels -> text probability), so
the detected box is known; the recogniser is a strided conv + softmax CTC head."""
import json

import numpy as np

from lumen_amd.resources.model_info import ModelInfo
from lumen_amd.utils import onnx_lite as ox

VOCAB = [chr(c) for c in range(ord("a"), ord("z") + 1)]
C = len(VOCAB) + 2          # blank + vocab + space


def det_graph():
    N = ox.Node
    init = {"w": np.array([[[[8.0]], [[8.0]], [[8.0]]]], np.float32), "b": np.array([-4.0], np.float32)}
    return ox.Graph([N("Conv", ["x", "w", "b"], ["c"], attrs={"kernel_shape": [1, 1]}),
                     N("Sigmoid", ["c"], ["prob"])], init, ["x"], ["prob"])


def rec_graph():
    N = ox.Node
    r = np.random.default_rng(0)
    init = {"w": (r.standard_normal((C, 3, 48, 4)) * 0.05).astype(np.float32), "b": np.zeros(C, np.float32),
            "ax": np.array([2], np.int64)}
    return ox.Graph([N("Conv", ["x", "w", "b"], ["c"], attrs={"kernel_shape": [48, 4], "strides": [48, 4]}),
                     N("Squeeze", ["c", "ax"], ["s"]),
                     N("Transpose", ["s"], ["t"], attrs={"perm": [0, 2, 1]}),
                     N("Softmax", ["t"], ["probs"], attrs={"axis": 2})], init, ["x"], ["probs"])


def write_pack(root):
    root.mkdir(parents=True)
    (root / "det.onnx").write_bytes(ox.write_model(det_graph()))
    (root / "rec.onnx").write_bytes(ox.write_model(rec_graph()))
    (root / "ppocr_keys_v1.txt").write_text("\n".join(VOCAB) + "\n")
    files = ["det.onnx", "rec.onnx", "ppocr_keys_v1.txt"]
    info = {"name": root.name, "version": "1.0.0", "description": "synthetic PP-OCR-layout ONNX pack",
            "model_type": "ocr", "source": {"format": "custom", "repo_id": "synthetic/x"},
            "runtimes": {"onnx": {"available": True, "files": files, "devices": ["cpu", "cuda"]}},
            "extra_metadata": {"rec_config": {"image_shape": [3, 48, 320], "character_dict_path": "ppocr_keys_v1.txt"}}}
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info))


def image():
    img = np.zeros((128, 256, 3), np.uint8)
    img[40:80, 30:200] = 255
    return img


def run_backend(tmp_path, device):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.ocr.backend import MI355XOcrBackend, OcrParams
    from lumen_amd.services.ocr.onnx_pack import OnnxDBNet

    root = tmp_path / "models" / "ppocr_onnx"
    if not root.exists():
        write_pack(root)
    res = load_model_resources(tmp_path, ModelConfig(model="ppocr_onnx", runtime=Runtime.onnx))
    be = MI355XOcrBackend(res, device=device)
    be.initialize()
    try:
        assert isinstance(be.det, OnnxDBNet)
        boxes = be.detect([image()], [OcrParams()])[0]
        texts = be.recognize([image()], [(0, b) for b in boxes])
        return boxes, texts
    finally:
        be.close()


def test_onnx_ocr_pack_served(tmp_path):
    boxes, texts = run_backend(tmp_path, "cpu")
    assert len(boxes) == 1
    b = np.asarray(boxes[0])
    # the DB unclip (ratio 1.5) grows the region by area * 1.5 / perimeter ~ 24 px per side
    assert b[:, 0].min() <= 30 and b[:, 0].max() >= 199 and b[:, 1].min() <= 40 and b[:, 1].max() >= 79
    assert abs(b[:, 0].mean() - 115) <= 4 and abs(b[:, 1].mean() - 60) <= 4
    t, conf = texts[0]
    assert set(t) <= set(VOCAB) | {" "} and 0.0 < conf <= 1.0
