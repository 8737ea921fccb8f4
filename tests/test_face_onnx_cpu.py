"""A reference-style InsightFace ONNX face pack (no lumen_face_config.json / safetensors:
SCRFD graph with the nine score/bbox/kps outputs in InsightFace order + an ArcFace-style
recogniser graph) served by the face backend through the ONNX graph executor.  The graphs
are synthetic (tiny, written by lumen_amd.utils.onnx_lite); the decode contract is pinned by
comparing against a NumPy SCRFD decode of the same graph outputs (InsightFace
distance2bbox convention)."""
import json

import numpy as np
import torch

from lumen_amd.resources.model_info import ModelInfo
from lumen_amd.runtime.onnx_graph import OnnxGraph
from lumen_amd.utils import onnx_lite as ox
from lumen_amd.utils.image import encode_jpeg

R = np.random.default_rng(3)
S, A = 64, 2


def _w(*s, scale=0.3):
    return (R.standard_normal(s) * scale).astype(np.float32)


def scrfd_graph():
    N = ox.Node
    init = {"w0": _w(16, 3, 3, 3), "b0": _w(16), "shape1": np.array([-1, 1], np.int64),
            "shape4": np.array([-1, 4], np.int64), "shape10": np.array([-1, 10], np.int64)}
    nodes, outs = [], {"score": [], "bbox": [], "kps": []}
    prev, ch = "x", 3
    nodes.append(N("Conv", ["x", "w0", "b0"], ["f4"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                              "strides": [4, 4]}))
    nodes.append(N("Relu", ["f4"], ["r4"]))
    prev = "r4"
    for s in (8, 16, 32):
        init[f"wd{s}"] = _w(16, 16, 3, 3)
        nodes.append(N("Conv", [prev, f"wd{s}"], [f"f{s}"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                                   "strides": [2, 2]}))
        nodes.append(N("Relu", [f"f{s}"], [f"r{s}"]))
        prev = f"r{s}"
        for kind, c in (("score", 1), ("bbox", 4), ("kps", 10)):
            init[f"h{kind}{s}"] = _w(A * c, 16, 1, 1, scale=0.5)
            init[f"hb{kind}{s}"] = (_w(A * c) + (1.0 if kind == "bbox" else 0.0)).astype(np.float32)
            nodes.append(N("Conv", [prev, f"h{kind}{s}", f"hb{kind}{s}"], [f"o{kind}{s}"], attrs={"kernel_shape": [1, 1]}))
            src = f"o{kind}{s}"
            if kind == "score":
                nodes.append(N("Sigmoid", [src], [f"sg{s}"]))
                src = f"sg{s}"
            elif kind == "bbox":          # positive distances, as trained SCRFD heads produce
                nodes.append(N("Sigmoid", [src], [f"bs{s}"]))
                src = f"bs{s}"
            nodes.append(N("Transpose", [src], [f"t{kind}{s}"], attrs={"perm": [0, 2, 3, 1]}))
            nodes.append(N("Reshape", [f"t{kind}{s}", f"shape{c}"], [f"{kind}_{s}"]))
            outs[kind].append(f"{kind}_{s}")
    return ox.Graph(nodes, init, ["x"], outs["score"] + outs["bbox"] + outs["kps"])


def rec_graph():
    N = ox.Node
    init = {"w0": _w(32, 3, 3, 3), "a0": np.full(32, 0.25, np.float32), "fc": _w(512, 32), "fcb": _w(512)}
    nodes = [N("Conv", ["data", "w0"], ["c0"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "strides": [2, 2]}),
             N("PRelu", ["c0", "a0"], ["p0"]),
             N("GlobalAveragePool", ["p0"], ["g"]),
             N("Flatten", ["g"], ["f"]),
             N("Gemm", ["f", "fc", "fcb"], ["fc1"], attrs={"transB": 1})]
    return ox.Graph(nodes, init, ["data"], ["fc1"])


def write_pack(root):
    root.mkdir(parents=True)
    (root / "onnx").mkdir()
    (root / "onnx" / "detection.fp32.onnx").write_bytes(ox.write_model(scrfd_graph()))
    (root / "onnx" / "recognition.fp32.onnx").write_bytes(ox.write_model(rec_graph()))
    files = ["onnx/detection.fp32.onnx", "onnx/recognition.fp32.onnx"]
    info = {"name": root.name, "version": "1.0.0", "description": "synthetic insightface-layout ONNX pack",
            "model_type": "face", "embedding_dim": 512, "source": {"format": "custom", "repo_id": "synthetic/x"},
            "runtimes": {"onnx": {"available": True, "files": files, "devices": ["cpu", "cuda"]}},
            "extra_metadata": {"insightface": {"detection": {"input_size": [S, S]}}}}
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info))


def numpy_decode(outs, thresh):
    """InsightFace SCRFD.forward decode (distance2bbox on anchor centres) at letterbox scale."""
    boxes, scores = [], []
    for i, s in enumerate((8, 16, 32)):
        H = W = S // s
        sc, bb = outs[i].reshape(-1), outs[3 + i].reshape(-1, 4) * s
        yy, xx = np.mgrid[:H, :W]
        centers = np.stack([xx, yy], -1).reshape(-1, 2).astype(np.float32) * s
        centers = np.repeat(centers, A, axis=0)
        keep = sc >= thresh
        b = np.concatenate([centers - bb[:, :2], centers + bb[:, 2:]], 1)
        boxes.append(b[keep])
        scores.append(sc[keep])
    return np.concatenate(boxes), np.concatenate(scores)


def test_onnx_face_pack_served(tmp_path):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.face.backend import DetParams, MI355XFaceBackend
    from lumen_amd.services.face.onnx_pack import OnnxSCRFD

    write_pack(tmp_path / "models" / "buffalo_onnx")
    res = load_model_resources(tmp_path, ModelConfig(model="buffalo_onnx", runtime=Runtime.onnx))
    be = MI355XFaceBackend(res, device="cpu")
    be.initialize()
    try:
        assert isinstance(be.det, OnnxSCRFD) and be.spec.det_size == S
        img = R.integers(0, 255, (S, S, 3), dtype=np.uint8)          # already S x S: letterbox scale 1
        faces = be.detect_images([img], [DetParams(conf=0.5, nms=1.0, size_min=0.0, size_max=1e9)])[0]
        # reference decode of the same graph outputs
        x = torch.from_numpy(((img.astype(np.float32) - 127.5) / 128.0).transpose(2, 0, 1)[None].copy())
        outs = [o.numpy() for o in OnnxGraph(tmp_path / "models" / "buffalo_onnx" / "onnx" / "detection.fp32.onnx")
                .run({"x": x})]
        rb, rs = numpy_decode(outs, 0.5)
        assert len(faces) == len(rs) > 0
        got = np.array(sorted([f.bbox for f in faces]))
        ref = np.array(sorted(np.clip(rb, 0, S).tolist()))
        assert got.shape == ref.shape
        np.testing.assert_allclose(got, ref, atol=0.05)
        e = be.face_to_embedding(cropped_face_array=R.integers(0, 255, (112, 112, 3), dtype=np.uint8))
        assert e.shape == (512,) and abs(float(np.linalg.norm(e)) - 1) < 1e-4
    finally:
        be.close()
