"""Synthetic RetinaFace-shaped ONNX face packs (F-4: the non-SCRFD detector path).

The reference keeps a generic decode for detectors that are not SCRFD
(packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py:810-880: ``detector_type``
"retinaface", outputs picked by an index map, boxes already decoded, optionally normalised to
the image).  No such pack ships with the reference and there is no network, so this module
writes random-init ONNX graphs of the RetinaFace output contract with
:mod:`lumen_amd.utils.onnx_lite`:

* ``encoding="priors"`` -- a raw RetinaFace export: a stride-4 stem and three FPN-like levels
  (strides 8 / 16 / 32), each with 2 priors per cell, and the three heads flattened NHWC and
  concatenated over levels: ``loc`` [N, P, 4] (centre / size regressions against the prior
  grid, variances 0.1 / 0.2), ``conf`` [N, P, 2] (softmax: background, face) and ``landms``
  [N, P, 10];
* ``encoding="decoded"`` -- the same trunk with the box decode inside the graph (the reference's
  contract): ``boxes`` [N, P, 4] corner boxes in input pixels, ``scores`` [N, P] and
  ``landmarks`` [N, P, 10] in input pixels.

Both come with a small ArcFace-style recogniser graph, so the pack is servable end to end by
the face backend (``services/face/onnx_pack.py:OnnxBoxDetector``).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from ..utils import onnx_lite as ox
from .model_info import ModelInfo

STEPS = (8, 16, 32)
MIN_SIZES = ((16, 32), (64, 128), (256, 512))


def retinaface_graph(size: int = 64, encoding: str = "priors", seed: int = 0, width: int = 16) -> ox.Graph:
    rng = np.random.default_rng(seed)
    N = ox.Node

    def w(*s, scale=0.3):
        return (rng.standard_normal(s) * scale).astype(np.float32)

    A = 2
    init = {"w0": w(width, 3, 3, 3, scale=0.004), "b0": w(width)}    # inputs are pixel - mean (~ +-130)
    for c in (2, 4, 10):
        init[f"shape{c}"] = np.array([0, -1, c], np.int64)
    nodes = [N("Conv", ["x", "w0", "b0"], ["f4"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                         "strides": [4, 4]}),
             N("Relu", ["f4"], ["r4"])]
    prev = "r4"
    flat = {"loc": [], "conf": [], "landms": []}
    for s in STEPS:
        init[f"wd{s}"] = w(width, width, 3, 3)
        nodes += [N("Conv", [prev, f"wd{s}"], [f"f{s}"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                                "strides": [2, 2]}),
                  N("Relu", [f"f{s}"], [f"r{s}"])]
        prev = f"r{s}"
        for kind, c in (("loc", 4), ("conf", 2), ("landms", 10)):
            init[f"h{kind}{s}"] = w(A * c, width, 1, 1, scale=0.4)
            b = w(A * c, scale=0.2)
            if kind == "conf":           # a face logit bias so random weights fire a few priors
                b[1::2] += 0.6
            init[f"hb{kind}{s}"] = b
            nodes += [N("Conv", [prev, f"h{kind}{s}", f"hb{kind}{s}"], [f"o{kind}{s}"], attrs={"kernel_shape": [1, 1]}),
                      N("Transpose", [f"o{kind}{s}"], [f"t{kind}{s}"], attrs={"perm": [0, 2, 3, 1]}),
                      N("Reshape", [f"t{kind}{s}", f"shape{c}"], [f"{kind}{s}"])]
            flat[kind].append(f"{kind}{s}")
    for kind in flat:
        nodes.append(N("Concat", flat[kind], [f"{kind}_raw"], attrs={"axis": 1}))
    nodes.append(N("Softmax", ["conf_raw"], ["conf"], attrs={"axis": -1}))
    if encoding == "priors":
        nodes += [N("Identity", ["loc_raw"], ["loc"]), N("Identity", ["landms_raw"], ["landms"])]
        return ox.Graph(nodes, init, ["x"], ["loc", "conf", "landms"])
    # in-graph decode: centre in [0, S), half-size in [4, 4 + S / 4): corner boxes in input pixels;
    # landmarks spread around the centre; face score = the softmax's face column
    S = float(size)
    init.update({"s0": np.array([0], np.int64), "s2": np.array([2], np.int64), "s4": np.array([4], np.int64),
                 "s1": np.array([1], np.int64), "ax": np.array([-1], np.int64), "S": np.array([S], np.float32),
                 "hs": np.array([S / 4], np.float32), "h0": np.array([4.0], np.float32),
                 "lscale": np.array([S / 3], np.float32), "shape_sc": np.array([0, -1], np.int64)})
    nodes += [N("Slice", ["loc_raw", "s0", "s2", "ax"], ["lc"]),
              N("Slice", ["loc_raw", "s2", "s4", "ax"], ["lw"]),
              N("Sigmoid", ["lc"], ["lcs"]), N("Mul", ["lcs", "S"], ["ctr"]),
              N("Sigmoid", ["lw"], ["lws"]), N("Mul", ["lws", "hs"], ["lwh"]), N("Add", ["lwh", "h0"], ["half"]),
              N("Sub", ["ctr", "half"], ["tl"]), N("Add", ["ctr", "half"], ["br"]),
              N("Concat", ["tl", "br"], ["boxes"], attrs={"axis": -1}),
              N("Slice", ["conf", "s1", "s2", "ax"], ["fc"]), N("Reshape", ["fc", "shape_sc"], ["scores"]),
              N("Tanh", ["landms_raw"], ["lt"]), N("Mul", ["lt", "lscale"], ["lo"]),
              N("Concat", ["ctr", "ctr", "ctr", "ctr", "ctr"], ["ctr5"], attrs={"axis": -1}),
              N("Add", ["ctr5", "lo"], ["landmarks"])]
    return ox.Graph(nodes, init, ["x"], ["boxes", "scores", "landmarks"])


def arcface_graph(seed: int = 1, dim: int = 512) -> ox.Graph:
    rng = np.random.default_rng(seed)
    N = ox.Node
    init = {"w0": (rng.standard_normal((32, 3, 3, 3)) * 0.3).astype(np.float32),
            "a0": np.full(32, 0.25, np.float32), "fc": (rng.standard_normal((dim, 32)) * 0.3).astype(np.float32),
            "fcb": (rng.standard_normal(dim) * 0.3).astype(np.float32)}
    nodes = [N("Conv", ["data", "w0"], ["c0"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "strides": [2, 2]}),
             N("PRelu", ["c0", "a0"], ["p0"]), N("GlobalAveragePool", ["p0"], ["g"]), N("Flatten", ["g"], ["f"]),
             N("Gemm", ["f", "fc", "fcb"], ["emb"], attrs={"transB": 1})]
    return ox.Graph(nodes, init, ["data"], ["emb"])


def detection_spec(size: int, encoding: str) -> dict:
    """The ``extra_metadata.insightface.detection`` block of such a pack."""
    d = {"type": "retinaface", "input_size": [size, size], "box_encoding": encoding,
         "mean": [104.0, 117.0, 123.0], "std": [1.0, 1.0, 1.0], "color_order": "bgr"}
    if encoding == "priors":
        d.update({"outputs": {"boxes": 0, "scores": 1, "landmarks": 2}, "steps": list(STEPS),
                  "min_sizes": [list(m) for m in MIN_SIZES], "variance": [0.1, 0.2]})
    else:
        d.update({"outputs": {"boxes": 0, "scores": 1, "landmarks": 2}, "normalized_boxes": False})
    return d


def write_retinaface_pack(root: Path, encoding: str = "priors", size: int = 64, seed: int = 0) -> Path:
    """``<root>/onnx/{detection,recognition}.fp32.onnx`` + model_info.json (type "retinaface")."""
    root = Path(root)
    (root / "onnx").mkdir(parents=True, exist_ok=True)
    (root / "onnx" / "detection.fp32.onnx").write_bytes(ox.write_model(retinaface_graph(size, encoding, seed)))
    (root / "onnx" / "recognition.fp32.onnx").write_bytes(ox.write_model(arcface_graph(seed + 1)))
    files = ["onnx/detection.fp32.onnx", "onnx/recognition.fp32.onnx"]
    info = {"name": root.name, "version": "1.0.0",
            "description": f"synthetic RetinaFace-shaped ONNX face pack ({encoding} boxes), random init",
            "model_type": "face", "embedding_dim": 512, "source": {"format": "custom", "repo_id": "synthetic/retinaface"},
            "runtimes": {"onnx": {"available": True, "files": files, "devices": ["cpu", "cuda"]}},
            "extra_metadata": {"insightface": {"detection": detection_spec(size, encoding)}}}
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info))
    return root
