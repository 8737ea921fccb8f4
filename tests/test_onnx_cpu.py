"""ONNX import: the wire-format reader/writer round-trips, and the graph executor's CPU
reference path matches a hand-written PyTorch forward of the same network.  GPU kernels
vs this CPU path: test_onnx_gpu.py.  (No onnx / onnxruntime package offline: graphs are
written by lumen_amd.utils.onnx_lite; parity against the reference's real model packs is
unpinned.)"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from lumen_amd.runtime.onnx_graph import OnnxGraph
from lumen_amd.utils import onnx_lite as ox

R = np.random.default_rng(0)


def _w(*s, scale=0.3):
    return (R.standard_normal(s) * scale).astype(np.float32)


def _bn(init, p, c):
    init[p + "_s"] = (1 + 0.1 * R.standard_normal(c)).astype(np.float32)
    init[p + "_b"] = (0.1 * R.standard_normal(c)).astype(np.float32)
    init[p + "_m"] = (0.1 * R.standard_normal(c)).astype(np.float32)
    init[p + "_v"] = (0.5 + R.random(c)).astype(np.float32)
    return [p + "_s", p + "_b", p + "_m", p + "_v"]


def resnet_graph():
    """IResNet-style: conv-BN-PReLU stem, pre-BN residual block, maxpool, GAP, Gemm."""
    N = ox.Node
    init = {"w0": _w(16, 3, 3, 3), "a0": np.full(16, 0.25, np.float32), "w1": _w(16, 16, 3, 3),
            "a1": np.full(16, 0.2, np.float32), "w2": _w(16, 16, 3, 3), "w3": _w(32, 16, 1, 1), "b3": _w(32),
            "fc": _w(64, 32), "fcb": _w(64)}
    nodes = [N("Conv", ["x", "w0"], ["c0"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1]}),
             N("BatchNormalization", ["c0"] + _bn(init, "bn0", 16), ["n0"], attrs={"epsilon": 1e-5}),
             N("PRelu", ["n0", "a0"], ["p0"]),
             N("BatchNormalization", ["p0"] + _bn(init, "bnpre", 16), ["q0"]),
             N("Conv", ["q0", "w1"], ["c1"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1]}),
             N("BatchNormalization", ["c1"] + _bn(init, "bn1", 16), ["n1"]),
             N("PRelu", ["n1", "a1"], ["p1"]),
             N("Conv", ["p1", "w2"], ["c2"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1]}),
             N("BatchNormalization", ["c2"] + _bn(init, "bn2", 16), ["n2"]),
             N("Add", ["n2", "p0"], ["r"]),
             N("MaxPool", ["r"], ["mp"], attrs={"kernel_shape": [2, 2], "strides": [2, 2]}),
             N("Conv", ["mp", "w3", "b3"], ["c3"], attrs={"kernel_shape": [1, 1]}),
             N("Relu", ["c3"], ["r3"]),
             N("GlobalAveragePool", ["r3"], ["g"]),
             N("Flatten", ["g"], ["f"], attrs={"axis": 1}),
             N("Gemm", ["f", "fc", "fcb"], ["y"], attrs={"transB": 1})]
    return ox.Graph(nodes, init, ["x"], ["y"]), init


def resnet_reference(x, i):
    t = {k: torch.from_numpy(v) for k, v in i.items()}

    def bn(z, p):
        return F.batch_norm(z, t[p + "_m"], t[p + "_v"], t[p + "_s"], t[p + "_b"], False, 0.0, 1e-5)

    def prelu(z, a):
        return torch.where(z > 0, z, z * t[a].view(1, -1, 1, 1))

    p0 = prelu(bn(F.conv2d(x, t["w0"], padding=1), "bn0"), "a0")
    q0 = bn(p0, "bnpre")
    p1 = prelu(bn(F.conv2d(q0, t["w1"], padding=1), "bn1"), "a1")
    r = bn(F.conv2d(p1, t["w2"], padding=1), "bn2") + p0
    mp = F.max_pool2d(r, 2, 2)
    r3 = F.relu(F.conv2d(mp, t["w3"], t["b3"]))
    f = r3.mean((2, 3))
    return f @ t["fc"].t() + t["fcb"]


def detnet_graph():
    """SCRFD / DBNet-style: strided convs, depthwise + relu6, SE (GAP-1x1-relu-1x1-hardsigmoid-mul),
    hardswish, FPN nearest x2 upsample + add, concat, sigmoid head -> NHWC reshape."""
    N = ox.Node
    init = {"w0": _w(16, 3, 3, 3), "b0": _w(16), "wd": _w(16, 1, 3, 3), "bd": _w(16), "w1": _w(24, 16, 1, 1),
            "w2": _w(24, 24, 3, 3), "b2": _w(24), "se1": _w(8, 24, 1, 1), "se1b": _w(8), "se2": _w(24, 8, 1, 1),
            "se2b": _w(24), "lat": _w(24, 24, 1, 1), "wh": _w(2, 48, 3, 3), "bh": _w(2),
            "shape": np.array([0, -1, 1], np.int64), "lo": np.array(0, np.float32), "hi": np.array(6, np.float32),
            "scales": np.array([1, 1, 2, 2], np.float32), "roi": np.zeros(0, np.float32),
            "wm": _w(48, 1, 3, 3), "bm": _w(48)}
    nodes = [N("Conv", ["x", "w0", "b0"], ["c0"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                          "strides": [2, 2]}),
             N("Relu", ["c0"], ["r0"]),
             N("Conv", ["r0", "wd", "bd"], ["d0"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "group": 16}),
             N("Clip", ["d0", "lo", "hi"], ["d1"]),
             N("Conv", ["d1", "w1"], ["c1"], attrs={"kernel_shape": [1, 1]}),
             N("BatchNormalization", ["c1"] + _bn(init, "bn1", 24), ["n1"]),
             N("HardSwish", ["n1"], ["h1"]),
             N("Conv", ["h1", "w2", "b2"], ["c2"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1],
                                                           "strides": [2, 2]}),
             N("LeakyRelu", ["c2"], ["l2"], attrs={"alpha": 0.1}),
             N("GlobalAveragePool", ["l2"], ["g"]),
             N("Conv", ["g", "se1", "se1b"], ["s1"], attrs={"kernel_shape": [1, 1]}),
             N("Relu", ["s1"], ["s2"]),
             N("Conv", ["s2", "se2", "se2b"], ["s3"], attrs={"kernel_shape": [1, 1]}),
             N("HardSigmoid", ["s3"], ["s4"], attrs={"alpha": 0.2, "beta": 0.5}),
             N("Mul", ["l2", "s4"], ["se"]),
             N("Resize", ["se", "roi", "scales"], ["up"], attrs={"mode": "nearest"}),
             N("Conv", ["h1", "lat"], ["lt"], attrs={"kernel_shape": [1, 1]}),
             N("Add", ["up", "lt"], ["fpn"]),
             N("Concat", ["fpn", "h1"], ["cat"], attrs={"axis": 1}),
             N("Conv", ["cat", "wm", "bm"], ["m"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "group": 48}),
             N("Conv", ["m", "wh", "bh"], ["hd"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1]}),
             N("Sigmoid", ["hd"], ["sg"]),
             N("Transpose", ["sg"], ["tp"], attrs={"perm": [0, 2, 3, 1]}),
             N("Reshape", ["tp", "shape"], ["y"]),
             N("Shape", ["fpn"], ["shp"])]
    return ox.Graph(nodes, init, ["x"], ["y", "fpn", "shp"]), init


def test_wire_format_roundtrip(tmp_path):
    g, init = resnet_graph()
    data = ox.write_model(g, opset=13)
    p = tmp_path / "m.onnx"
    p.write_bytes(data)
    m = ox.load_model(p)
    assert m.opset == 13 and [n.op_type for n in m.graph.nodes] == [n.op_type for n in g.nodes]
    assert m.graph.inputs == ["x"] and m.graph.outputs == ["y"]
    for k, v in init.items():
        np.testing.assert_array_equal(m.graph.initializers[k], v)
    conv = m.graph.nodes[0]
    assert conv.attrs["kernel_shape"] == [3, 3] and conv.attrs["pads"] == [1, 1, 1, 1]
    assert abs(m.graph.nodes[1].attrs["epsilon"] - 1e-5) < 1e-9
    assert set(ox.load_initializers(p)) == set(init)


def test_executor_matches_torch_reference():
    g, init = resnet_graph()
    x = torch.randn(2, 3, 16, 16)
    got = OnnxGraph(ox.write_model(g))
    y = got.run({"x": x})[0]
    assert torch.allclose(y, resnet_reference(x, init), atol=1e-4), (y - resnet_reference(x, init)).abs().max()
    # planning folded BN + PReLU / residual into the convs
    kinds = [k for k, _ in got.plan]
    assert kinds.count("conv") == 4 and len(got.plan) == 4 + 1 + 1 + 2 + 1   # + pre-BN, MaxPool, Relu..Gemm


def test_executor_detnet_shapes():
    g, _ = detnet_graph()
    ex = OnnxGraph(ox.write_model(g))
    y, fpn, shp = ex.run({"x": torch.randn(1, 3, 32, 32)})
    assert y.shape == (1, 16 * 16 * 2, 1) and fpn.shape == (1, 24, 16, 16)
    assert shp.tolist() == [1, 24, 16, 16]
    assert float(y.min()) >= 0 and float(y.max()) <= 1


def test_unsupported_op_is_loud():
    g = ox.Graph([ox.Node("NonMaxSuppression", ["x"], ["y"])], {}, ["x"], ["y"])
    with pytest.raises(NotImplementedError):
        OnnxGraph(ox.write_model(g)).run({"x": torch.zeros(1)})


def test_unsupported_op_fails_at_load():
    g = ox.Graph([ox.Node("Relu", ["x"], ["r"]), ox.Node("NonMaxSuppression", ["r"], ["y"]),
                  ox.Node("Einsum", ["r"], ["z"])], {}, ["x"], ["y", "z"])
    with pytest.raises(NotImplementedError, match="Einsum, NonMaxSuppression"):
        OnnxGraph(ox.write_model(g))


def ocrnet_graph():
    """PP-OCR-style coverage of the executor's remaining node kinds: asymmetric conv padding,
    grouped conv, ConvTranspose (k == s) + BN + ReLU, bilinear Resize, a decomposed LayerNorm
    subgraph, LayerNormalization, attention (MatMul of activations + Softmax), broadcast
    binary ops, unary ops, PRelu, Clip."""
    N = ox.Node
    init = {"w0": _w(32, 3, 3, 3), "b0": _w(32), "wg": _w(32, 16, 3, 3), "bg": _w(32),
            "wt": _w(32, 16, 2, 2), "bt": _w(16), "wq": _w(16, 16), "wk": _w(16, 16), "wv": _w(16, 16),
            "g1": (1 + 0.1 * R.standard_normal(16)).astype(np.float32), "be1": _w(16),
            "g2": (1 + 0.1 * R.standard_normal(16)).astype(np.float32), "be2": _w(16),
            "two": np.array(2.0, np.float32), "eps": np.array(1e-5, np.float32),
            "sc": np.array(0.25, np.float32), "sz": np.array([1, 16, 20, 28], np.int64),
            "roi": np.zeros(0, np.float32), "noscale": np.zeros(0, np.float32),
            "shp3": np.array([0, 16, -1], np.int64), "pr": np.full(16, 0.2, np.float32),
            "lo": np.array(-1.0, np.float32), "hi": np.array(2.0, np.float32)}
    nodes = [N("Conv", ["x", "w0", "b0"], ["c0"], attrs={"kernel_shape": [3, 3], "pads": [0, 0, 1, 1],
                                                          "strides": [2, 2]}),
             N("Relu", ["c0"], ["r0"]),
             N("Conv", ["r0", "wg", "bg"], ["cg"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "group": 2}),
             N("ConvTranspose", ["cg", "wt", "bt"], ["ct"], attrs={"kernel_shape": [2, 2], "strides": [2, 2]}),
             N("BatchNormalization", ["ct"] + _bn(init, "bnt", 16), ["btn"]),
             N("Relu", ["btn"], ["rt"]),
             N("Resize", ["rt", "roi", "noscale", "sz"], ["rs"], attrs={"mode": "linear",
                                                                       "coordinate_transformation_mode": "half_pixel"}),
             N("Reshape", ["rs", "shp3"], ["seq0"]),                  # [1, 16, 560]
             N("Transpose", ["seq0"], ["seq"], attrs={"perm": [0, 2, 1]}),   # [1, 560, 16]
             # decomposed LayerNorm
             N("ReduceMean", ["seq"], ["m"], attrs={"axes": [-1], "keepdims": 1}),
             N("Sub", ["seq", "m"], ["d"]),
             N("Pow", ["d", "two"], ["d2"]),
             N("ReduceMean", ["d2"], ["v"], attrs={"axes": [-1], "keepdims": 1}),
             N("Add", ["v", "eps"], ["ve"]),
             N("Sqrt", ["ve"], ["sd"]),
             N("Div", ["d", "sd"], ["nn"]),
             N("Mul", ["nn", "g1"], ["ng"]),
             N("Add", ["ng", "be1"], ["ln1"]),
             # attention
             N("MatMul", ["ln1", "wq"], ["q"]), N("MatMul", ["ln1", "wk"], ["k"]), N("MatMul", ["ln1", "wv"], ["vv"]),
             N("Transpose", ["k"], ["kt"], attrs={"perm": [0, 2, 1]}),
             N("MatMul", ["q", "kt"], ["qk"]),
             N("Mul", ["qk", "sc"], ["qks"]),
             N("Softmax", ["qks"], ["att"], attrs={"axis": -1}),
             N("MatMul", ["att", "vv"], ["ctx"]),
             N("Add", ["ctx", "ln1"], ["res"]),
             N("LayerNormalization", ["res", "g2", "be2"], ["ln2"], attrs={"axis": -1, "epsilon": 1e-5}),
             N("PRelu", ["ln2", "pr"], ["p"]),
             N("Clip", ["p", "lo", "hi"], ["cl"]),
             N("Tanh", ["cl"], ["th"]),
             N("HardSigmoid", ["th"], ["y"], attrs={"alpha": 0.2, "beta": 0.5})]
    return ox.Graph(nodes, init, ["x"], ["y", "ct"]), init


def test_ocrnet_graph_matches_torch():
    g, i = ocrnet_graph()
    x = torch.randn(1, 3, 20, 28)
    y, ct = OnnxGraph(ox.write_model(g)).run({"x": x})
    t = {k: torch.from_numpy(v) for k, v in i.items()}
    c0 = F.relu(F.conv2d(F.pad(x, (0, 1, 0, 1)), t["w0"], t["b0"], stride=2))
    cg = F.conv2d(c0, t["wg"], t["bg"], padding=1, groups=2)
    ct_ref = F.conv_transpose2d(cg, t["wt"], t["bt"], stride=2)
    torch.testing.assert_close(ct, ct_ref, rtol=1e-4, atol=1e-4)
    bt = F.relu(F.batch_norm(ct_ref, t["bnt_m"], t["bnt_v"], t["bnt_s"], t["bnt_b"], False, 0.0, 1e-5))
    rs = F.interpolate(bt, size=(20, 28), mode="bilinear", align_corners=False)
    seq = rs.reshape(1, 16, -1).transpose(1, 2)
    ln1 = F.layer_norm(seq, (16,), t["g1"], t["be1"], 1e-5)
    q, k, v = ln1 @ t["wq"], ln1 @ t["wk"], ln1 @ t["wv"]
    ctx = torch.softmax(q @ k.transpose(1, 2) * 0.25, -1) @ v
    ln2 = F.layer_norm(ctx + ln1, (16,), t["g2"], t["be2"], 1e-5)
    p = torch.where(ln2 > 0, ln2, ln2 * 0.2)
    ref = torch.clamp(torch.tanh(torch.clamp(p, -1, 2)) * 0.2 + 0.5, 0, 1)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
