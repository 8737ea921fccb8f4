"""ONNX graph executor on the MI355X kernels (NHWC conv / depthwise / pooling / resize /
fused BN-activation-residual) vs its fp32 CPU reference path."""
import pytest
import torch

from lumen_amd.runtime.onnx_graph import OnnxGraph
from lumen_amd.utils import onnx_lite as ox

from test_onnx_cpu import detnet_graph, resnet_graph

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float().cpu() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("build", [resnet_graph, detnet_graph])
def test_onnx_executor_gpu_matches_cpu(build):
    g, _ = build()
    data = ox.write_model(g)
    x = torch.randn(2, 3, 32, 32)
    ref = OnnxGraph(data).run({"x": x})
    gpu = OnnxGraph(data, device="cuda")
    assert any(k == "conv" and s["mode"] in ("dense", "dw") for k, s in gpu.plan)
    got = gpu.run({"x": x.cuda()})
    for a, b in zip(got, ref):
        if b.is_floating_point():
            assert _rel(a, b) < 3e-2, _rel(a, b)
        else:
            assert a.cpu().tolist() == b.tolist()


def test_ocrnet_graph_gpu_all_hip():
    """Asymmetric padding, grouped conv, ConvTranspose, bilinear Resize, LayerNorm (subgraph + op),
    attention MatMuls, Softmax, broadcast / unary ops on the GPU path vs the CPU reference; the plan
    uses the HIP forms (no torch conv fallbacks)."""
    from test_onnx_cpu import ocrnet_graph

    g, _ = ocrnet_graph()
    data = ox.write_model(g)
    x = torch.randn(1, 3, 20, 28)
    ref = OnnxGraph(data).run({"x": x})
    gpu = OnnxGraph(data, device="cuda")
    kinds = [k for k, _ in gpu.plan]
    assert "convt" in kinds and "ln" in kinds
    assert all(s["mode"] != "ref" for k, s in gpu.plan if k == "conv")
    got = gpu.run({"x": x.cuda()})
    for a, b in zip(got, ref):
        assert _rel(a, b) < 3e-2, _rel(a, b)


def test_torch_tier_nodes_are_reported_at_load_and_counted():
    """A compute node with no HIP path (AveragePool) is listed when the graph is loaded, counted
    when it runs on the torch tier, and refused with strict=True; the HIP-covered graphs report
    nothing."""
    import numpy as np

    N = ox.Node
    g = ox.Graph(nodes=[N("Conv", ["x", "w"], ["c"], attrs={"kernel_shape": [3, 3], "pads": [1, 1, 1, 1]}),
                        N("AveragePool", ["c"], ["y"], attrs={"kernel_shape": [2, 2], "strides": [2, 2]})],
                 initializers={"w": (np.random.default_rng(0).standard_normal((16, 8, 3, 3)) * 0.1).astype(np.float32)},
                 inputs=["x"], outputs=["y"])
    data = ox.write_model(g)
    gpu = OnnxGraph(data, device="cuda")
    assert [op for op, _ in gpu.fallback_nodes] == ["AveragePool"]
    x = torch.randn(1, 8, 16, 16)
    got = gpu.run({"x": x.cuda()})[0]
    ref = OnnxGraph(data).run({"x": x})[0]
    assert _rel(got, ref) < 3e-2
    assert gpu.fallback_counts == {"AveragePool": 1}
    with pytest.raises(NotImplementedError, match="AveragePool"):
        OnnxGraph(data, device="cuda", strict=True)
    g2, _ = resnet_graph()
    assert OnnxGraph(ox.write_model(g2), device="cuda").fallback_nodes == []
