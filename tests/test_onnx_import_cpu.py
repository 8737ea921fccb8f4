"""ONNX pack ingestion for CLIP and FastVLM (reference defaults: CLIP onnxrt_backend.py:140-289,
FastVLM onnxrt_backend.py:55-160 / 538-659).  Synthetic packs are written the way
torch.onnx.export lays out initializers (Linear weights folded to ``onnx::MatMul_<n>``,
everything else by parameter name) and must give the same embeddings / tokens as the
safetensors packs of the same weights.  Parity against real reference-exported files is
unpinned (no packs offline)."""
import json

import numpy as np
import pytest
import torch

from lumen_amd.utils import onnx_import, onnx_lite


def _linear_keys(sd):
    return [k for k, v in sd.items() if getattr(v, "dim", lambda: 0)() == 2 and
            (k.endswith("in_proj_weight") or k.endswith(("out_proj.weight", "c_fc.weight", "c_proj.weight")))]


def _write_clip_onnx(root, fp16=False):
    from safetensors.torch import load_file

    sd = load_file(str(root / "model.safetensors"))
    vis = {k: v.float() for k, v in sd.items() if k.startswith("visual.")}
    txt = {k: v.float() for k, v in sd.items() if not k.startswith("visual.") and k != "logit_scale"}
    (root / "onnx").mkdir(exist_ok=True)
    suf = ".fp16" if fp16 else ""
    onnx_import.export_like_torch(vis, _linear_keys(vis), root / "onnx" / f"vision{suf}.onnx", "pixel_values",
                                  fp16=fp16)
    onnx_import.export_like_torch(txt, _linear_keys(txt), root / "onnx" / f"text{suf}.onnx", "input_ids",
                                  fp16=fp16)


@pytest.mark.parametrize("fp16", [False, True])
def test_clip_onnx_pack_matches_safetensors(tmp_path, fp16):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.services.clip.backend import create_backend
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    src = tmp_path / "models" / "clip-tiny"
    write_clip_model(src, "clip-tiny", preset="tiny", dataset=None)
    settings = type("S", (), {"device": "cpu", "batch_size": 4})()
    # square images: the torch runtime's centre crop and the ONNX runtime's squash resize coincide
    imgs = [encode_jpeg(np.random.default_rng(i).integers(0, 255, (40, 40, 3), dtype=np.uint8)) for i in range(3)]

    def embed(root_cache, rt):
        res = ResourceLoader.load_model_resources(root_cache, ModelConfig(model="clip-tiny", runtime=rt))
        b = create_backend(settings, res, rt.value)
        b.initialize()
        try:
            return b.image_batch_to_vectors(imgs), b.text_batch_to_vectors(["a cat", "two dogs"])
        finally:
            b.close()

    ref_i, ref_t = embed(tmp_path, Runtime.torch)
    _write_clip_onnx(src, fp16)
    (src / "model.safetensors").unlink()                       # ONNX pack only
    got_i, got_t = embed(tmp_path, Runtime.onnx)
    tol = 2e-3 if fp16 else 1e-6                               # fp16 initializers vs bf16 safetensors
    np.testing.assert_allclose(got_i, ref_i, atol=tol)
    np.testing.assert_allclose(got_t, ref_t, atol=tol)


def test_scope_and_bias_name_recovery(tmp_path):
    """HF-style graph: q_proj recovered from its bias, o_proj (no bias) from the node scope,
    Gemm transB, and the one unscoped projection reported as unresolved."""
    rng = np.random.default_rng(0)
    q, o, p, gw = (rng.standard_normal(s).astype(np.float32) for s in ((8, 4), (4, 8), (6, 4), (5, 4)))
    nodes = [onnx_lite.Node("MatMul", ["x", "onnx::MatMul_1"], ["m1"], name="/vision_model/encoder/layers.0/self_attn/q_proj/MatMul"),
             onnx_lite.Node("Add", ["vision_model.encoder.layers.0.self_attn.q_proj.bias", "m1"], ["a1"], name="/a"),
             onnx_lite.Node("MatMul", ["a1", "onnx::MatMul_2"], ["m2"], name="/vision_model/encoder/layers.0/self_attn/o_proj/MatMul"),
             onnx_lite.Node("Gemm", ["m2", "onnx::Gemm_3", "head.bias"], ["g"], name="/head/Gemm", attrs={"transB": 1}),
             onnx_lite.Node("MatMul", ["g", "onnx::MatMul_4"], ["y"], name="")]
    inits = {"onnx::MatMul_1": q.T.copy(), "vision_model.encoder.layers.0.self_attn.q_proj.bias": np.zeros(8, np.float32),
             "onnx::MatMul_2": o.T.copy(), "onnx::Gemm_3": gw, "head.bias": np.zeros(5, np.float32),
             "onnx::MatMul_4": p.T.copy()}
    path = tmp_path / "g.onnx"
    path.write_bytes(onnx_lite.write_model(onnx_lite.Graph(nodes, inits, ["x"], ["y"])))
    sd, un = onnx_import.recover_state_dict(path)
    np.testing.assert_array_equal(sd["vision_model.encoder.layers.0.self_attn.q_proj.weight"], q)
    np.testing.assert_array_equal(sd["vision_model.encoder.layers.0.self_attn.o_proj.weight"], o)
    np.testing.assert_array_equal(sd["head.weight"], gw)
    assert len(un) == 1 and un[0][1].shape == (6, 4)
    np.testing.assert_array_equal(un[0][1], p)
    assert onnx_import._scope_to_param("/model/mm_projector/mm_projector.0/MatMul") == "model.mm_projector.0.weight"


def _write_vlm_onnx(root, m):
    """FastVLM pack (vision = FastViTHD trunk + projector, embed, decoder) from a VLM's weights."""
    (root / "onnx").mkdir(exist_ok=True)
    vis = {k: v.float() for k, v in m.vision.export_timm(prefix="model.vision_tower.vision_tower.model.").items()}
    vis["model.mm_projector.0.weight"] = m.proj1_w.float()
    vis["model.mm_projector.0.bias"] = m.proj1_b.float()
    vis["model.mm_projector.2.weight"] = m.proj2_w.float()
    vis["model.mm_projector.2.bias"] = m.proj2_b.float()
    onnx_import.export_like_torch(vis, ["model.mm_projector.0.weight", "model.mm_projector.2.weight"],
                                  root / "onnx" / "vision.onnx", "pixel_values")
    sd = {k: v.float() for k, v in m.export_state_dict().items() if k.startswith(("model.", "lm_head"))}
    emb = {"model.embed_tokens.weight": sd.pop("model.embed_tokens.weight")}
    onnx_import.export_like_torch(emb, [], root / "onnx" / "embed.onnx", "input_ids")
    lin = [k for k in sd if k.endswith("_proj.weight")]
    onnx_import.export_like_torch(sd, lin, root / "onnx" / "decoder.onnx", "inputs_embeds")


def test_fastvlm_onnx_pack_generates_same_tokens(tmp_path):
    from lumen_amd.models.vlm import VLM, write_vlm_model
    from lumen_amd.services.common import load_safetensors

    src = tmp_path / "models" / "fastvlm-tiny"
    write_vlm_model(src, "fastvlm-tiny", preset="tiny-fastvit", weights=True)
    cfgd = json.loads((src / "lumen_vlm_config.json").read_text())
    from lumen_amd.models.vlm import VLMConfig

    cfg = VLMConfig.from_dict(cfgd)
    ref = VLM(cfg, dtype=torch.float32, device="cpu")
    ref.load_pack_state_dict(load_safetensors(src / "model.safetensors"))
    _write_vlm_onnx(src, ref)
    got = VLM(cfg, dtype=torch.float32, device="cpu")
    onnx_import.load_vlm(got, *onnx_import.find_vlm_pack(src))
    for (ka, a), (kb, b) in zip(sorted(ref.state_dict().items()), sorted(got.state_dict().items())):
        assert ka == kb
        torch.testing.assert_close(a, b, rtol=0, atol=0, msg=ka)


def test_vlm_service_serves_onnx_pack(tmp_path):
    """A reference-style ``runtime: onnx`` FastVLM pack (no model.safetensors) starts and generates
    the same greedy tokens as the safetensors pack."""
    from lumen_amd.models.vlm import VLM, VLMConfig, write_vlm_model
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources, load_safetensors
    from lumen_amd.services.vlm.backend import ChatMessage, GenerationRequest, create_backend
    from lumen_amd.utils.image import encode_jpeg

    src = tmp_path / "models" / "fastvlm-tiny"
    write_vlm_model(src, "fastvlm-tiny", preset="tiny-fastvit", weights=True)
    img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (48, 64, 3), dtype=np.uint8))
    settings = type("S", (), {"device": "cpu", "batch_size": 1})()

    def run():
        res = load_model_resources(tmp_path, ModelConfig(model="fastvlm-tiny", runtime=Runtime.onnx))
        b = create_backend(settings, res, "onnx")
        b.initialize()
        try:
            req = GenerationRequest(messages=[ChatMessage("user", "describe")], image_bytes=img, max_new_tokens=6,
                                    temperature=0.0)
            return b.generate(req).tokens
        finally:
            b.close()

    ref = run()
    cfg = VLMConfig.from_dict(json.loads((src / "lumen_vlm_config.json").read_text()))
    m = VLM(cfg, dtype=torch.float32, device="cpu")
    m.load_pack_state_dict(load_safetensors(src / "model.safetensors"))
    _write_vlm_onnx(src, m)
    (src / "model.safetensors").unlink()
    info = json.loads((src / "model_info.json").read_text())
    files = [f for f in info["runtimes"]["onnx"]["files"] if f != "model.safetensors"]
    info["runtimes"]["onnx"]["files"] = files + ["onnx/vision.onnx", "onnx/embed.onnx", "onnx/decoder.onnx"]
    (src / "model_info.json").write_text(json.dumps(info))
    got = run()
    assert got == ref


# ----------------------------------------------------------------------------- quantised CLIP packs
def _quantize_pack(src_path, dst_path, mode):
    """Re-encode every generated MatMul weight of an exported graph the way ONNX Runtime's
    quantisers do: "qdq" (DequantizeLinear of an int8 per-channel initializer), "dynamic"
    (MatMulInteger + <w>_scale / <w>_zero_point, uint8 asymmetric per tensor), "q4"
    (com.microsoft MatMulNBits, 4-bit blocks of 32, fp16 scales, no zero points)."""
    from lumen_amd.utils import onnx_lite as ox

    m = ox.load_model(src_path)
    g = m.graph
    inits = dict(g.initializers)
    nodes = []
    for n in g.nodes:
        if n.op_type != "MatMul" or n.inputs[1] not in inits or not n.inputs[1].startswith("onnx::"):
            nodes.append(n)
            continue
        wname = n.inputs[1]
        B = np.asarray(inits.pop(wname), np.float32)          # [K, N]
        K, N = B.shape
        if mode == "qdq":
            sc = np.abs(B).max(0) / 127 + 1e-12                # per output column (axis 1)
            inits[wname + "_quantized"] = np.clip(np.round(B / sc), -127, 127).astype(np.int8)
            inits[wname + "_scale"] = sc.astype(np.float32)
            inits[wname + "_zero_point"] = np.zeros(N, np.int8)
            dq = wname + "_DequantizeLinear_Output"
            nodes.append(ox.Node("DequantizeLinear", [wname + "_quantized", wname + "_scale", wname + "_zero_point"],
                                 [dq], name=n.name + "_dq", attrs={"axis": 1}))
            nodes.append(ox.Node("MatMul", [n.inputs[0], dq], list(n.outputs), name=n.name))
        elif mode == "dynamic":
            lo, hi = min(B.min(), 0.0), max(B.max(), 0.0)
            sc = (hi - lo) / 255 + 1e-12
            zp = np.uint8(np.clip(np.round(-lo / sc), 0, 255))
            inits[wname + "_quantized"] = np.clip(np.round(B / sc) + zp, 0, 255).astype(np.uint8)
            inits[wname + "_scale"] = np.array(sc, np.float32)
            inits[wname + "_zero_point"] = np.array(zp, np.uint8)
            o = n.outputs[0]
            nodes += [ox.Node("DynamicQuantizeLinear", [n.inputs[0]], [o + "_xq", o + "_xs", o + "_xz"]),
                      ox.Node("MatMulInteger", [o + "_xq", wname + "_quantized", o + "_xz", wname + "_zero_point"],
                              [o + "_i32"], name=n.name + "_quant"),
                      ox.Node("Cast", [o + "_i32"], [o + "_f"], attrs={"to": 1}),
                      ox.Node("Mul", [o + "_xs", wname + "_scale"], [o + "_s"]),
                      ox.Node("Mul", [o + "_f", o + "_s"], [o])]
        else:
            bs = 32
            Wt = B.T                                            # [N, K]
            nb = -(-K // bs)
            Wp = np.zeros((N, nb * bs), np.float32)
            Wp[:, :K] = Wt
            blk = Wp.reshape(N, nb, bs)
            sc = np.abs(blk).max(-1) / 7 + 1e-12
            q = (np.clip(np.round(blk / sc[..., None]), -8, 7) + 8).astype(np.uint8)
            packed = (q[..., 0::2] | (q[..., 1::2] << 4)).astype(np.uint8)
            inits[wname + "_Q4"] = packed
            inits[wname + "_scales"] = sc.astype(np.float16).reshape(-1)
            nodes.append(ox.Node("MatMulNBits", [n.inputs[0], wname + "_Q4", wname + "_scales"], list(n.outputs),
                                 name=n.name, domain="com.microsoft",
                                 attrs={"K": K, "N": N, "bits": 4, "block_size": bs}))
    g2 = ox.Graph(nodes=nodes, initializers=inits, inputs=g.inputs, outputs=g.outputs, name=g.name)
    dst_path.write_bytes(ox.write_model(g2, opset=17))


@pytest.mark.parametrize("mode,prec,tol", [("qdq", "int8", 0.995), ("dynamic", "int8", 0.99), ("q4", "q4fp16", 0.97)])
def test_quantized_clip_pack_imports(tmp_path, mode, prec, tol):
    """vision/text.{int8,q4fp16}.onnx (QDQ, MatMulInteger dynamic, MatMulNBits 4-bit) load onto the
    native CLIP model: dequantised weights under their recovered names, embeddings close to the
    fp32 pack (quantisation error only)."""
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.services.clip.backend import create_backend
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    src = tmp_path / "models" / "clip-tiny"
    write_clip_model(src, "clip-tiny", preset="tiny", dataset=None)
    imgs = [encode_jpeg(np.random.default_rng(i).integers(0, 255, (40, 40, 3), dtype=np.uint8)) for i in range(3)]

    def embed(precision=None):
        settings = type("S", (), {"device": "cpu", "batch_size": 4})()
        res = ResourceLoader.load_model_resources(tmp_path, ModelConfig(model="clip-tiny", runtime=Runtime.onnx,
                                                                        precision=precision))
        b = create_backend(settings, res, "onnx", precision)
        b.initialize()
        try:
            return b.image_batch_to_vectors(imgs), b.text_batch_to_vectors(["a cat", "two dogs"])
        finally:
            b.close()

    _write_clip_onnx(src)
    (src / "model.safetensors").unlink()
    ref_i, ref_t = embed()
    for comp in ("vision", "text"):
        _quantize_pack(src / "onnx" / f"{comp}.onnx", src / "onnx" / f"{comp}.{prec}.onnx", mode)
    sd, unresolved = onnx_import.recover_state_dict(src / "onnx" / f"vision.{prec}.onnx")
    assert not any(k.endswith(("_quantized", "_Q4", "_scales")) for k in sd)
    got_i, got_t = embed(prec)
    for a, b in ((got_i, ref_i), (got_t, ref_t)):
        cos = [float(np.dot(x, y) / np.linalg.norm(x) / np.linalg.norm(y)) for x, y in zip(a, b)]
        assert min(cos) > tol, cos
