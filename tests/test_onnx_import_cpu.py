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
