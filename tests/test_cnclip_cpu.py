"""Chinese-CLIP (the reference's default general CLIP: CN-CLIP_ViT-B-16 / L-14): our BERT
text tower + ViT vision tower loaded from HF ``ChineseCLIPModel`` weights must reproduce
transformers' get_text_features / get_image_features (random-init tiny config, fp32, CPU
reference path; the GPU kernels are checked against this path in test_clip_gpu.py)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from lumen_amd.models.clip import BertConfig, CLIPConfig, CLIPModel, TextConfig, VisionConfig, \
    export_chinese_clip_state_dict  # noqa: E402


def _feat(out):
    """transformers >= 5 returns a ModelOutput whose pooler_output is the projected feature."""
    return out if isinstance(out, torch.Tensor) else out.pooler_output


def _pair(seed=0):
    from transformers import ChineseCLIPConfig, ChineseCLIPModel

    torch.manual_seed(seed)
    tc = dict(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
              max_position_embeddings=64)
    vc = dict(image_size=32, patch_size=8, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
              intermediate_size=128)
    hf = ChineseCLIPModel(ChineseCLIPConfig(text_config=tc, vision_config=vc, projection_dim=32)).eval()
    cfg = CLIPConfig(embed_dim=32, vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=4,
                                                       mlp_ratio=2.0, act="quick_gelu"),
                     text=TextConfig(), text_arch="bert",
                     bert=BertConfig(vocab_size=300, width=64, layers=2, heads=4, intermediate=128, max_position=64,
                                     context_length=20))
    m = CLIPModel(cfg, dtype=torch.float32, device="cpu")
    m.load_state_dict_any({k: v.clone() for k, v in hf.state_dict().items()})
    return hf, m


def test_cn_clip_text_matches_transformers():
    hf, m = _pair()
    ids = torch.randint(1, 300, (3, 20), generator=torch.Generator().manual_seed(1))
    ids[0, 12:] = 0          # right padding (pad id 0)
    ids[1, 5:] = 0
    mask = (ids != 0).long()
    with torch.no_grad():
        ref = _feat(hf.get_text_features(input_ids=ids, attention_mask=mask, token_type_ids=torch.zeros_like(ids)))
    ref = ref / ref.norm(dim=-1, keepdim=True)
    got = m.encode_text_ids(ids)
    assert torch.allclose(got, ref, atol=2e-5), (got - ref).abs().max()


def test_cn_clip_image_matches_transformers():
    hf, m = _pair(1)
    pix = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        ref = _feat(hf.get_image_features(pixel_values=pix))
    ref = ref / ref.norm(dim=-1, keepdim=True)
    got = m.visual.forward_patches(m.visual.preprocess_nchw_to_patches(pix), 2)
    assert torch.allclose(got, ref, atol=2e-5), (got - ref).abs().max()


def test_cn_clip_export_roundtrip():
    cfg = CLIPConfig(embed_dim=32, vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=1, heads=2),
                     text_arch="bert", bert=BertConfig(vocab_size=100, width=64, layers=1, heads=2, intermediate=128,
                                                       max_position=32, context_length=16))
    a = CLIPModel.random(cfg, seed=3, dtype=torch.float32)
    b = CLIPModel(cfg, dtype=torch.float32, device="cpu")
    b.load_state_dict_any(export_chinese_clip_state_dict(a))
    ids = torch.randint(1, 100, (2, 16), generator=torch.Generator().manual_seed(0))
    assert torch.allclose(a.encode_text_ids(ids), b.encode_text_ids(ids), atol=1e-6)
    assert CLIPConfig.from_dict(cfg.to_dict()).bert == cfg.bert


def test_cn_clip_backend_end_to_end(tmp_path):
    """Synthetic CN-CLIP directory (HF ChineseCLIP layout + WordPiece tokenizer) through the
    CLIP backend: config detection, 52-token [CLS]..[SEP] + [PAD] tokenisation, text/image
    embeddings and zero-shot classification against the label bank."""
    import numpy as np

    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.services.clip.backend import MI355XClipBackend
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    name = "CN-CLIP_ViT-B-16-tiny"
    write_clip_model(tmp_path / "models" / name, name, dataset="ImageNet_1k", n_labels=12)
    res = ResourceLoader.load_model_resources(tmp_path, ModelConfig(model=name, runtime=Runtime.torch,
                                                                    dataset="ImageNet_1k"))
    cfg = res.clip_config()
    assert cfg.text_arch == "bert" and cfg.context_length == 16
    be = MI355XClipBackend(res, device="cpu")
    be.initialize()
    try:
        ids = be.tokenize(["一只猫", "a photo of 狗"])
        assert ids.shape == (2, 16)
        assert int(ids[0, 0]) == 2 and int(ids[0, 4]) == 3 and int(ids[0, 5]) == 0   # [CLS] 一 只 猫 [SEP] [PAD]
        t = be.text_batch_to_vectors(["一只猫", "a photo of 狗"])
        assert t.shape == (2, cfg.embed_dim) and np.allclose(np.linalg.norm(t, axis=1), 1, atol=1e-4)
        # padding must not change the embedding: same text alone vs in a batch with a longer one
        assert np.allclose(be.text_batch_to_vectors(["一只猫"])[0], t[0], atol=1e-5)
        img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (40, 48, 3), dtype=np.uint8))
        v = be.image_to_vector(img)
        assert v.shape == (cfg.embed_dim,)
    finally:
        be.close()
