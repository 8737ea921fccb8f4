"""CLIP towers on the GPU (HIP kernels) vs the CPU fp32 reference path."""
import pytest
import torch

from lumen_amd.models.clip import CLIPModel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset", ["tiny", "ViT-B-32"])
def test_clip_image_text_gpu_matches_cpu(preset):
    m_cpu = CLIPModel.random(preset, seed=3, dtype=torch.float32)
    m_gpu = CLIPModel.random(preset, seed=3, dtype=torch.bfloat16, device="cuda")
    s = m_cpu.cfg.vision.image_size
    imgs = torch.randint(0, 256, (4, s + 13, s + 7, 3), dtype=torch.uint8)
    e_ref = m_cpu.encode_image_uint8(imgs)
    e = m_gpu.encode_image_uint8(imgs.cuda()).cpu()
    assert torch.allclose(e.norm(dim=-1), torch.ones(4), atol=1e-3)
    cos = (e * e_ref).sum(-1)
    assert cos.min().item() > 0.995, cos
    ctx = m_cpu.cfg.text.context_length
    ids = torch.randint(1, 400, (3, ctx))
    ids[:, 5] = m_cpu.cfg.text.vocab_size - 1
    t_ref = m_cpu.encode_text_ids(ids)
    t = m_gpu.encode_text_ids(ids.cuda()).cpu()
    assert (t * t_ref).sum(-1).min().item() > 0.995


def test_vit_l14_batch_runs():
    m = CLIPModel.random("ViT-L-14", seed=0, device="cuda", with_text=False)
    imgs = torch.randint(0, 256, (8, 256, 256, 3), dtype=torch.uint8, device="cuda")
    e = m.encode_image_uint8(imgs)
    assert e.shape == (8, 768) and torch.isfinite(e).all()
    # batch invariance: an image's embedding does not depend on its batch mates
    e1 = m.encode_image_uint8(imgs[:1])
    assert (e1[0] * e[0]).sum().item() > 0.999


@pytest.mark.parametrize("preset", ["cn-tiny", "CN-ViT-B-16"])
def test_cn_clip_bert_text_gpu_matches_cpu(preset):
    """Chinese-CLIP BERT text tower (post-LN, padded key lengths, CLS pooling) on the HIP
    kernels vs the CPU fp32 path; right-padded rows of different lengths in one batch."""
    m_cpu = CLIPModel.random(preset, seed=5, dtype=torch.float32)
    m_gpu = CLIPModel.random(preset, seed=5, dtype=torch.bfloat16, device="cuda")
    c = m_cpu.cfg.bert
    ids = torch.randint(5, c.vocab_size, (5, c.context_length), generator=torch.Generator().manual_seed(0))
    ids[:, 0] = 2
    for i, n in enumerate([c.context_length, 3, 7, 1, c.context_length // 2]):
        ids[i, n:] = 0
    t_ref = m_cpu.encode_text_ids(ids)
    t = m_gpu.encode_text_ids(ids.cuda()).float().cpu()
    cos = (t * t_ref).sum(-1)
    assert cos.min().item() > 0.995, cos
    # a row's embedding is independent of its batch mates' lengths
    t1 = m_gpu.encode_text_ids(ids[1:2].cuda()).float().cpu()
    assert (t1[0] * t[1]).sum().item() > 0.999


@pytest.mark.parametrize("n", [2, 3])
def test_vit_micro_batch_streams_match(monkeypatch, n):
    """Micro-batched image tower (row ranges on separate HIP streams, layer-interleaved,
    GEMMs without the tail split) vs the single-stream tower and the CPU fp32 reference."""
    import lumen_amd.models.clip as clip_mod

    m_cpu = CLIPModel.random("ViT-B-32", seed=5, dtype=torch.float32)
    m_gpu = CLIPModel.random("ViT-B-32", seed=5, dtype=torch.bfloat16, device="cuda")
    imgs = torch.randint(0, 256, (37, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(3))
    e_ref = m_cpu.encode_image_uint8(imgs[:8])
    monkeypatch.setattr(clip_mod, "_VIT_MICRO", 1)
    e1 = m_gpu.encode_image_uint8(imgs.cuda()).cpu()
    monkeypatch.setattr(clip_mod, "_VIT_MICRO", n)
    monkeypatch.setattr(clip_mod, "_VIT_MICRO_MIN_ROWS", 0)
    e2 = m_gpu.encode_image_uint8(imgs.cuda()).cpu()
    torch.cuda.synchronize()
    assert (e1 * e2).sum(-1).min().item() > 0.9995
    assert (e2[:8] * e_ref).sum(-1).min().item() > 0.995


def test_text_micro_batch_streams_match(monkeypatch):
    """Text tower (causal) micro-batched over 2 streams == single stream, and vs the CPU reference."""
    import lumen_amd.models.clip as clip_mod

    m_cpu = CLIPModel.random("ViT-B-32", seed=6, dtype=torch.float32)
    m_gpu = CLIPModel.random("ViT-B-32", seed=6, dtype=torch.bfloat16, device="cuda")
    ids = torch.randint(1, 4000, (41, 77), generator=torch.Generator().manual_seed(4))
    ids[:, 20] = m_cpu.cfg.text.vocab_size - 1
    t_ref = m_cpu.encode_text_ids(ids[:6])
    monkeypatch.setattr(clip_mod, "_TEXT_MICRO_MIN_ROWS", 1 << 30)
    t1 = m_gpu.encode_text_ids(ids.cuda()).cpu()
    monkeypatch.setattr(clip_mod, "_TEXT_MICRO_MIN_ROWS", 0)
    t2 = m_gpu.encode_text_ids(ids.cuda()).cpu()
    assert (t1 * t2).sum(-1).min().item() > 0.9995
    assert (t2[:6] * t_ref).sum(-1).min().item() > 0.995
