"""FastViT / MobileCLIP2 towers on the HIP kernels vs the CPU fp32 reference path."""
import pytest
import torch

from lumen_amd.models.clip import CLIPModel
from lumen_amd.models.fastvit import FASTVIT_PRESETS, FastViTTower

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset", ["tiny", "tiny-ln"])
def test_fastvit_tower_gpu_matches_cpu(preset):
    c = FASTVIT_PRESETS[preset]
    cpu = FastViTTower(c, embed_dim=64, dtype=torch.float32)
    cpu.random_init(torch.Generator().manual_seed(3))
    gpu = FastViTTower(c, embed_dim=64, dtype=torch.bfloat16)
    gpu.load_timm(cpu.export_timm())
    gpu = gpu.cuda()
    x = torch.randn(3, c.image_size, c.image_size, 3, generator=torch.Generator().manual_seed(4))
    x8 = torch.nn.functional.pad(x, (0, 5))
    ref = cpu.forward_embed(x8)
    got = gpu.forward_embed(x8.cuda().bfloat16()).float().cpu()
    cos = (got * ref).sum(-1)
    assert cos.min().item() > 0.99, cos


def test_mobileclip2_s2_full_size():
    m = CLIPModel.random("MobileCLIP2-S2", seed=0, device="cuda")
    imgs = torch.randint(0, 256, (8, 300, 280, 3), dtype=torch.uint8, device="cuda")
    e = m.encode_image_uint8(imgs)
    assert e.shape == (8, 512) and torch.isfinite(e).all()
    e1 = m.encode_image_uint8(imgs[2:3])
    assert (e1[0] * e[2]).sum().item() > 0.995
    ids = torch.randint(1, 49000, (4, 77), device="cuda")
    ids[:, 10] = 49407
    t = m.encode_text_ids(ids)
    assert t.shape == (4, 512) and torch.isfinite(t).all()


def test_fastvlm_05b_vision_full_size():
    """FastViTHD at 1024 px on the HIP kernels: 256 tokens x 3072 -> projector (896)."""
    from lumen_amd.models.vlm import VLM, VLM_PRESETS

    cfg = VLM_PRESETS["fastvlm-0.5b"]
    m = VLM(cfg, device="cuda")
    m.random_init(0)
    imgs = [torch.randint(0, 256, (768, 1024, 3), dtype=torch.uint8, device="cuda"),
            torch.randint(0, 256, (1024, 1024, 3), dtype=torch.uint8, device="cuda")]
    e = m.encode_images(imgs)
    assert e.shape == (512, cfg.llm.hidden_size) and torch.isfinite(e).all()
    e1 = m.encode_images(imgs[1:])
    assert torch.allclose(e1.float(), e[256:].float(), atol=5e-2, rtol=5e-2)


def test_tiny_fastvlm_gpu_matches_cpu():
    from lumen_amd.models.vlm import VLM, VLM_PRESETS

    cfg = VLM_PRESETS["tiny-fastvit"]
    cpu = VLM(cfg, dtype=torch.float32, device="cpu")
    cpu.random_init(0)
    gpu = VLM(cfg, device="cuda")
    gpu.load_pack_state_dict({k: v.cuda() for k, v in cpu.export_state_dict().items()})
    imgs = [torch.randint(0, 256, (40, 70, 3), dtype=torch.uint8)]
    ref = cpu.encode_images(imgs)
    got = gpu.encode_images([i.cuda() for i in imgs]).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert cos.min().item() > 0.99, cos
