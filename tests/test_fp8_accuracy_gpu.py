"""Accuracy pins of the fp8 shortcuts in the VLM time-to-first-token path, at FULL model size
(random-init weights of the real architectures; the reference has no fp8 path to compare with,
so the pin is against this framework's own bf16 path on the same weights):

* the W8A8 MX vision chain (clip.run_blocks_mx, on by default for fp8 VLMs) on the 24-layer
  LLaVA ViT-L/14-336 tower, 577 tokens per image, penultimate-layer features (what LLaVA feeds the
  projector): per-token cosine >= 0.99 against the bf16 tower;
* the Llama-3-8B W8A8 prefill (LLM.quantize_fp8: fp8 weights, per-token fp8 activations on the
  block-scaled matrix cores) at a 624-token prompt: last-token logits cosine >= 0.97 against bf16
  and the fp8 first token among the bf16 top-5 (random-init logits are close to one another;
  measured r5: cosine 0.981).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_vit_l14_336_w8a8_full_depth_matches_bf16():
    from lumen_amd.models.clip import VisionTower
    from lumen_amd.models.vlm import VLM_PRESETS

    cfg = VLM_PRESETS["llava-llama3-8b"].vision
    assert (cfg.image_size, cfg.patch_size, cfg.width, cfg.layers) == (336, 14, 1024, 24)
    v = VisionTower(cfg, 16, torch.bfloat16, DEV)
    v.random_init(torch.Generator().manual_seed(0))
    g = torch.Generator().manual_seed(1)
    imgs = [torch.randint(0, 256, (336, 336, 3), dtype=torch.uint8, generator=g).to(DEV) for _ in range(2)]
    with torch.no_grad():
        patches = v.preprocess(imgs, (0.48145466, 0.4578275, 0.40821073), (0.26862954, 0.26130258, 0.27577711))
        ref = v.forward_features(patches, 2, -2).float()
        v.w8a8 = True
        got = v.forward_features(patches, 2, -2).float()
    assert got.shape == ref.shape and got.shape[-1] == 1024 and got.numel() // 1024 >= 2 * 576
    cos = torch.nn.functional.cosine_similarity(got.reshape(-1, 1024), ref.reshape(-1, 1024))
    assert cos.min().item() >= 0.99, (cos.min().item(), cos.mean().item())


def test_llama3_8b_w8a8_prefill_first_token():
    from lumen_amd.models.llm import LLM, LLM_PRESETS
    from lumen_amd.runtime.kv_cache import PagedKVCache

    cfg = LLM_PRESETS["llama3-8b"]
    m = LLM(cfg, dtype=torch.bfloat16, device=DEV)
    m.random_init(3)
    T = 624
    ids = torch.randint(0, cfg.vocab_size, (T,), generator=torch.Generator().manual_seed(2)).to(DEV)
    logits = []
    with torch.no_grad():
        for fp8 in (False, True):
            if fp8:
                m.quantize_fp8()
            kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=16, device=DEV, dtype=torch.bfloat16)
            kv.blocks.reserve(1, T)
            slots = torch.from_numpy(kv.slots(1, 0, T)).to(DEV)
            logits.append(m.prefill(m.embed_tokens(ids), kv, slots).float().cpu().flatten())
    ref, got = logits
    cos = torch.nn.functional.cosine_similarity(ref, got, dim=0).item()
    assert cos >= 0.97, cos
    top5 = set(torch.topk(ref, 5).indices.tolist())
    assert int(got.argmax()) in top5
