"""Weight-only fp8 (OCP e4m3fn, per-row scales): quantizer and the CPU reference path of
ops.linear / LLM.quantize_fp8 (the GPU kernels are checked against this in test_fp8_gpu.py)."""
import torch

from lumen_amd import ops
from lumen_amd.models.llm import LLM, LLM_PRESETS


def test_quantize_rows_error_bound():
    w = torch.randn(64, 256) * torch.logspace(-3, 1, 64)[:, None]   # rows of very different scale
    w8, s = ops.quantize_fp8_rows(w)
    assert w8.dtype == torch.float8_e4m3fn and s.shape == (64,)
    deq = w8.float() * s[:, None]
    rel = ((deq - w).norm(dim=1) / w.norm(dim=1)).max().item()
    assert rel < 0.04, rel                                    # e4m3: 3 mantissa bits
    assert (w8.float().abs().amax(dim=1) <= 448).all()


def test_linear_fp8_reference_matches_dequantized():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 128, generator=g)
    w = torch.randn(48, 128, generator=g)
    b = torch.randn(48, generator=g)
    w8, s = ops.quantize_fp8_rows(w)
    y = ops.linear(x, w8, b, act="gelu", w_scale=s)
    ref = ops.linear(x, w8.float() * s[:, None], b, act="gelu")
    assert torch.allclose(y, ref, atol=1e-6)


def test_llm_fp8_close_to_bf16_weights():
    cfg = LLM_PRESETS["tiny"]
    m = LLM(cfg, dtype=torch.float32, device="cpu")
    m.random_init(1)
    ids = torch.randint(0, cfg.vocab_size, (24,), generator=torch.Generator().manual_seed(3))
    ref = m.prefill(m.embed_tokens(ids))
    m.quantize_fp8()
    assert m.layers[0].qkv_w.dtype == torch.float8_e4m3fn and m.weight_dtype == "fp8"
    got = m.prefill(m.embed_tokens(ids))
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.98, cos       # e4m3 per-channel weights on a random-init model


def test_llm_w8a8_prefill_close_to_bf16_weights():
    """>= 33 prompt tokens: the fp8 model's prefill quantises activations per token (W8A8,
    RMSNorm+quant / row-quant producers); still close to the unquantised model."""
    from lumen_amd.models import llm as llm_mod

    cfg = LLM_PRESETS["tiny"]
    m = LLM(cfg, dtype=torch.float32, device="cpu")
    m.random_init(4)
    ids = torch.randint(0, cfg.vocab_size, (64,), generator=torch.Generator().manual_seed(5))
    ref = m.prefill(m.embed_tokens(ids))
    m.quantize_fp8()
    assert m._f8_ok(64) and not m._f8_ok(llm_mod._F8_MIN_ROWS - 1)
    got = m.prefill(m.embed_tokens(ids))
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.97, cos
