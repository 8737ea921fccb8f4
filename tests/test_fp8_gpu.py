"""fp8 (OCP e4m3fn) weight GEMMs on MI355X vs the fp32 reference of the dequantized weights:
decode-shaped split-K skinny kernel and the register-staged prefill kernel, with the
LLM epilogues (bias, SwiGLU, residual, fp32 out); the fp8 LLM vs its CPU reference."""
import pytest
import torch

from lumen_amd import ops
from lumen_amd.models.llm import LLM, LLM_PRESETS

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(1, 896, 896), (4, 4864, 896), (16, 896, 4864), (30, 1024, 14336),
                                   (100, 1024, 4096), (624, 4096, 4096), (700, 2048, 640)])
def test_gemm_w8_vs_dequantized(M, N, K):
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).bfloat16()
    w8, s = ops.quantize_fp8_rows(torch.randn(N, K, generator=g) * K ** -0.5)
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x.float(), w8, b, residual=r.float(), w_scale=s)
    got = ops.linear(x.to(DEV), w8.to(DEV), b.to(DEV), residual=r.to(DEV), w_scale=s.to(DEV))
    assert _rel(got, ref) < 1e-2
    ref32 = ops.linear(x.float(), w8, w_scale=s)
    got32 = ops.linear(x.to(DEV), w8.to(DEV), w_scale=s.to(DEV), out_dtype=torch.float32)
    assert got32.dtype == torch.float32 and _rel(got32, ref32) < 5e-3


@pytest.mark.parametrize("M", [3, 200])
def test_gemm_w8_swiglu(M):
    g = torch.Generator().manual_seed(M)
    I, K = 512, 896
    x = torch.randn(M, K, generator=g).bfloat16()
    gu = ops.glu_interleave(torch.randn(I, K, generator=g), torch.randn(I, K, generator=g)) * K ** -0.5
    w8, s = ops.quantize_fp8_rows(gu)
    ref = ops.linear(x.float(), w8, glu=True, w_scale=s)
    got = ops.linear(x.to(DEV), w8.to(DEV), glu=True, w_scale=s.to(DEV))
    assert got.shape == (M, I) and _rel(got, ref) < 1e-2


def test_llm_fp8_matches_cpu_reference():
    cfg = LLM_PRESETS["tiny"]
    cpu = LLM(cfg, dtype=torch.float32, device="cpu")
    cpu.random_init(2)
    gpu = LLM(cfg, device=DEV)
    gpu.load_state_dict({k: v.to(gpu.state_dict()[k].dtype) for k, v in cpu.state_dict().items()}, strict=False)
    cpu.quantize_fp8()
    gpu.quantize_fp8()
    ids = torch.randint(0, cfg.vocab_size, (40,), generator=torch.Generator().manual_seed(1))
    ref = cpu.prefill(cpu.embed_tokens(ids))
    got = gpu.prefill(gpu.embed_tokens(ids.to(DEV)))
    cos = torch.nn.functional.cosine_similarity(got.float().cpu().flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.99, cos
