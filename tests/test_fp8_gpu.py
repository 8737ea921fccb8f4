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
                                   (100, 1024, 4096), (624, 4096, 4096), (700, 2048, 640),
                                   (1, 28672, 4096), (13, 26640, 1024)])   # two tiles per workgroup
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


# ----------------------------------------------------------------------------- W8A8 (fp8 x fp8 MFMA)
def _f8_operands(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    x8, xs = ops.quant_rows_fp8(torch.randn(M, K, generator=g).bfloat16())
    w8, ws = ops.quantize_fp8_rows(torch.randn(N, K, generator=g) * K ** -0.5)
    return g, x8, xs, w8, ws


def test_gemm_f8_exact_small_integers():
    """Asymmetric integer operands (exact in e4m3 and in fp32 accumulation): catches any
    row/column swap or k-permutation mismatch between the A and W fragments."""
    M, N, K = 160, 144, 256
    a = (torch.arange(M)[:, None] * 3 + torch.arange(K)[None, :] * 5) % 7 - 3
    w = (torch.arange(N)[:, None] * 2 + torch.arange(K)[None, :] * 11) % 5 - 2
    a8, w8 = a.float().to(torch.float8_e4m3fn), w.float().to(torch.float8_e4m3fn)
    sa = torch.ones(M)
    sw = torch.arange(1, N + 1).float() / 16
    ref = (a.float() @ w.float().t()) * sw
    got = ops.linear_f8(a8.to(DEV), sa.to(DEV), w8.to(DEV), sw.to(DEV), out_dtype=torch.float32)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(1, 128, 128), (33, 896, 896), (129, 4864, 896), (624, 6144, 4096),
                                   (624, 4096, 14336), (700, 1024, 640)])
def test_gemm_f8_vs_fp32_reference(M, N, K):
    g, x8, xs, w8, ws = _f8_operands(M, N, K, M + N)
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :] + b + r.float()
    got = ops.linear_f8(x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV), bias=b.to(DEV), residual=r.to(DEV))
    assert _rel(got, ref) < 8e-3                     # bf16 output rounding only
    ref32 = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :]
    got32 = ops.linear_f8(x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV), out_dtype=torch.float32)
    assert _rel(got32, ref32) < 1e-4                 # fp32 accumulation order


@pytest.mark.parametrize("M", [7, 300])
def test_gemm_f8_swiglu(M):
    K, I = 1024, 2816
    g = torch.Generator().manual_seed(M)
    x8, xs = ops.quant_rows_fp8(torch.randn(M, K, generator=g).bfloat16())
    w8, ws = ops.quantize_fp8_rows(ops.glu_interleave(torch.randn(I, K, generator=g) * K ** -0.5,
                                                      torch.randn(I, K, generator=g) * K ** -0.5))
    ref = ops.linear_f8(x8, xs, w8, ws, glu=True)
    got = ops.linear_f8(x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV), glu=True)
    assert got.shape == (M, I) and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("M,K", [(1, 896), (37, 4096), (624, 14336), (3, 20480)])
def test_quant_rows_fp8_matches_torch(M, K):
    x = (torch.randn(M, K) * torch.logspace(-2, 2, M)[:, None]).bfloat16()
    ref8, refs = ops.quant_rows_fp8(x)
    got8, gots = ops.quant_rows_fp8(x.to(DEV))
    torch.testing.assert_close(gots.cpu(), refs, rtol=1e-6, atol=0)
    # e4m3 bytes: round-to-nearest-even on both sides; a few 1-ulp differences
    diff = (got8.cpu().view(torch.uint8).int() - ref8.view(torch.uint8).int()).abs()
    assert diff.max() <= 1 and (diff > 0).float().mean() < 1e-3


@pytest.mark.parametrize("M,K,add", [(5, 896, False), (624, 4096, True)])
def test_rms_norm_quant_fp8(M, K, add):
    g = torch.Generator().manual_seed(K)
    x = torch.randn(M, K, generator=g).bfloat16()
    a = torch.randn(M, K, generator=g).bfloat16() if add else None
    w = (1 + 0.1 * torch.randn(K, generator=g)).bfloat16()
    ref_res = torch.empty_like(x) if add else None
    ref8, refs = ops.rms_norm_quant_fp8(x, w, 1e-5, add=a, resid_out=ref_res)
    xd = x.to(DEV)
    got8, gots = ops.rms_norm_quant_fp8(xd, w.to(DEV), 1e-5, add=a.to(DEV) if add else None,
                                        resid_out=xd if add else None)
    torch.testing.assert_close(gots.cpu(), refs, rtol=1e-4, atol=0)
    deq = got8.cpu().float() * gots.cpu()[:, None]
    assert _rel(deq, ref8.float() * refs[:, None]) < 2e-2
    if add:
        torch.testing.assert_close(xd.cpu(), ref_res, rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K,glu", [(624, 1024, 4096, False), (300, 2048, 1024, True), (130, 640, 2048, False)])
def test_gemm_f8_splitk_vs_fp32_reference(M, N, K, glu):
    """Grids of <= 128 128x128 tiles split K over gridDim.y (fp32 slabs + ordered reduce with the
    real epilogue): bias + residual, SwiGLU, and repeat launches are bitwise identical."""
    g, x8, xs, w8, ws = _f8_operands(M, N, K, M + N + 1)
    if glu:
        ref = ops.linear_f8(x8, xs, w8, ws, glu=True)
        got = ops.linear_f8(x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV), glu=True)
        assert got.shape == (M, N // 2) and _rel(got, ref) < 1e-2
        return
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :] + b + r.float()
    args = (x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV))
    got = ops.linear_f8(*args, bias=b.to(DEV), residual=r.to(DEV))
    assert _rel(got, ref) < 8e-3
    again = ops.linear_f8(*args, bias=b.to(DEV), residual=r.to(DEV))
    assert torch.equal(got, again)


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16])
@pytest.mark.parametrize("M,N,K,splits", [(624, 6144, 4096, 1), (624, 4096, 4096, 2), (300, 1536, 1024, 1),
                                          (97, 768, 2048, 4), (130, 1040, 1024, 1)])
def test_gemm_f8_pipeline_variants(M, N, K, splits, variant):
    """Every fp8 pipeline shape (ring depth, waves, 128- / 256-wide tiles), with and without K
    splits, against the fp32 reference (bias + residual epilogue)."""
    g, x8, xs, w8, ws = _f8_operands(M, N, K, M + N + variant)
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :] + b + r.float()
    wd = w8.to(DEV)
    got = ops.linear_f8(x8.to(DEV), xs.to(DEV), wd, ws.to(DEV), bias=b.to(DEV), residual=r.to(DEV),
                        splits=splits, variant=variant)
    assert _rel(got, ref) < 8e-3


@pytest.mark.parametrize("M,N,K", [(624, 6144, 4096), (624, 4096, 14336), (130, 1040, 128), (200, 512, 256),
                                   (333, 768, 384), (624, 1024, 1152), (64, 256, 1024)])
@pytest.mark.parametrize("epi", ["bf16_bias_res", "f32_bias", "glu", "plain"])
@pytest.mark.parametrize("variant", [16, 17, 18])
def test_gemm_f8_intra_wg_splitk(M, N, K, epi, variant):
    """Intra-workgroup split-K fp8 GEMM (variant 16, csrc/gemm_f8ks.hip: both wave groups' K
    halves, odd and even K-step counts, one K-step), its Stream-K form (variant 18: one workgroup per
    CU over the (tile, K-step) sequence, tiles finished by their last segment from the others' fp32
    partials; 64 x 256 x 1024 puts 8 workgroups on one tile) and the 256 x 256 ping-pong fp8 GEMM (variant 17,
    csrc/gemm_f8pp.hip: peeled last K-tiles, automatic split-K with fp32 slabs for narrow grids):
    ragged M, the fast epilogue (bf16 bias, residual, SwiGLU) and the generic one (fp32 bias)
    against the fp32 reference; repeat launches are bitwise identical."""
    g, x8, xs, w8, ws = _f8_operands(M, N, K, M + N + K)
    dev_args = (x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV))
    acc = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :]
    if epi == "glu":
        ref = ops.linear_f8(x8, xs, w8, ws, glu=True)
        got = ops.linear_f8(*dev_args, glu=True, variant=variant)
        assert got.shape == (M, N // 2) and _rel(got, ref) < 1e-2
        return
    kw, ref = {}, acc
    if epi == "bf16_bias_res":
        b = torch.randn(N, generator=g).bfloat16()
        r = torch.randn(M, N, generator=g).bfloat16()
        kw = {"bias": b.to(DEV), "residual": r.to(DEV)}
        ref = acc + b.float() + r.float()
    elif epi == "f32_bias":
        b = torch.randn(N, generator=g)
        kw = {"bias": b.to(DEV)}
        ref = acc + b
    got = ops.linear_f8(*dev_args, variant=variant, **kw)
    assert _rel(got, ref) < 8e-3
    assert torch.equal(got, ops.linear_f8(*dev_args, variant=variant, **kw))


@pytest.mark.parametrize("M,N,glu,resid", [(624, 28672, True, False), (624, 22016 + 4096, False, True),
                                           (300, 36864, True, False)])
def test_gemm_f8_auto_prefill_split_columns(M, N, glu, resid):
    """Auto selection at prefill sizes (multi-round grids on the 256 x 256 ping-pong, code 17;
    single-round ones on the 128 x 128 split-K form, Stream-K when a quarter of the CUs would idle):
    same result as the fp32 reference with bias / residual / SwiGLU epilogues."""
    K = 1024
    g, x8, xs, w8, ws = _f8_operands(M, N, K, N + M)
    b = torch.randn(N, generator=g).bfloat16()
    args = (x8.to(DEV), xs.to(DEV), w8.to(DEV), ws.to(DEV))
    if glu:
        ref = ops.linear_f8(x8, xs, w8, ws, bias=b.float(), glu=True)
        got = ops.linear_f8(*args, bias=b.to(DEV), glu=True)
        assert got.shape == (M, N // 2) and _rel(got, ref) < 1e-2
        return
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = (x8.float() @ w8.float().t()) * xs[:, None] * ws[None, :] + b.float() + r.float()
    got = ops.linear_f8(*args, bias=b.to(DEV), residual=r.to(DEV))
    assert _rel(got, ref) < 8e-3


@pytest.mark.parametrize("tile", [20011, 20012, 20013, 20014, 20015, 20016, 20017, 20018, 20019, 20020, 20021,
                                  20022, 20023, 20024, 20025])
@pytest.mark.parametrize("M,N,K,act", [(577, 3072, 1024, None), (577, 1024, 4096, None), (200, 512, 640, "quick_gelu")])
def test_gemm_bf16_pipeline_variants(M, N, K, act, tile):
    """bf16 operands on every LDS-DMA pipeline shape (tile codes 20010 + launch_variant code)."""
    g = torch.Generator().manual_seed(M + N + tile)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x.float(), w.float(), b.float(), act=act, residual=r.float())
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), act=act, residual=r.to(DEV), tile=tile)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("M,N,K,act", [(577, 1024, 4096, None), (577, 3072, 1024, None), (577, 4096, 1024, "quick_gelu"),
                                       (300, 1024, 1024, None)])
def test_gemm_bf16_lds128_splitk_vs_fp32(M, N, K, act):
    """Mid-size bf16 GEMMs (the LLaVA vision tower at 577 tokens) on the 128x128 LDS-DMA
    pipeline with K split across workgroups, vs the fp32 CPU reference (bias / act / residual)."""
    g = torch.Generator().manual_seed(M * 3 + N)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x.float(), w.float(), b.float(), act=act, residual=r.float())
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), act=act, residual=r.to(DEV))
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("M", [1, 16])
def test_gemm_w8_two_tile_glu_norm(M):
    """Two-tile-per-workgroup decode kernel (wide N) through linear_dec: SwiGLU + folded RMSNorm."""
    K, I = 1024, 14336
    g = torch.Generator().manual_seed(M + 5)
    x = (torch.randn(M, K, generator=g) * 2).bfloat16()
    w8, ws = ops.quantize_fp8_rows(ops.glu_interleave(torch.randn(I, K, generator=g) * K ** -0.5,
                                                      torch.randn(I, K, generator=g) * K ** -0.5))
    ref = ops.linear(ops.rms_norm(x.float(), torch.ones(K), 1e-5), w8, glu=True, w_scale=ws)
    got = ops.linear_dec(x.to(DEV), w8.to(DEV), ws.to(DEV), glu=True, norm_eps=1e-5)
    assert got.shape == (M, I) and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(64, 512, 25088), (37, 512, 25088), (8, 256, 4096)])
def test_gemm_bf16_few_rows_deep_k_vs_fp32(M, N, K):
    """Few rows over a deep K (the IResNet embedding FC, fp32 output + bias) on the split-K
    LDS-DMA pipeline, vs the fp32 CPU reference."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g)
    ref = ops.linear(x.float(), w.float(), b)
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), out_dtype=torch.float32)
    assert got.dtype == torch.float32 and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("n", [40, 1000, 37])
def test_label_bank_any_label_count(n):
    """Label banks of any size on the GPU (the score GEMM tiles N in 16s: the bank is zero-padded
    and the padded scores cut before the top-k) == the fp32 reference top-k."""
    import numpy as np

    from lumen_amd.runtime.label_bank import LabelBank

    rng = np.random.default_rng(n)
    emb = rng.standard_normal((n, 768)).astype(np.float32)
    q = rng.standard_normal((3, 768)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    bank = LabelBank(emb, torch.device(DEV))
    p, idx = bank.topk(q, 5, scale=100.0, softmax=True)
    ref = q @ (emb / np.linalg.norm(emb, axis=1, keepdims=True)).T
    want = np.argsort(-ref, axis=1)[:, :5]
    assert np.asarray(idx).shape == (3, 5)
    assert (np.asarray(idx) < n).all()
    assert (np.asarray(idx)[:, 0] == want[:, 0]).all()
