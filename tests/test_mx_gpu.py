"""MX (block-scaled) W8A8 prefill chain on the gfx950 scaled matrix cores vs the CPU references:
quant_rows_mx (bit-exact E8M0 + e4m3 bytes), gemm_mx with every epilogue the fused prefill
uses (rstd row scale from producer sums of squares, SwiGLU -> MX fp8, residual -> bf16 + MX
fp8 + sums of squares) and the attention kernel's MX fp8 output."""
import pytest
import torch

from lumen_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def _rows(M, K, g, spread=True):
    x = torch.randn(M, K, generator=g)
    if spread:   # per-block magnitudes over ~2^-8 .. 2^8 so the E8M0 bytes differ along a row
        x = x * torch.exp2(torch.randint(-8, 9, (M, K // 32), generator=g).float()).repeat_interleave(32, 1)
    return x.bfloat16()


@pytest.mark.parametrize("M,K", [(1, 128), (37, 896), (624, 4096)])
def test_quant_rows_mx_bit_exact(M, K):
    g = torch.Generator().manual_seed(M + K)
    x = _rows(M, K, g)
    x[0, :32] = 0     # an all-zero block: smallest scale
    q_ref, s_ref = ops.mx_quant_ref(x)
    ssq = torch.empty(M, K // 128, device=DEV)
    q8, qs = ops.quant_rows_mx(x.to(DEV), ssq=ssq)
    assert torch.equal(qs.cpu(), s_ref)
    assert torch.equal(q8.cpu().view(torch.uint8), q_ref.view(torch.uint8))
    ref_ssq = (x.float() ** 2).reshape(M, K // 128, 128).sum(-1)
    assert torch.allclose(ssq.cpu(), ref_ssq, rtol=1e-4, atol=1e-6)


def _operands(M, N, K, g):
    x = _rows(M, K, g)
    x8, xs = ops.mx_quant_ref(x)
    w8, sw = ops.quantize_fp8_rows(torch.randn(N, K, generator=g) * K ** -0.5)
    return x8, xs, w8, sw


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 9, 10, 11, 12, 13, 15])
@pytest.mark.parametrize("M,N,K", [(130, 1024, 512), (624, 2048, 4096), (33, 256, 128)])
def test_gemm_mx_plain_vs_reference(M, N, K, variant):
    """A scale bytes reach the MFMA per lane (k 32g .. 32g+31) -- wrong lanes or a wrong k order
    would scale whole blocks by up to 2^16 and blow the error up."""
    g = torch.Generator().manual_seed(M * N + K)
    x8, xs, w8, sw = _operands(M, N, K, g)
    b = torch.randn(N, generator=g)
    ref = ops.linear_mx(x8, xs, w8, sw, bias=b)
    got = ops.linear_mx(x8.to(DEV), xs.to(DEV), w8.to(DEV), sw.to(DEV), bias=b.to(DEV), variant=variant)
    assert _rel(got, ref) < 1e-2


def test_gemm_mx_exact_small_integers():
    """Integer operands and power-of-two block scales are exact in fp32: bitwise-equal result."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 64, 128, 256
    x8 = torch.randint(-4, 5, (M, K), generator=g).float().to(torch.float8_e4m3fn)
    xs = ops.mx_planes(torch.randint(124, 131, (M, K // 32), generator=g).to(torch.uint8))
    w8 = torch.randint(-4, 5, (N, K), generator=g).float().to(torch.float8_e4m3fn)
    sw = torch.ones(N)
    ref = ops.mx_dequant(x8, xs) @ w8.float().t()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear_mx(x8.to(DEV), xs.to(DEV), w8.to(DEV), sw.to(DEV), out=out)
    assert torch.equal(out.cpu().float(), ref.bfloat16().float())


@pytest.mark.parametrize("variant", [0, 1, 2, 4, 10])
@pytest.mark.parametrize("M,N,K", [(200, 1024, 512), (624, 4096, 4096)])
def test_gemm_mx_residual_outputs(M, N, K, variant):
    """o / down projection: bf16 residual stream + its MX fp8 copy + per-128-column sums of squares."""
    g = torch.Generator().manual_seed(M + 7 * N)
    x8, xs, w8, sw = _operands(M, N, K, g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref_q, ref_s = torch.empty(M, N, dtype=torch.float8_e4m3fn), torch.empty(N // 128, M, 4, dtype=torch.uint8)
    ref_ss = torch.empty(M, N // 128)
    ref = ops.linear_mx(x8, xs, w8, sw, residual=r, out=r.clone(), q_out=(ref_q, ref_s), ssq_out=ref_ss)
    xg = r.to(DEV)
    q8 = torch.empty(M, N, device=DEV, dtype=torch.float8_e4m3fn)
    qs = torch.empty(N // 128, M, 4, device=DEV, dtype=torch.uint8)
    ss = torch.empty(M, N // 128, device=DEV)
    ops.linear_mx(x8.to(DEV), xs.to(DEV), w8.to(DEV), sw.to(DEV), residual=xg, out=xg, q_out=(q8, qs),
                  ssq_out=ss, variant=variant)
    assert _rel(xg, ref) < 1e-2
    # the MX copy is the exact quantisation of the stored bf16 rows
    q_self, s_self = ops.mx_quant_ref(xg.cpu().float())
    assert torch.equal(qs.cpu(), s_self)
    assert torch.equal(q8.cpu().view(torch.uint8), q_self.view(torch.uint8))
    assert torch.allclose(ss.cpu(), (xg.cpu().float() ** 2).reshape(M, N // 128, 128).sum(-1), rtol=1e-4)
    assert _rel(ss, ref_ss) < 2e-2


@pytest.mark.parametrize("variant", [0, 1, 2, 4, 10])
@pytest.mark.parametrize("write_out", [True, False])
def test_gemm_mx_swiglu_mx_output(variant, write_out):
    """gate|up projection: SwiGLU straight to MX fp8 (the down projection's A operand)."""
    g = torch.Generator().manual_seed(11 + variant)
    M, N, K = 300, 2048, 1024
    x8, xs, w8, sw = _operands(M, N, K, g)
    ref_q, ref_s = torch.empty(M, N // 2, dtype=torch.float8_e4m3fn), torch.empty(N // 256, M, 4, dtype=torch.uint8)
    ref = ops.linear_mx(x8, xs, w8, sw, glu=True, q_out=(ref_q, ref_s))
    q8 = torch.empty(M, N // 2, device=DEV, dtype=torch.float8_e4m3fn)
    qs = torch.empty(N // 256, M, 4, device=DEV, dtype=torch.uint8)
    got = ops.linear_mx(x8.to(DEV), xs.to(DEV), w8.to(DEV), sw.to(DEV), glu=True, q_out=(q8, qs),
                        write_out=write_out, variant=variant)
    if write_out:
        assert _rel(got, ref) < 1e-2
    deq, deq_ref = ops.mx_dequant(q8.cpu(), qs.cpu()), ops.mx_dequant(ref_q, ref_s)
    assert _rel(deq, deq_ref) < 3e-2
    assert (qs.cpu().int() - ref_s.int()).abs().max().item() <= 1


@pytest.mark.parametrize("M,N,K", [(150, 1024, 1024), (624, 6144, 4096)])
def test_gemm_mx_rstd_from_producer_ssq(M, N, K):
    """qkv / gate|up: RMSNorm as the rstd row scale from the producer's sums of squares."""
    g = torch.Generator().manual_seed(M + N + K)
    x = _rows(M, K, g, spread=False) * 3
    ssq = torch.empty(M, K // 128, device=DEV)
    x8, xs = ops.quant_rows_mx(x.to(DEV), ssq=ssq)
    w8, sw = ops.quantize_fp8_rows(torch.randn(N, K, generator=g) * K ** -0.5)
    got = ops.linear_mx(x8, xs, w8.to(DEV), sw.to(DEV), ssq_in=ssq, norm_eps=1e-5)
    xn = x.float() * torch.rsqrt((x.float() ** 2).mean(1, keepdim=True) + 1e-5)
    ref = xn @ (w8.float() * sw[:, None]).t()
    assert _rel(got, ref) < 3e-2


def test_gemm_mx_graph_capture_and_repeat():
    g = torch.Generator().manual_seed(5)
    M, N, K = 624, 4096, 4096
    x8, xs, w8, sw = [t.to(DEV) for t in _operands(M, N, K, g)]
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.linear_mx(x8, xs, w8, sw, out=out, variant=10)
    first = out.clone()
    for v in (10, 10):
        ops.linear_mx(x8, xs, w8, sw, out=out, variant=v)
        assert torch.equal(out, first)
    # captured on torch's capture stream, which has no stream-K workspace yet: the launch falls back
    # to the tiled pipeline (other K summation order) -- replays are bit-identical to each other
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ops.linear_mx(x8, xs, w8, sw, out=out, variant=10)
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    rep = out.clone()
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, rep) and _rel(rep, first) < 1e-2


@pytest.mark.parametrize("S,H,Hkv,D,causal", [(624, 32, 8, 128, True), (577, 16, 16, 64, False), (70, 4, 2, 128, True)])
def test_attention_mx_output(S, H, Hkv, D, causal):
    """The attention kernel's MX fp8 output: the exact MX quantisation of its own fp32 O (checked
    against the bf16 O of the same launch) and close to the fp32 reference."""
    g = torch.Generator().manual_seed(S + H)
    q = torch.randn(1, S, H, D, generator=g).bfloat16()
    k = torch.randn(1, S, Hkv, D, generator=g).bfloat16()
    v = torch.randn(1, S, Hkv, D, generator=g).bfloat16()
    qg, kg, vg = q.to(DEV), k.to(DEV), v.to(DEV)
    ob = torch.empty(1, S, H, D, device=DEV, dtype=torch.bfloat16)
    o8, os_ = ops.attention_mx(qg, kg, vg, causal=causal, out=ob)
    plain = ops.attention(qg, kg, vg, causal=causal)
    assert torch.equal(ob, plain)
    deq = ops.mx_dequant(o8.cpu(), os_.cpu())
    ref = ops.attention(q.float(), k.float(), v.float(), causal=causal).reshape(S, H * D)
    assert _rel(deq, ref) < 4e-2
    # scale bytes: those of the (bf16-rounded) kernel output, up to one step at block boundaries
    _, s_b = ops.mx_quant_ref(ob.cpu().float().reshape(S, H * D))
    assert (os_.cpu().int() - s_b.int()).abs().max().item() <= 1
    o8b, osb = ops.attention_mx(qg, kg, vg, causal=causal)     # fp8 only: same bytes
    assert torch.equal(o8b.view(torch.uint8), o8.view(torch.uint8)) and torch.equal(osb, os_)


def test_ln_row_stats_mx_copy():
    """LayerNorm row statistics + the raw rows' MX copy in one pass (the W8A8 vision tower's qkv / fc1
    operand): stats as the plain kernel, bytes as mx_quant_ref."""
    g = torch.Generator().manual_seed(7)
    x = _rows(577, 1024, g)
    st0 = ops.ln_row_stats(x.to(DEV), 1e-5)
    q8 = torch.empty(577, 1024, device=DEV, dtype=torch.float8_e4m3fn)
    qs = torch.empty(8, 577, 4, device=DEV, dtype=torch.uint8)
    st = ops.ln_row_stats(x.to(DEV), 1e-5, q_out=(q8, qs))
    assert torch.equal(st, st0)
    q_ref, s_ref = ops.mx_quant_ref(x)
    assert torch.equal(qs.cpu(), s_ref) and torch.equal(q8.cpu().view(torch.uint8), q_ref.view(torch.uint8))


@pytest.mark.parametrize("mx_only", [False, True])
def test_gemm_mx_ln_fold_and_act(mx_only):
    """qkv / fc1 of the vision chain: LN folded (row_aff, col_aff), quick_gelu, bf16 out or MX out only."""
    g = torch.Generator().manual_seed(9)
    M, N, K = 577, 1024, 1024
    x = (torch.randn(M, K, generator=g) * 2 + 0.5).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5)
    gamma, beta, b = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1, torch.randn(N, generator=g)
    wf, caff = ops.ln_fold_weights(w.bfloat16(), b, gamma, beta)
    w8, sw = ops.quantize_fp8_rows(wf)
    caff[0] = (w8.float() * sw[:, None]).sum(1)
    xd = x.to(DEV)
    x8 = torch.empty(M, K, device=DEV, dtype=torch.float8_e4m3fn)
    xs = torch.empty(K // 128, M, 4, device=DEV, dtype=torch.uint8)
    st = ops.ln_row_stats(xd, 1e-5, q_out=(x8, xs))
    q8 = torch.empty(M, N, device=DEV, dtype=torch.float8_e4m3fn)
    qs = torch.empty(N // 128, M, 4, device=DEV, dtype=torch.uint8)
    got = ops.linear_mx(x8, xs, w8.to(DEV), sw.to(DEV), row_aff=st, col_aff=caff.to(DEV), act="quick_gelu",
                        q_out=(q8, qs) if mx_only else None, write_out=not mx_only)
    ln = torch.nn.functional.layer_norm(x.float(), (K,), gamma, beta, 1e-5)
    ref = ln @ w.t() + b
    ref = ref * torch.sigmoid(1.702 * ref)
    res = ops.mx_dequant(q8.cpu(), qs.cpu()) if mx_only else got
    assert _rel(res, ref) < 4e-2


def test_vision_tower_w8a8_matches_bf16():
    """The W8A8 MX vision chain (run_blocks_mx) vs the bf16 tower on the same weights."""
    from lumen_amd.models.clip import VisionConfig, VisionTower

    cfg = VisionConfig(image_size=64, patch_size=16, width=256, layers=3, heads=4)
    vt = VisionTower(cfg, 16, torch.float32, "cpu")
    vt.random_init(torch.Generator().manual_seed(0))
    v = VisionTower(cfg, 16, torch.bfloat16, DEV)
    v.load_state_dict({k: t.to(v.state_dict()[k].dtype) for k, t in vt.state_dict().items()})
    imgs = [torch.randint(0, 256, (64, 64, 3), dtype=torch.uint8, device=DEV) for _ in range(3)]
    patches = v.preprocess(imgs, (0.48, 0.46, 0.41), (0.27, 0.26, 0.28))
    ref = v.forward_features(patches, 3, -2).float()
    v.w8a8 = True
    got = v.forward_features(patches, 3, -2).float()
    cos = torch.nn.functional.cosine_similarity(got.reshape(-1, 256), ref.reshape(-1, 256)).min().item()
    assert cos > 0.98, cos
