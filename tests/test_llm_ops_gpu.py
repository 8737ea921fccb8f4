"""Decoder-LLM HIP kernels (SwiGLU epilogue, RoPE + paged KV write, paged decode attention,
repetition penalty) vs the fp32 PyTorch references."""
import math

import numpy as np
import pytest
import torch

from lumen_amd import ops
from lumen_amd.ops import llm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("M,K,I", [(1, 896, 4864), (37, 512, 1024), (300, 1024, 2816)])
def test_swiglu_epilogue(M, K, I):
    g = torch.Generator().manual_seed(M)
    x = torch.randn(M, K, generator=g).bfloat16()
    wg = (torch.randn(I, K, generator=g) * K ** -0.5).bfloat16()
    wu = (torch.randn(I, K, generator=g) * K ** -0.5).bfloat16()
    w = ops.glu_interleave(wg, wu)
    ref = ops.linear(x, w, glu=True)
    got = ops.linear(x.to(DEV), w.to(DEV), glu=True)
    assert got.shape == (M, I)
    assert _rel(got, ref) < 1e-2


def _cache(NB, Hkv, D, g):
    k = (torch.randn(NB, Hkv, 64, D, generator=g)).bfloat16()
    v = (torch.randn(NB, Hkv, D, 64, generator=g)).bfloat16()
    return k, v


@pytest.mark.parametrize("H,Hkv,D", [(14, 2, 64), (32, 8, 128), (4, 4, 64)])
def test_rope_kv(H, Hkv, D):
    g = torch.Generator().manual_seed(H)
    T = 75
    qkv = torch.randn(T, (H + 2 * Hkv) * D + 16, generator=g).bfloat16()[:, :(H + 2 * Hkv) * D]
    pos = torch.randint(0, 4000, (T,), generator=g, dtype=torch.int32)
    cs = llm.rope_cos_sin(4096, D, 1e6)
    kc, vc = _cache(6, Hkv, D, g)
    slots = torch.randperm(6 * 64, generator=g)[:T].long()
    slots[5] = -1
    q_ref, kc_ref, vc_ref = qkv.clone(), kc.clone(), vc.clone()
    llm.rope_kv(q_ref, pos, cs, H, Hkv, D, slots, kc_ref, vc_ref)
    q_g, kc_g, vc_g = qkv.to(DEV), kc.to(DEV), vc.to(DEV)
    llm.rope_kv(q_g, pos.to(DEV), cs.to(DEV), H, Hkv, D, slots.to(DEV), kc_g, vc_g)
    assert (q_g.cpu().float() - q_ref.float()).abs().max().item() < 0.05
    assert (kc_g.cpu().float() - kc_ref.float()).abs().max().item() < 0.05
    assert torch.equal(vc_g.cpu(), vc_ref)


@pytest.mark.parametrize("H,Hkv,D", [(32, 8, 128), (14, 2, 64)])
@pytest.mark.parametrize("start", [0, 37])
@pytest.mark.parametrize("fp8", [False, True])
def test_rope_kv_prefill_tiles(H, Hkv, D, start, fp8):
    """Prefill-sized rope_kv (64-token tiles, d-major V runs through LDS): a sequence whose slots
    run through its blocks from an unaligned start, vs the CPU reference."""
    g = torch.Generator().manual_seed(H + start)
    T = 200
    qkv = torch.randn(T, (H + 2 * Hkv) * D, generator=g).bfloat16()
    pos = torch.arange(start, start + T, dtype=torch.int32)
    cs = llm.rope_cos_sin(4096, D, 5e5)
    kc, vc = _cache(8, Hkv, D, g)
    table = torch.tensor([5, 2, 7, 0, 3, 6, 1, 4])
    p = torch.arange(start, start + T)
    slots = (table[p // 64] * 64 + p % 64).long()
    if fp8:
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    q_ref, kc_ref, vc_ref = qkv.clone(), kc.clone(), vc.clone()
    llm.rope_kv(q_ref, pos, cs, H, Hkv, D, slots, kc_ref, vc_ref)
    q_g, kc_g, vc_g = qkv.to(DEV), kc.to(DEV), vc.to(DEV)
    llm.rope_kv(q_g, pos.to(DEV), cs.to(DEV), H, Hkv, D, slots.to(DEV), kc_g, vc_g)
    assert (q_g.cpu().float() - q_ref.float()).abs().max().item() < 0.05
    dk = (kc_g.cpu().float() - kc_ref.float()).abs()
    if fp8:     # one e4m3 step where the rotated bf16 value itself differs by an ulp
        assert (dk <= 0.13 * kc_ref.float().abs() + 1e-3).all() and (dk > 0).float().mean().item() < 0.02
    else:
        assert dk.max().item() < 0.05
    assert (vc_g.cpu().float() - vc_ref.float()).abs().max().item() == 0.0


@pytest.mark.parametrize("H,Hkv,D", [(14, 2, 64), (32, 8, 128), (32, 32, 128), (16, 1, 64), (4, 2, 32)])
@pytest.mark.parametrize("lens", [[1, 64, 65], [700, 3, 2048 + 17], [5000], [70, 700, 3, 1, 2048 + 17, 64]])
def test_paged_decode(H, Hkv, D, lens):
    g = torch.Generator().manual_seed(H * D + len(lens))
    B = len(lens)
    maxb = max(-(-L // 64) for L in lens)
    NB = B * maxb + 3
    kc, vc = _cache(NB, Hkv, D, g)
    perm = torch.randperm(NB, generator=g)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for b in range(B):
        bt[b] = perm[b * maxb:(b + 1) * maxb].int()
    ctx = torch.tensor(lens, dtype=torch.int32)
    q = torch.randn(B, (H + 2 * Hkv) * D, generator=g).bfloat16()
    ref = llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv)
    args = (q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), ctx.to(DEV), H, Hkv)
    got = llm.paged_decode(*args)
    assert got.shape == (B, H * D)
    assert _rel(got, ref) < 2e-2
    # split partials are merged in-launch by the last arriving split (self-resetting counters):
    # repeat launches and a graph replay give the same bits
    for _ in range(3):
        assert torch.equal(llm.paged_decode(*args), got)
    # weight prefetch workgroups in the same launch (read-only side stream of two tensors) change nothing
    pf = (torch.randn(3 << 20, device=DEV).bfloat16(), torch.empty(12345, device=DEV, dtype=torch.uint8))
    assert torch.equal(llm.paged_decode(*args, prefetch=pf), got)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        llm.paged_decode(*args)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        cap = llm.paged_decode(*args)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(cap, got)


def test_rep_penalty():
    g = torch.Generator().manual_seed(0)
    lg = torch.randn(3, 1000, generator=g)
    ids = [[1, 5, 5, 999], [], [0, 2, 3]]
    ref = llm.rep_penalty_(lg.clone(), ids, [1.3, 1.1, 0.7])
    got = llm.rep_penalty_(lg.to(DEV), ids, [1.3, 1.1, 0.7]).cpu()
    assert torch.allclose(got, ref)


@pytest.mark.parametrize("M", [1, 3, 16, 17, 32])
@pytest.mark.parametrize("N,K", [(896, 4864), (9728, 896), (4096, 14336), (256, 128)])
def test_skinny_gemm(M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x, w, b, residual=r)
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), residual=r.to(DEV))
    assert _rel(got, ref) < 1e-2
    ref32 = ops.linear(x, w, act="silu", out_dtype=torch.float32)
    got32 = ops.linear(x.to(DEV), w.to(DEV), act="silu", out_dtype=torch.float32)
    assert got32.dtype == torch.float32 and _rel(got32, ref32) < 1e-2
    if N % 16 == 0:
        ref_g = ops.linear(x, w, glu=True)
        got_g = ops.linear(x.to(DEV), w.to(DEV), glu=True)
        assert got_g.shape == (M, N // 2) and _rel(got_g, ref_g) < 1e-2


@pytest.mark.parametrize("B,N,k", [(1, 151936, 8), (5, 128256, 64), (3, 20000, 16), (2, 1000, 8)])
def test_row_topk_long_rows(B, N, k):
    g = torch.Generator().manual_seed(N)
    s = torch.randn(B, N, generator=g) * 4
    v, i, lse = ops.row_topk(s, k, scale=0.7, with_lse=True, index_offset=11)
    vg, ig, lg = ops.row_topk(s.to(DEV), k, scale=0.7, with_lse=True, index_offset=11)
    assert torch.equal(ig.cpu(), i) and torch.allclose(vg.cpu(), v)
    assert torch.allclose(lg.cpu(), lse, atol=1e-3)


@pytest.mark.parametrize("fp8", [False, True])
def test_skinny_splitk_inkernel_reduction(fp8):
    """Split-K decode GEMMs reduce in the last-arriving workgroup (per-tile counters that
    reset themselves): repeated launches, differently split shapes back to back, two
    streams and a hipGraph replay must all match the eager result bit for bit."""
    g = torch.Generator().manual_seed(11)
    # all four split K under the per-shape policy (ntiles < 256): 896/1024/2048 wide
    shapes = [(1, 2048, 14336), (5, 1152, 4096), (16, 896, 4864), (32, 1024, 4096)]
    cases = []
    for M, N, K in shapes:
        x = torch.randn(M, K, generator=g).bfloat16().to(DEV)
        wf = torch.randn(N, K, generator=g) * K ** -0.5
        if fp8:
            w8, s = ops.quantize_fp8_rows(wf)
            cases.append((x, w8.to(DEV), s.to(DEV)))
        else:
            cases.append((x, wf.bfloat16().to(DEV), None))

    def run():
        return [ops.linear(x, w, w_scale=s) for x, w, s in cases]

    first = run()
    for (x, w, s), got in zip(cases, first):
        ref = ops.linear(x.float().cpu(), w.cpu(), w_scale=None if s is None else s.cpu())
        assert _rel(got, ref) < 1e-2
    for _ in range(5):
        for a, b in zip(run(), first):
            assert torch.equal(a, b)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        o1 = [run() for _ in range(3)]
    with torch.cuda.stream(s2):
        o2 = [run() for _ in range(3)]
    torch.cuda.synchronize()
    for outs in o1 + o2:
        for a, b in zip(outs, first):
            assert torch.equal(a, b)
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(graph):
        captured = run()
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        for a, b in zip(captured, first):
            assert torch.equal(a, b)


def test_llm_fp8_w8a8_prefill_vs_weight_only():
    """fp8 model: W8A8 prefill (fp8 x fp8 MFMA, per-token scales) vs the weight-only fp8 path
    (bf16 activations) of the same weights; no bf16 weight image is kept."""
    from lumen_amd.models import llm as llm_mod
    cfg = llm_mod.LLM_PRESETS["qwen2-0.5b"]
    m = llm_mod.LLM(cfg, device=torch.device(DEV))
    m.random_init(0)
    m.quantize_fp8()
    assert not any(n.endswith("_wb") for n, _ in m.named_buffers())
    x0 = (torch.randn(300, cfg.hidden_size, generator=torch.Generator().manual_seed(3)) * 0.5).bfloat16().to(DEV)
    assert m._f8_ok(300)
    a = m.prefill(x0.clone())
    old = llm_mod._F8_MIN_ROWS
    try:
        llm_mod._F8_MIN_ROWS = 1 << 30
        b = m.prefill(x0.clone())
    finally:
        llm_mod._F8_MIN_ROWS = old
    cos = torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()
    assert torch.isfinite(a).all() and cos > 0.99, cos


def test_llm_prefill_large_bias_fp32():
    """HF-scale q/k biases (Qwen2 has |b| of several units): the prefill adds them in fp32 in the
    GEMM epilogue (no bf16 rounding of the bias), matching the fp32 CPU model."""
    from lumen_amd.models import llm as llm_mod
    cfg = llm_mod.LLM_PRESETS["tiny"]
    cpu = llm_mod.LLM(cfg, dtype=torch.float32, device="cpu")
    cpu.random_init(5)
    with torch.no_grad():
        for l in cpu.layers:
            l.qkv_b.copy_(torch.randn(l.qkv_b.shape, generator=torch.Generator().manual_seed(7)) * 8.0)
    gpu = llm_mod.LLM(cfg, device=torch.device(DEV))
    gpu.load_state_dict({k: v.to(gpu.state_dict()[k].dtype) for k, v in cpu.state_dict().items()}, strict=False)
    ids = torch.randint(0, cfg.vocab_size, (200,), generator=torch.Generator().manual_seed(1))
    ref = cpu.prefill(cpu.embed_tokens(ids))
    got = gpu.prefill(gpu.embed_tokens(ids.to(DEV)))
    cos = torch.nn.functional.cosine_similarity(got.float().cpu().flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.995, cos


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("M,N,K,glu", [(1, 6144, 4096, False), (5, 896 + 256, 896, False), (16, 2048, 4096, True),
                                       (32, 1024, 4096, False), (3, 128256 // 8, 4096, False)])
def test_linear_dec_norm_folding_matches_cpu(fp8, M, N, K, glu):
    """Decode GEMM with the RMSNorm folded (gamma in W, rstd as an epilogue row scale) vs
    rms_norm -> linear in fp32 on the CPU: rstd computed from x, and rstd from the sums of
    squares a producing residual GEMM wrote (ssq_out -> ssq_in); split-K shapes included."""
    g = torch.Generator().manual_seed(M * 7 + N)
    x0 = (torch.randn(M, K, generator=g) * 3).bfloat16()
    gamma = (1 + 0.3 * torch.randn(K, generator=g)).bfloat16()
    wf = torch.randn(N, K, generator=g) * K ** -0.5
    b = None if glu else torch.randn(N, generator=g) * 0.1
    wfold = wf * gamma.float()[None, :]
    if fp8:
        w, s = ops.quantize_fp8_rows(wf)
        wd, sd = ops.quantize_fp8_rows(wfold)
    else:
        w, s = wf.bfloat16(), None
        wd, sd = wfold.bfloat16(), None
    # producer: x = x0 + a @ Wp^T (residual GEMM) writing the per-tile sums of squares
    a = torch.randn(M, 512, generator=g).bfloat16()
    wp = (torch.randn(K, 512, generator=g) * 512 ** -0.5).bfloat16()
    x_ref = ops.linear(a.float(), wp.float(), residual=x0.float()).bfloat16()
    ssq = torch.zeros(32, K // 16, device=DEV)
    x = x0.to(DEV).clone()
    ops.linear_dec(a.to(DEV), wp.to(DEV), residual=x, out=x, ssq_out=ssq)
    assert _rel(x, x_ref) < 1e-2
    xr = x.cpu()
    ref_ssq = (xr.float() ** 2).view(M, K // 16, 16).sum(-1)
    torch.testing.assert_close(ssq[:M].cpu(), ref_ssq, rtol=1e-4, atol=1e-3)
    one = torch.ones(K)
    # same (folded, quantised) weights: the kernel's norm folding itself
    ref = ops.linear(ops.rms_norm(xr.float(), one, 1e-5), wd, bias=b, glu=glu, w_scale=sd)
    # unfolded fp32 model (bf16: folding costs one extra weight rounding; fp8: requantisation noise)
    ref_unfold = ops.linear(ops.rms_norm(xr.float(), gamma.float(), 1e-5), w, bias=b, glu=glu, w_scale=s)
    sdev = None if sd is None else sd.to(DEV)
    for sq in (None, ssq):
        got = ops.linear_dec(x, wd.to(DEV), sdev, bias=None if b is None else b.to(DEV), glu=glu, norm_eps=1e-5,
                             ssq_in=sq)
        assert got.shape == ref.shape
        assert _rel(got, ref) < 1e-2
        assert _rel(got, ref_unfold) < (6e-2 if fp8 else 1.5e-2)
    if not glu:
        got32 = ops.linear_dec(x, wd.to(DEV), sdev, norm_eps=1e-5, ssq_in=ssq, out_dtype=torch.float32)
        ref32 = ops.linear(ops.rms_norm(xr.float(), one, 1e-5), wd, w_scale=sd)
        assert got32.dtype == torch.float32 and _rel(got32, ref32) < 1e-2


@pytest.mark.parametrize("H,Hkv,D", [(32, 8, 128), (14, 2, 64)])
@pytest.mark.parametrize("lens", [[1, 64, 65], [700, 3, 2048 + 17]])
def test_paged_decode_fused_rope_matches_rope_kv(H, Hkv, D, lens):
    """Decode attention with RoPE + current-token cache write fused in (q unrotated) == rope_kv
    then paged_decode: the same K / V cache contents, and the same attention output up to the
    summation order of the current token's score (the fused kernel takes q . k_cur from
    registers as a lane-group dot product instead of reading the token back through MFMA)."""
    g = torch.Generator().manual_seed(H + D + len(lens))
    B = len(lens)
    maxb = max(-(-L // 64) for L in lens)
    NB = B * maxb + 3
    kc, vc = _cache(NB, Hkv, D, g)
    perm = torch.randperm(NB, generator=g)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for b in range(B):
        bt[b] = perm[b * maxb:(b + 1) * maxb].int()
    ctx = torch.tensor(lens, dtype=torch.int32)
    pos = ctx - 1
    slots = torch.tensor([int(bt[b, (L - 1) // 64]) * 64 + (L - 1) % 64 for b, L in enumerate(lens)], dtype=torch.long)
    cs = llm.rope_cos_sin(4096, D, 500000.0)
    qkv = torch.randn(B, (H + 2 * Hkv) * D, generator=g).bfloat16()
    q1, k1, v1 = qkv.to(DEV), kc.to(DEV), vc.to(DEV)
    llm.rope_kv(q1, pos.to(DEV), cs.to(DEV), H, Hkv, D, slots.to(DEV), k1, v1)
    ref = llm.paged_decode(q1, k1, v1, bt.to(DEV), ctx.to(DEV), H, Hkv)
    q2, k2, v2 = qkv.to(DEV), kc.to(DEV), vc.to(DEV)
    got = llm.paged_decode(q2, k2, v2, bt.to(DEV), ctx.to(DEV), H, Hkv,
                           rope=(pos.to(DEV), cs.to(DEV), slots.to(DEV)))
    torch.cuda.synchronize()
    assert torch.equal(k2, k1) and torch.equal(v2, v1)
    assert _rel(got, ref) < 2e-3
    assert (got.float() - ref.float()).abs().max().item() < 2e-2
    assert torch.equal(q2, qkv.to(DEV))            # the QKV rows are not rotated in place


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("H,Hkv,D", [(32, 8, 128), (14, 2, 64)])
def test_fp8_kv_cache_matches_cpu(H, Hkv, D, fused):
    """OCP e4m3 paged KV cache: the GPU writers (rope_kv / the fused decode path) store the same
    bytes as the CPU reference cast (saturated), and decode attention over the fp8 cache matches
    the CPU reference over the same cache."""
    g = torch.Generator().manual_seed(D + H)
    lens = [1, 200, 1000]
    B = len(lens)
    maxb = max(-(-L // 64) for L in lens)
    NB = B * maxb + 2
    kc = (torch.randn(NB, Hkv, 64, D, generator=g) * 2).to(torch.float8_e4m3fn)
    vc = (torch.randn(NB, Hkv, D, 64, generator=g) * 2).to(torch.float8_e4m3fn)
    perm = torch.randperm(NB, generator=g)
    bt = torch.stack([perm[b * maxb:(b + 1) * maxb] for b in range(B)]).int()
    ctx = torch.tensor(lens, dtype=torch.int32)
    pos = ctx - 1
    slots = torch.tensor([int(bt[b, (L - 1) // 64]) * 64 + (L - 1) % 64 for b, L in enumerate(lens)], dtype=torch.long)
    cs = llm.rope_cos_sin(4096, D, 1e6)
    qkv = (torch.randn(B, (H + 2 * Hkv) * D, generator=g) * 3).bfloat16()
    q_ref, k_ref, v_ref = qkv.clone(), kc.clone(), vc.clone()
    llm.rope_kv(q_ref, pos, cs, H, Hkv, D, slots, k_ref, v_ref)
    ref = llm.paged_decode(q_ref, k_ref, v_ref, bt, ctx, H, Hkv)
    kg, vg = kc.to(DEV), vc.to(DEV)
    if fused:
        got = llm.paged_decode(qkv.to(DEV), kg, vg, bt.to(DEV), ctx.to(DEV), H, Hkv,
                               rope=(pos.to(DEV), cs.to(DEV), slots.to(DEV)))
    else:
        qg = qkv.to(DEV)
        llm.rope_kv(qg, pos.to(DEV), cs.to(DEV), H, Hkv, D, slots.to(DEV), kg, vg)
        got = llm.paged_decode(qg, kg, vg, bt.to(DEV), ctx.to(DEV), H, Hkv)
    assert torch.equal(kg.cpu().view(torch.uint8), k_ref.view(torch.uint8))
    assert torch.equal(vg.cpu().view(torch.uint8), v_ref.view(torch.uint8))
    assert _rel(got, ref) < 2e-2


def test_upload_small_and_h2d_ahead():
    """Small integer uploads through kernel arguments (ops_llm.cpp:upload_small) land exactly, in
    stream order behind queued work; larger / non-integer inputs fall back to the pinned copy."""
    import numpy as np

    from lumen_amd.utils.h2d import h2d_ahead

    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    for _ in range(4):
        a = a @ a * 0.01                          # queued work ahead of the uploads
    ids = list(np.random.default_rng(0).integers(0, 128256, 624))
    t = h2d_ahead(ids, "cuda", torch.long)
    slots = np.arange(7, 7 + 896, dtype=np.int64)
    s = h2d_ahead(slots, "cuda")
    big = h2d_ahead(np.arange(2000, dtype=np.int64), "cuda")
    neg = h2d_ahead(np.array([-5, 3, 2 ** 40], dtype=np.int64), "cuda")
    torch.cuda.synchronize()
    assert t.dtype == torch.long and t.tolist() == [int(v) for v in ids]
    assert s.tolist() == slots.tolist() and big.tolist() == list(range(2000))
    assert neg.tolist() == [-5, 3, 2 ** 40]
