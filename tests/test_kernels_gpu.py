"""Numerics of the hand-written gfx950 kernels vs the PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

from lumen_amd import ops
from lumen_amd._native import native_status

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def test_native_library_loaded():
    ops.linear(torch.zeros(16, 64, device=DEV, dtype=torch.bfloat16), torch.zeros(16, 64, device=DEV, dtype=torch.bfloat16))
    st = native_status()
    assert st["hip_loaded"], st


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 768, 1024), (131, 3072, 1024), (512, 4096, 1024),
                                   (37, 64, 128), (4096, 1024, 4096), (2, 512, 512), (2570, 1024, 640)])
@pytest.mark.parametrize("act", [None, "gelu", "quick_gelu"])
@pytest.mark.parametrize("tile", [-1, 4, 5, 6, 7, 8, 9, 209, 609, 709, 809, 909, 109, 20000, 20002, 20003])
def test_gemm_vs_fp32(M, N, K, act, tile):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x, w, b, act=act, residual=r)
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), act=act, residual=r.to(DEV), tile=tile)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 609, 709, 809, 909, 20002, 20003])
def test_gemm_tiles_asymmetric(tile):
    # A = I, asymmetric B: catches a transposed C write
    M = N = K = 256
    x = torch.eye(M, K).bfloat16()
    w = torch.arange(N * K, dtype=torch.float32).reshape(N, K).remainder(97).sub(48).bfloat16()
    got = ops.linear(x.to(DEV), w.to(DEV), tile=tile).cpu().float()
    assert torch.equal(got, w.float().t())


def test_gemm_row_scatter_table_f32out():
    B, P, S, W, K = 3, 16, 17, 128, 192
    x = torch.randn(B * P, K).bfloat16()
    w = (torch.randn(W, K) * 0.1).bfloat16()
    pos = torch.randn(S, W).bfloat16()
    out_ref = torch.zeros(B * S, W).bfloat16()
    ops.linear(x, w, table=pos, table_period=P, table_offset=1, out=out_ref, out_group=P, out_group_stride=S,
               out_row_offset=1)
    out = torch.zeros(B * S, W, device=DEV).bfloat16()
    ops.linear(x.to(DEV), w.to(DEV), table=pos.to(DEV), table_period=P, table_offset=1, out=out, out_group=P,
               out_group_stride=S, out_row_offset=1)
    assert _rel(out, out_ref) < 1e-2
    f = ops.linear(x.to(DEV), w.to(DEV), out_dtype=torch.float32)
    assert f.dtype == torch.float32 and _rel(f, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("rows,D", [(1, 64), (257, 1024), (1000, 768), (33, 4096), (7, 896), (5, 3584), (64, 8192), (65, 2048)])
def test_layernorm_rmsnorm(rows, D):
    x = torch.randn(rows, D).bfloat16() * 3
    w = torch.randn(D).bfloat16()
    b = torch.randn(D).bfloat16()
    assert _rel(ops.layer_norm(x.to(DEV), w.to(DEV), b.to(DEV)), ops.layer_norm(x, w, b)) < 1e-2
    add = torch.randn(rows, D).bfloat16()
    ro_ref = torch.empty_like(x)
    ro = torch.empty_like(x, device=DEV)
    ref = ops.rms_norm(x, w, add=add, resid_out=ro_ref)
    got = ops.rms_norm(x.to(DEV), w.to(DEV), add=add.to(DEV), resid_out=ro)
    assert _rel(got, ref) < 1e-2 and _rel(ro, ro_ref) < 1e-2


@pytest.mark.parametrize("rows,D", [(1, 4096), (16, 896), (300, 1024)])
def test_norm_add_inplace_residual(rows, D):
    """Decode-style fused residual update: resid_out aliases the add operand (block-per-row
    kernel for few rows, wave-per-row kernel for many), LayerNorm and RMSNorm."""
    g = torch.Generator().manual_seed(rows)
    y = torch.randn(rows, D, generator=g).bfloat16()
    r = torch.randn(rows, D, generator=g).bfloat16() * 4
    w, b = torch.randn(D, generator=g).bfloat16(), torch.randn(D, generator=g).bfloat16()
    r_ref = r.clone()
    ref = ops.layer_norm(y, w, b, add=r_ref, resid_out=r_ref)
    r_d = r.to(DEV)
    got = ops.layer_norm(y.to(DEV), w.to(DEV), b.to(DEV), add=r_d, resid_out=r_d)
    assert _rel(got, ref) < 1e-2 and _rel(r_d, r_ref) < 1e-2
    ref = ops.rms_norm(y, w, add=r_ref, resid_out=r_ref)
    got = ops.rms_norm(y.to(DEV), w.to(DEV), add=r_d, resid_out=r_d)
    assert _rel(got, ref) < 1e-2 and _rel(r_d, r_ref) < 1e-2


def test_layernorm_row_gather_and_l2():
    x = torch.randn(5 * 17, 256).bfloat16()
    w = torch.ones(256).bfloat16()
    idx = torch.arange(5) * 17
    ref = ops.layer_norm(x, w, row_idx=idx)
    got = ops.layer_norm(x.to(DEV), w.to(DEV), row_idx=idx.to(DEV))
    assert _rel(got, ref) < 1e-2
    e = torch.randn(9, 768)
    ops.l2_normalize_(e_d := e.to(DEV))
    assert torch.allclose(e_d.cpu(), e / e.norm(dim=-1, keepdim=True), atol=1e-5)


@pytest.mark.parametrize("B,Sq,Sk,H,Hkv,D,causal", [
    (2, 257, 257, 16, 16, 64, False), (3, 77, 77, 8, 8, 64, True), (1, 197, 197, 12, 12, 64, False),
    (2, 130, 130, 14, 2, 64, True), (1, 33, 300, 8, 2, 128, True), (2, 65, 65, 4, 4, 128, False),
    (2, 20, 20, 4, 4, 32, False)])
def test_attention_vs_fp32(B, Sq, Sk, H, Hkv, D, causal):
    g = torch.Generator().manual_seed(Sq * H + D)
    q = torch.randn(B, Sq, H, D, generator=g).bfloat16()
    k = torch.randn(B, Sk, Hkv, D, generator=g).bfloat16()
    v = torch.randn(B, Sk, Hkv, D, generator=g).bfloat16()
    ref = ops.attention(q, k, v, causal=causal)
    got = ops.attention(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal)
    assert _rel(got, ref) < 2e-2


def test_attention_packed_qkv_and_kv_len():
    B, S, H, D = 3, 52, 12, 64
    qkv = torch.randn(B, S, 3, H, D).bfloat16()
    kl = torch.tensor([52, 10, 31], dtype=torch.int32)
    ref = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], kv_len=kl)
    qd = qkv.to(DEV)
    got = ops.attention(qd[:, :, 0], qd[:, :, 1], qd[:, :, 2], kv_len=kl.to(DEV))
    assert _rel(got, ref) < 2e-2


@pytest.mark.parametrize("filt", ["pil_bicubic", "pil_bilinear", "cv2_linear", "cv2_cubic"])
def test_image_prep_matches_reference(filt):
    g = torch.Generator().manual_seed(1)
    imgs = [torch.randint(0, 256, (45, 61, 3), generator=g, dtype=torch.uint8),
            torch.randint(0, 256, (20, 16, 3), generator=g, dtype=torch.uint8)]
    kw = dict(mean=(0.48, 0.45, 0.40), std=(0.26, 0.26, 0.27), filter=filt)
    ref = ops.image_prep(imgs, (32, 32), **kw)
    got = ops.image_prep([i.to(DEV) for i in imgs], (32, 32), **kw)
    # one uint8 LSB of rounding slack
    assert (got.cpu() - ref).abs().max().item() <= 1.01 / (255 * 0.26)


def test_image_prep_patches_layout():
    imgs = torch.randint(0, 256, (2, 30, 30, 3), dtype=torch.uint8)
    ref = ops.image_prep(imgs, (16, 16), layout="patches", patch=8, kpad=256, out_dtype=torch.bfloat16)
    got = ops.image_prep(imgs.to(DEV), (16, 16), layout="patches", patch=8, kpad=256, out_dtype=torch.bfloat16)
    assert got.shape == (8, 256)
    assert (got.cpu().float() - ref.float()).abs().max().item() < 0.05
    assert got[:, 192:].abs().max().item() == 0


def test_embed_gather():
    table = torch.randn(100, 64).bfloat16()
    pos = torch.randn(9, 64).bfloat16()
    ids = torch.randint(0, 100, (3, 9))
    ref = ops.embed(ids, table, pos)
    got = ops.embed(ids.to(DEV), table.to(DEV), pos.to(DEV))
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("B,N,k", [(1, 1000, 5), (3, 100000, 10), (2, 37, 37), (4, 5000, 64)])
def test_row_topk_and_lse(B, N, k):
    s = torch.randn(B, N)
    v_ref, i_ref, lse_ref = ops.row_topk(s, k, scale=100.0, with_lse=True)
    v, i, lse = ops.row_topk(s.to(DEV), k, scale=100.0, with_lse=True)
    assert torch.allclose(v.cpu(), v_ref, atol=1e-6)
    assert torch.equal(i.cpu(), i_ref)
    assert torch.allclose(lse.cpu(), lse_ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("act", ["gelu", "quick_gelu", "silu", "gelu_tanh", "relu", "hardswish", "sigmoid"])
def test_gemm_activations(act):
    x = torch.randn(300, 128).bfloat16()
    w = (torch.randn(256, 128) * 0.2).bfloat16()
    ref = ops.linear(x, w, act=act)
    got = ops.linear(x.to(DEV), w.to(DEV), act=act)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(40 * 256, 2048, 1024), (600 * 256 + 77, 1024, 128), (3000, 768, 256)])
@pytest.mark.parametrize("tile", [7, 1007, 47, 17, 8, 48, 1008, 609, 709, 1709, 109, 909, 1929, 1829])
def test_gemm_persistent_multi_tile(M, N, K, tile):
    """Persistent kernel: several tiles per workgroup (cross-tile prefetch), epilogue with
    bias + GELU + residual, bf16 and fp32 outputs, with/without the tail split."""
    g = torch.Generator().manual_seed(M + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    xd, wd = x.to(DEV), w.to(DEV)
    got = ops.linear(xd, wd, b.to(DEV), act="gelu", residual=r.to(DEV), tile=tile).cpu().float()
    rows = torch.cat([torch.arange(0, 512), torch.arange(M // 2, M // 2 + 512), torch.arange(M - 700, M)])
    ref = ops.linear(x[rows], w, b, act="gelu", residual=r[rows])
    assert _rel(got[rows], ref) < 1e-2
    got32 = ops.linear(xd, wd, out_dtype=torch.float32, tile=tile).cpu()
    ref32 = x[rows].float() @ w.float().t()
    assert _rel(got32[rows], ref32) < 1e-2
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("M,N,K", [(40 * 256, 2048, 192), (24 * 256, 3072, 128), (600 * 256, 1024, 1024),
                                   (300 * 256, 768, 64 * 7)])
@pytest.mark.parametrize("tile", [709, 1709, 609, 809, 909, 1929])
@pytest.mark.parametrize("act", [None, "quick_gelu"])
def test_gemm_pingpong_fast_epilogue(M, N, K, tile, act):
    """Ping-pong kernels on interior tiles (bf16 bias -> FAST epilogue), several tiles per
    workgroup for the persistent form, odd and minimal K-tile counts (nk = 2, 3, 7): the
    cross-tile LDS-DMA stream and the vmcnt counts after each epilogue."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    r = torch.randn(M, N, generator=g).bfloat16()
    xd, wd, bd, rd = x.to(DEV), w.to(DEV), b.to(DEV), r.to(DEV)
    rows = torch.cat([torch.arange(0, 700), torch.randint(0, M, (1500,), generator=g), torch.arange(M - 700, M)])
    for kw in ({}, {"bias": b}, {"bias": b, "residual": r}):
        kd = {k: v.to(DEV) for k, v in kw.items()}
        got = ops.linear(xd, wd, act=act, tile=tile, **kd).cpu().float()
        kr = dict(kw)
        if "residual" in kr:
            kr["residual"] = r[rows]
        ref = ops.linear(x[rows], w, act=act, **kr)
        assert _rel(got[rows], ref) < 1e-2, kw.keys()
        assert torch.isfinite(got).all()


@pytest.mark.parametrize("tile", [-1, 5, 7, 709])
def test_gemm_tail_round_split(tile):
    # 66 row tiles x 4 column tiles: rows [0, 16384) on 256x256, the 300-row tail on 128x128
    M, N, K = 64 * 256 + 300, 1024, 512
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    ref = ops.linear(x, w, b, act="gelu", residual=r)
    got = ops.linear(x.to(DEV), w.to(DEV), b.to(DEV), act="gelu", residual=r.to(DEV), tile=tile)
    assert _rel(got, ref) < 1e-2
    assert _rel(got[-300:], ref[-300:]) < 1e-2
    ref32 = ops.linear(x, w, out_dtype=torch.float32)
    got32 = ops.linear(x.to(DEV), w.to(DEV), out_dtype=torch.float32, tile=tile)
    assert _rel(got32[-300:], ref32[-300:]) < 1e-2


@pytest.mark.parametrize("B,Sq,Sk,H,Hkv,D,causal", [
    (64, 257, 257, 16, 16, 64, False), (128, 77, 77, 8, 8, 64, True), (40, 100, 100, 32, 8, 128, False),
    (64, 197, 197, 16, 16, 32, False), (32, 300, 300, 32, 32, 64, True)])
def test_attention_kv_resident_path(B, Sq, Sk, H, Hkv, D, causal):
    # B*H >= 1024 and K/V <= 80 KiB -> the K/V-resident kernel
    g = torch.Generator().manual_seed(Sq + H + D)
    q = torch.randn(B, Sq, H, D, generator=g).bfloat16()
    k = torch.randn(B, Sk, Hkv, D, generator=g).bfloat16()
    v = torch.randn(B, Sk, Hkv, D, generator=g).bfloat16()
    kl = torch.randint(Sk // 2, Sk + 1, (B,), generator=g, dtype=torch.int32)
    ref = ops.attention(q, k, v, causal=causal, kv_len=kl)
    got = ops.attention(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal, kv_len=kl.to(DEV))
    assert _rel(got, ref) < 2e-2


def test_image_prep_center_crop_matches_reference():
    """centre-crop geometry (negative destination offsets) on the HIP prep kernels vs the CPU
    reference, patch-row layout as the CLIP towers consume it."""
    g = torch.Generator().manual_seed(3)
    imgs = [torch.randint(0, 256, (90, 61, 3), generator=g, dtype=torch.uint8),
            torch.randint(0, 256, (40, 120, 3), generator=g, dtype=torch.uint8)]
    kw = dict(mean=(0.48, 0.45, 0.40), std=(0.26, 0.26, 0.27), center_crop=True)
    ref = ops.image_prep(imgs, (32, 32), **kw)
    got = ops.image_prep([i.to(DEV) for i in imgs], (32, 32), **kw)
    assert (got.cpu() - ref).abs().max().item() <= 1.01 / (255 * 0.26)
    refp = ops.image_prep(imgs, (32, 32), layout="patches", patch=8, kpad=256, out_dtype=torch.bfloat16, **kw)
    gotp = ops.image_prep([i.to(DEV) for i in imgs], (32, 32), layout="patches", patch=8, kpad=256,
                          out_dtype=torch.bfloat16, **kw)
    assert (gotp.float().cpu() - refp.float()).abs().max().item() <= 0.05


@pytest.mark.parametrize("M,N,K,tile", [(24 * 256, 3072, 1024, 1629), (24 * 256, 4096, 1024, 609),
                                        (16 * 256, 1024, 1024, 709), (24 * 256 + 77, 3072, 1024, -1),
                                        (577, 3072, 1024, -1), (577, 4096, 1024, -1), (40, 768, 768, -1),
                                        (512 * 77, 2304, 768, -1), (300 * 256 + 300, 1024, 512, 609),
                                        (257 * 256, 3072, 1024, -1), (24 * 256, 3072, 1024, 1829),
                                        (16 * 256, 4096, 1024, 1929), (300 * 256 + 300, 1024, 512, 809),
                                        (24 * 256, 4096, 1024, 1839)])
@pytest.mark.parametrize("act", [None, "quick_gelu"])
def test_gemm_layernorm_folded(M, N, K, tile, act):
    """LayerNorm folded into the projection (ln_row_stats + gemm_lnf): ping-pong FAST form (interior
    tiles), persistent form, generic / tail-split / 128x128 / small-M epilogues, against the fp32
    LayerNorm + Linear reference."""
    g = torch.Generator().manual_seed(M + N)
    x = (torch.randn(M, K, generator=g) * 2 + 0.5).bfloat16()
    gam, bet = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    rows = torch.cat([torch.arange(0, min(M, 600)), torch.randint(0, M, (800,), generator=g),
                      torch.arange(max(0, M - 600), M)])
    ref = ops.linear(ops.layer_norm(x[rows].float(), gam, bet, 1e-5), w.float(), b.float(), act=act)
    wf, ca = ops.ln_fold_weights(w.to(DEV), b.to(DEV), gam.to(DEV).bfloat16(), bet.to(DEV).bfloat16())
    xd = x.to(DEV)
    st = ops.ln_row_stats(xd, 1e-5)
    st_ref = ops.ln_row_stats(x[rows], 1e-5)
    assert torch.allclose(st.cpu()[rows], st_ref, rtol=1e-4, atol=1e-5)
    got = ops.linear_lnf(xd, wf, ca, st, act=act, tile=tile).cpu().float()
    assert _rel(got[rows], ref) < 1e-2
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("case", ["vit_l14", "vit_b32", "ragged", "center_crop", "bilinear_swap", "upscale",
                                  "big_downscale", "pad_square", "odd_offsets"])
def test_image_prep_band_kernel_bit_identical_to_two_pass(case, monkeypatch):
    """csrc/image.hip prep_band_kernel (fused per-band ViT prep: uint8 row pass in LDS) against the
    two-pass prep_h / prep_v path it replaces for patch rows with the PIL filters: same weights,
    same accumulation order -> identical bf16 bits."""
    g = torch.Generator().manual_seed(11)
    r = lambda h, w: torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8)  # noqa: E731
    kw = dict(mean=(0.48, 0.46, 0.41), std=(0.27, 0.26, 0.28), layout="patches", out_dtype=torch.bfloat16)
    out, patch, kpad = (224, 14, 640)
    if case == "vit_l14":
        imgs = torch.randint(0, 256, (6, 256, 256, 3), generator=g, dtype=torch.uint8)
    elif case == "vit_b32":
        imgs, (out, patch, kpad) = torch.randint(0, 256, (3, 256, 256, 3), generator=g, dtype=torch.uint8), (224, 32, 3072)
    elif case == "ragged":
        imgs = [r(300, 200), r(97, 411), r(224, 224), r(640, 480)]
    elif case == "center_crop":
        imgs, kw["center_crop"] = [r(300, 200), r(97, 411), r(500, 500)], True
    elif case == "bilinear_swap":
        imgs, kw["filter"], kw["swap_rb"] = [r(333, 250), r(120, 90)], "pil_bilinear", True
    elif case == "upscale":
        imgs, (out, patch, kpad) = [r(40, 30), r(17, 64)], (336, 14, 640)
    elif case == "pad_square":           # VLM pad-to-square canvas with an integral pad value
        imgs, kw["pad"], (out, patch, kpad) = [r(200, 150), r(90, 160)], 122.0, (336, 14, 640)
        kw["geoms"] = None
    elif case == "odd_offsets":          # ragged flat buffer: rows start at unaligned byte offsets
        imgs = [r(37, 53), r(101, 77), r(64, 65)]
    else:
        imgs = [r(1024, 768), r(900, 1400)]
    if case == "pad_square":
        geoms, off = [], 0
        for im in imgs:
            geoms.append(ops.ImageGeom.pad_square(im.shape[0], im.shape[1], off, out))
            off += im.numel()
        kw["geoms"] = geoms
    if isinstance(imgs, torch.Tensor):
        dimgs = imgs.to(DEV)
    else:
        dimgs = [i.to(DEV) for i in imgs]
    monkeypatch.setattr(ops, "_PREP_BAND_LDS", 96 * 1024)   # every case through the band kernel
    assert ops._prep_band_bounds([ops.ImageGeom.resize(8, 8, 0, out, out)], 0, 2, patch, kpad, out,
                                 torch.bfloat16) is not None
    band = ops.image_prep(dimgs, (out, out), patch=patch, kpad=kpad, **kw)
    monkeypatch.setattr(ops, "_prep_band_bounds", lambda *a, **k: None)
    two = ops.image_prep(dimgs, (out, out), patch=patch, kpad=kpad, **kw)
    torch.cuda.synchronize()
    assert torch.equal(band.view(torch.int16), two.view(torch.int16))
    ref = ops.image_prep(imgs, (out, out), patch=patch, kpad=kpad, **kw)          # CPU reference
    assert (band.cpu().float() - ref.float()).abs().max().item() <= 0.05
