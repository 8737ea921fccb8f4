"""Implicit-GEMM conv / depthwise / pooling / FPN kernels vs the PyTorch fp32 reference."""
import pytest
import torch

from lumen_amd.ops import cnn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("N,H,W,Cin,Cout,K,s,p,d", [
    (2, 33, 31, 8, 16, 3, 1, 1, 1), (1, 64, 64, 32, 64, 3, 2, 1, 1), (2, 20, 20, 64, 128, 1, 1, 0, 1),
    (1, 17, 19, 16, 32, 5, 1, 2, 1), (1, 40, 40, 24, 48, 3, 1, 2, 2), (3, 28, 28, 128, 256, 3, 2, 1, 1),
    (1, 112, 112, 8, 64, 3, 1, 1, 1), (2, 7, 7, 512, 512, 3, 1, 1, 1)])
@pytest.mark.parametrize("tile", [-1, 0, 1, 2])
def test_conv2d(N, H, W, Cin, Cout, K, s, p, d, tile):
    g = torch.Generator().manual_seed(H * Cin + K)
    x = torch.randn(N, H, W, Cin, generator=g).bfloat16()
    w = (torch.randn(Cout, K, K, Cin, generator=g) * (K * K * Cin) ** -0.5).bfloat16()
    b = torch.randn(Cout, generator=g).bfloat16()
    pr = (torch.rand(Cout, generator=g) * 0.3).bfloat16()
    ref = cnn.conv2d(x, w, b, s, p, d, act=None, prelu=pr)
    got = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, d, prelu=pr.to(DEV), tile=tile)
    assert got.shape == ref.shape
    assert _rel(got, ref) < 1e-2
    r = torch.randn(*ref.shape, generator=g).bfloat16()
    ref2 = cnn.conv2d(x, w, b, s, p, d, act="relu", residual=r)
    got2 = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, d, act="relu", residual=r.to(DEV), tile=tile)
    assert _rel(got2, ref2) < 1e-2
    # ResNet tail: relu(conv + bias + shortcut)
    ref3 = cnn.conv2d(x, w, b, s, p, d, residual=r, post_act="relu")
    got3 = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, d, residual=r.to(DEV), tile=tile, post_act="relu")
    assert _rel(got3, ref3) < 1e-2 and got3.min().item() >= 0


@pytest.mark.parametrize("N,H,W,Cin,Cout,K,s,p,d", [
    (2, 20, 20, 64, 128, 1, 1, 0, 1), (3, 28, 28, 128, 256, 3, 2, 1, 1), (2, 7, 7, 512, 512, 3, 1, 1, 1),
    (4, 56, 56, 64, 64, 3, 1, 1, 1), (2, 30, 30, 64, 48, 3, 1, 2, 2), (1, 13, 9, 192, 80, 5, 2, 2, 1)])
@pytest.mark.parametrize("tile", [-1, 11, 12, 13, 14, 15, 16, 17, 18])
def test_conv2d_lds_pipeline(N, H, W, Cin, Cout, K, s, p, d, tile):
    """Cin % 64 == 0: the LDS-DMA implicit-GEMM pipeline (conv_lds.hip; -1 picks it), incl. zero
    padding taps, stride / dilation, residual + PReLU + post-ReLU epilogues."""
    g = torch.Generator().manual_seed(H * Cin + K + Cout)
    x = torch.randn(N, H, W, Cin, generator=g).bfloat16()
    w = (torch.randn(Cout, K, K, Cin, generator=g) * (K * K * Cin) ** -0.5).bfloat16()
    b = torch.randn(Cout, generator=g).bfloat16()
    pr = (torch.rand(Cout, generator=g) * 0.3).bfloat16()
    ref = cnn.conv2d(x, w, b, s, p, d, act=None, prelu=pr)
    got = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, d, prelu=pr.to(DEV), tile=tile)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2
    r = torch.randn(*ref.shape, generator=g).bfloat16()
    ref3 = cnn.conv2d(x, w, b, s, p, d, residual=r, post_act="relu")
    got3 = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, d, residual=r.to(DEV), tile=tile, post_act="relu")
    assert _rel(got3, ref3) < 1e-2 and got3.min().item() >= 0


@pytest.mark.parametrize("N,H,W,Cin,Cout,K,s,p", [
    (2, 33, 31, 8, 32, 3, 2, 1), (1, 40, 40, 32, 32, 3, 1, 1), (2, 21, 19, 32, 64, 3, 2, 1),
    (3, 28, 28, 8, 64, 3, 1, 1), (1, 17, 23, 16, 48, 5, 1, 2), (2, 12, 12, 32, 128, 1, 1, 0)])
@pytest.mark.parametrize("tile", [-1, 19, 20, 21])
def test_conv2d_lds_small_cin(N, H, W, Cin, Cout, K, s, p, tile):
    """Cin 8 / 16 / 32: the LDS-DMA pipeline with several filter taps per 64-wide K step (per-lane
    tap offsets, zero taps past KH * KW in the last step), every tile width."""
    g = torch.Generator().manual_seed(H * Cin + K + Cout)
    x = torch.randn(N, H, W, Cin, generator=g).bfloat16()
    w = (torch.randn(Cout, K, K, Cin, generator=g) * (K * K * Cin) ** -0.5).bfloat16()
    b = torch.randn(Cout, generator=g).bfloat16()
    pr = (torch.rand(Cout, generator=g) * 0.3).bfloat16()
    ref = cnn.conv2d(x, w, b, s, p, 1, act="relu", prelu=pr)
    got = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, 1, act="relu", prelu=pr.to(DEV), tile=tile)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2
    r = torch.randn(*ref.shape, generator=g).bfloat16()
    ref3 = cnn.conv2d(x, w, b, s, p, 1, residual=r, post_act="relu")
    got3 = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), s, p, 1, residual=r.to(DEV), tile=tile, post_act="relu")
    assert _rel(got3, ref3) < 1e-2


@pytest.mark.parametrize("Cin,tile", [(8, -1), (64, -1), (64, 12), (128, 15)])
def test_conv2d_output_affine(Cin, tile):
    """The next layer's channel affine emitted by the conv epilogue: as a second output next to the
    plain result, and in place of it (both vs the fp32 reference of conv -> round -> affine)."""
    g = torch.Generator().manual_seed(Cin + tile)
    x = torch.randn(2, 18, 18, Cin, generator=g).bfloat16()
    w = (torch.randn(64, 3, 3, Cin, generator=g) * (9 * Cin) ** -0.5).bfloat16()
    b = torch.randn(64, generator=g).bfloat16()
    r = torch.randn(2, 18, 18, 64, generator=g).bfloat16()
    sc, sh = 1 + 0.1 * torch.randn(64, generator=g), 0.1 * torch.randn(64, generator=g)
    ref = cnn.conv2d(x, w, b, 1, 1, 1, residual=r)
    ref_aff = (ref.float() * sc + sh)
    out, ao = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), 1, 1, 1, residual=r.to(DEV), tile=tile,
                         aff=(sc.to(DEV), sh.to(DEV)), aff_out=True)
    assert _rel(out, ref) < 1e-2 and _rel(ao, ref_aff) < 1e-2
    # the affine of exactly the stored bf16 output
    exact = out.float() * sc.to(DEV) + sh.to(DEV)
    assert (ao.float() - exact).abs().max().item() <= 0.02 * exact.abs().max().item()
    inplace = cnn.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), 1, 1, 1, residual=r.to(DEV), tile=tile,
                         aff=(sc.to(DEV), sh.to(DEV)))
    assert torch.equal(inplace, ao)


def test_conv2d_into_channel_slice():
    x = torch.randn(1, 16, 16, 32).bfloat16()
    w = (torch.randn(16, 3, 3, 32) * 0.05).bfloat16()
    big = torch.zeros(1, 16, 16, 64, device=DEV).bfloat16()
    cnn.conv2d(x.to(DEV), w.to(DEV), None, 1, 1, out=big[..., 16:32])
    ref = cnn.conv2d(x, w, None, 1, 1)
    assert _rel(big[..., 16:32], ref) < 1e-2
    assert big[..., :16].abs().max().item() == 0 and big[..., 32:].abs().max().item() == 0


@pytest.mark.parametrize("C,K,s", [(16, 3, 1), (64, 3, 2), (128, 5, 1), (24, 3, 1), (96, 7, 1), (80, 7, 2), (32, 5, 2)])
def test_depthwise(C, K, s):
    x = torch.randn(2, 30, 26, C).bfloat16()
    w = torch.randn(K, K, C).bfloat16() * 0.2
    b = torch.randn(C).bfloat16()
    ref = cnn.conv2d_dw(x, w, b, s, K // 2, act="hardswish")
    got = cnn.conv2d_dw(x.to(DEV), w.to(DEV), b.to(DEV), s, K // 2, act="hardswish")
    assert _rel(got, ref) < 1e-2


def test_pool_affine_upsample_scale_shuffle():
    x = torch.randn(2, 17, 15, 32).bfloat16()
    for mx in (True, False):
        assert _rel(cnn.pool2d(x.to(DEV), 3, 2, 1, mx), cnn.pool2d(x, 3, 2, 1, mx)) < 1e-2
    assert _rel(cnn.global_avgpool(x.to(DEV)), cnn.global_avgpool(x)) < 1e-3
    sc, sh = torch.rand(32) + 0.5, torch.randn(32)
    pr = torch.rand(32).bfloat16()
    assert _rel(cnn.channel_affine(x.to(DEV), sc.to(DEV), sh.to(DEV), prelu=pr.to(DEV)),
                cnn.channel_affine(x, sc, sh, prelu=pr)) < 1e-2
    add = torch.randn(2, 34, 30, 32).bfloat16()
    assert _rel(cnn.upsample_add(x.to(DEV), add.to(DEV), 2), cnn.upsample_add(x, add, 2)) < 1e-2
    s = torch.rand(2, 32)
    a = x.clone()
    b = x.to(DEV)
    assert _rel(cnn.channel_scale_(b, s.to(DEV)), cnn.channel_scale_(a, s)) < 1e-2
    y = torch.randn(2, 5, 6, 4 * 16).bfloat16()
    assert torch.equal(cnn.pixel_shuffle_up(y.to(DEV), 16, 2).cpu(), cnn.pixel_shuffle_up(y, 16, 2))
