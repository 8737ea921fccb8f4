"""CPU references of the MX (block-scaled fp8) W8A8 chain: quantisation round trip, the E8M0
exponent rule and linear_mx's epilogues against plain fp32 math (the GPU kernels are checked
against these in tests/test_mx_gpu.py)."""
import torch

from lumen_amd import ops


def test_mx_quant_round_trip_and_exponent_rule():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 256, generator=g) * torch.exp2(torch.randint(-20, 20, (9, 8), generator=g).float()).repeat_interleave(32, 1)
    x[0, :32] = 0
    x[1, :32] = 448.0 * 4        # amax / 448 a power of two: e = 2 exactly, no clamping
    q, s = ops.mx_quant_ref(x)
    sr = ops.mx_rows(s)
    assert sr[0, 0].item() == 0 and sr[1, 0].item() == 129 and torch.equal(ops.mx_planes(sr), s)
    d = ops.mx_dequant(q, s)
    assert ((d - x).abs() <= x.abs() * 2 ** -4 + 1e-30).all()
    blk = x.abs().reshape(9, 8, 32).amax(-1)
    sc = torch.exp2(sr.float() - 127)
    assert (blk / sc <= 448).all() and ((blk == 0) | (blk / sc > 224)).all()


def test_linear_mx_reference_epilogues():
    g = torch.Generator().manual_seed(1)
    M, N, K = 20, 256, 384
    x = torch.randn(M, K, generator=g)
    x8, xs = ops.mx_quant_ref(x)
    w8, sw = ops.quantize_fp8_rows(torch.randn(N, K, generator=g) * K ** -0.5)
    wf = w8.float() * sw[:, None]
    xd = ops.mx_dequant(x8, xs)
    ssq = (x ** 2).reshape(M, K // 128, 128).sum(-1)
    y = ops.linear_mx(x8, xs, w8, sw, ssq_in=ssq, norm_eps=1e-6)
    ref = (xd @ wf.t()) * torch.rsqrt((x ** 2).mean(1, keepdim=True) + 1e-6)
    assert torch.allclose(y.float(), ref, rtol=2e-2, atol=2e-2)
    q8, qs = torch.empty(M, N // 2, dtype=torch.float8_e4m3fn), torch.empty(N // 256, M, 4, dtype=torch.uint8)
    out = ops.linear_mx(x8, xs, w8, sw, glu=True, q_out=(q8, qs))
    gu = (xd @ wf.t()).view(M, N // 16, 2, 8)
    r = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, N // 2)
    assert torch.allclose(out.float(), r, rtol=2e-2, atol=2e-2)
    assert torch.allclose(ops.mx_dequant(q8, qs), r, rtol=7e-2, atol=1e-3)
