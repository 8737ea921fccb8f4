"""LayerNorm partials of a residual GEMM's output rows (ops.linear ln_part + ops.ln_part_finalize, the
CPU reference of the direct-store ping-pong epilogue in csrc/gemm_pp.hip): the merged statistics equal
ln_row_stats of the same rows, and the tower path with partials matches the one without."""
import torch

from lumen_amd import ops


def test_partials_finalize_match_row_stats():
    g = torch.Generator().manual_seed(0)
    M, N, K = 300, 1024, 96
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.1
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g) * 4 + 2
    part = torch.empty(M, N // 64, 2)
    y = ops.linear(x, w, b, residual=r, ln_part=part)
    assert torch.allclose(ops.ln_part_finalize(part, 1e-5), ops.ln_row_stats(y, 1e-5), rtol=1e-5, atol=1e-6)
    cols = ops._ln_slot_cols(N)
    assert sorted(cols.flatten().tolist()) == list(range(N))


def test_res_ln_ok_codes():
    assert ops.res_ln_ok(65792, 1024, 1849)
    assert ops.res_ln_ok(512, 256, 1829, torch.zeros(256, dtype=torch.bfloat16))
    assert not ops.res_ln_ok(65792, 1024, 1629)
    assert not ops.res_ln_ok(65792, 1024, 1949)
    assert not ops.res_ln_ok(65792 + 1, 1024, 1849)
    assert not ops.res_ln_ok(512, 256, 1849, torch.zeros(256))
