"""The fused DBNet head tail's weight packing (ops/cnn.py db_head_pack_up2), checked on the CPU by
emulating csrc/conv.hip db_head_up_kernel's MFMA data flow lane by lane against the unfused
up1 -> pixel shuffle -> up2 path of models/ocr.py DBNet (fp32)."""
import numpy as np
import pytest
import torch

from lumen_amd.models.ocr import ConvT2
from lumen_amd.ops import cnn


def _emulate(h, w1, b1, w2p, b2):
    """numpy model of db_head_up_kernel: h [N, H4, W4, C] -> [N, 4*H4, 4*W4]"""
    N, H4, W4, C = h.shape
    hp = h.reshape(-1, C)
    P = hp.shape[0]
    out = np.zeros((N, 4 * H4, 4 * W4), np.float32)
    for g in range((P + 15) // 16):
        px = np.arange(g * 16, min(P, g * 16 + 16))
        X = w1 @ hp[px].T + b1[:, None]                     # up1^T: [4C, px]
        Xr = np.maximum(X, 0.0)
        Y = np.zeros((16, len(px)), np.float32)
        for s1 in range(4):
            # B operand of k-step s1: lane (px, hq) element j = channel c(hq, j) of sub-position s1
            B = np.zeros((32, len(px)), np.float32)
            for k in range(32):
                hq, j = k // 8, k % 8
                c = 4 * hq + j if j < 4 else 12 + 4 * hq + j
                if c < C:
                    B[k] = Xr[s1 * C + c]
            A = np.zeros((16, 32), np.float32)
            for row in range(16):
                for k in range(32):
                    A[row, k] = w2p[s1, row + 16 * (k // 8), k % 8]
            Y += A @ B
        for q, p in enumerate(px):
            n, rem = divmod(int(p), H4 * W4)
            yy, xx = divmod(rem, W4)
            for s1 in range(4):
                for s2 in range(4):
                    v = 1.0 / (1.0 + np.exp(-(Y[4 * s1 + s2, q] + b2[s2])))
                    out[n, 4 * yy + 2 * (s1 >> 1) + (s2 >> 1), 4 * xx + 2 * (s1 & 1) + (s2 & 1)] = v
    return out


@pytest.mark.parametrize("C", [16, 32])
def test_db_head_packing_matches_unfused(C):
    g = torch.Generator().manual_seed(C)
    up1 = ConvT2(C, C, act="relu")
    up2 = ConvT2(C, 1, act="sigmoid", out_dtype=torch.float32)
    up1.random_init(g)
    up2.random_init(g)
    up1.g.b.data[:4 * C] = torch.randn(4 * C, generator=g) * 0.1
    up2.g.b.data[:4] = torch.randn(4, generator=g) * 0.1
    N, H4, W4 = 2, 3, 5                       # 30 pixels: a partial 16-pixel group, groups spanning rows
    h = torch.randn(N, H4, W4, C, generator=g)
    # unfused reference (the CPU path of DBNet.forward's tail)
    y = up2.gemm(up1(h))
    ref = y.view(N, 2 * H4, 2 * W4, 2, 2).permute(0, 1, 3, 2, 4).reshape(N, 4 * H4, 4 * W4).float().numpy()
    w1 = up1.g.w[:4 * C, :C].float().numpy()
    b1 = up1.g.b[:4 * C].float().numpy()
    w2p = cnn.db_head_pack_up2(up2.g.w[:4, :C]).float().numpy()
    b2 = up2.g.b[:4].float().numpy()
    got = _emulate(h.numpy(), w1, b1, w2p, b2)
    np.testing.assert_allclose(got, ref, atol=2e-2)
