"""CPU reference of the NHWC CNN ops vs PyTorch NCHW functional ops."""
import torch
import torch.nn.functional as F

from lumen_amd.ops import cnn


def test_conv_ref_matches_nchw():
    x = torch.randn(2, 9, 11, 8)
    w = torch.randn(16, 8, 3, 3)
    b = torch.randn(16)
    y = cnn.conv2d(x, cnn.conv_weight_from_torch(w), b, 2, 1)
    ref = F.conv2d(x.permute(0, 3, 1, 2), w, b, 2, 1).permute(0, 2, 3, 1)
    assert torch.allclose(y, ref, atol=1e-4)


def test_pixel_shuffle_is_convtranspose():
    x = torch.randn(1, 4, 5, 8)
    wt = torch.randn(8, 16, 2, 2)  # ConvTranspose2d weight [Cin, Cout, kh, kw]
    ref = F.conv_transpose2d(x.permute(0, 3, 1, 2), wt, stride=2).permute(0, 2, 3, 1)
    # GEMM weight [(dy*2+dx)*Cout + c, Cin]
    wg = wt.permute(2, 3, 1, 0).reshape(4 * 16, 8)
    y = (x.reshape(-1, 8) @ wg.t()).reshape(1, 4, 5, 64)
    got = cnn.pixel_shuffle_up(y, 16, 2)
    assert torch.allclose(got, ref, atol=1e-5)
