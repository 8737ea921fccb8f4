"""Depthwise-conv microbenchmark (FastViT / MobileCLIP shapes): the register-blocked HIP kernel
(bf16 NHWC, fused bias + GELU) vs torch's depthwise conv (MIOpen, NCHW, separate bias/GELU),
with the max difference to an fp32 torch reference."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd.ops import cnn

SHAPES = [  # (N, H, W, C, K, stride)
    (1, 256, 256, 96, 3, 1), (1, 256, 256, 96, 7, 1), (1, 256, 256, 96, 7, 2), (1, 64, 64, 384, 7, 1),
    (64, 64, 64, 80, 3, 1), (64, 64, 64, 80, 7, 1), (64, 16, 16, 320, 7, 1), (64, 32, 32, 160, 7, 2),
]
for (N, H, W, C, K, s) in SHAPES:
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, K, C, device="cuda") * 0.1).bfloat16()
    b = torch.randn(C, device="cuda")
    r = {"N": N, "H": H, "W": W, "C": C, "K": K, "stride": s}
    xc = x.permute(0, 3, 1, 2).contiguous()
    wc = w.permute(2, 0, 1).unsqueeze(1).contiguous()
    bb = b.bfloat16()

    def ours():
        return cnn.conv2d_dw(x, w, b, s, K // 2, act="gelu")

    def lib():
        return torch.nn.functional.gelu(torch.nn.functional.conv2d(xc, wc, bb, s, K // 2, groups=C))

    for name, f in (("rb", ours), ("torch", lib)):
        for _ in range(3):
            y = f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            y = f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        r[f"{name}_us"] = round(ms * 1e3, 1)
        r[f"{name}_GBs"] = round((x.numel() + y.numel()) * 2 / ms / 1e6, 1)
    ref = torch.nn.functional.gelu(torch.nn.functional.conv2d(xc.float(), wc.float(), b, s, K // 2, groups=C))
    r["max_diff"] = float((ours().float() - ref.permute(0, 2, 3, 1)).abs().max())
    print(json.dumps(r), flush=True)
