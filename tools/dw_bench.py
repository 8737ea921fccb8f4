"""Depthwise-conv microbenchmark (FastViT / MobileCLIP shapes): register-blocked kernel vs
the one-pixel-per-thread kernel (LUMEN_DW_NAIVE=1), bf16 NHWC, random data."""
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
    outs = {}
    for name, naive in (("rb", False), ("naive", True)):
        if naive:
            os.environ["LUMEN_DW_NAIVE"] = "1"
        else:
            os.environ.pop("LUMEN_DW_NAIVE", None)
        for _ in range(3):
            y = cnn.conv2d_dw(x, w, b, s, K // 2, act="gelu")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            y = cnn.conv2d_dw(x, w, b, s, K // 2, act="gelu")
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        r[f"{name}_us"] = round(ms * 1e3, 1)
        r[f"{name}_GBs"] = round((x.numel() + y.numel()) * 2 / ms / 1e6, 1)
        outs[name] = y.float()
    os.environ.pop("LUMEN_DW_NAIVE", None)
    r["max_diff"] = float((outs["rb"] - outs["naive"]).abs().max())
    print(json.dumps(r), flush=True)
