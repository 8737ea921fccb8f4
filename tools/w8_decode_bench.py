"""Decode-shaped fp8 weight GEMM bandwidth on the Llama-3-8B layer shapes (M = 1 and 16).

Times ops.linear(x[M, K], w8[N, K], w_scale) with hipEvents over many launches and
reports achieved weight GB/s.  The kernel variant comes from LUMEN_W8_SKINNY (read once
per process), so run one process per variant.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    load_hip(required=True)
    dev = torch.device("cuda")
    out = {"variant": int(os.environ.get("LUMEN_W8_SKINNY", "0"))}
    total_bytes, total_us = 0, 0.0
    for name, (N, K) in SHAPES.items():
        w8, s = ops.quantize_fp8_rows(torch.randn(N, K, device=dev) * K ** -0.5)
        for M in (1, 16):
            x = torch.randn(M, K, device=dev).bfloat16()
            for _ in range(5):
                ops.linear(x, w8, w_scale=s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 200
            e0.record()
            for _ in range(it):
                ops.linear(x, w8, w_scale=s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / it
            out[f"{name}_M{M}_us"] = round(us, 2)
            out[f"{name}_M{M}_GBs"] = round(N * K / us / 1e3, 1)
            if M == 1:
                total_bytes += N * K
                total_us += us
    out["layer_M1_us"] = round(total_us, 2)
    out["layer_M1_GBs"] = round(total_bytes / total_us / 1e3, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
