"""Mid-size bf16 GEMMs (LLaVA vision tower: ViT-L/14-336 at 577 tokens) through ops.linear with
the auto tile choice (128x128 LDS-DMA pipeline, K split for the small grids), next to the same
product through torch (hipBLASLt, bias/activation/residual as separate ops) as the library baseline.

    python tools/mid_gemm_bench.py [--M 577]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402

SHAPES = [("qkv", 3072, 1024, None, False), ("out", 1024, 1024, None, True), ("fc1", 4096, 1024, "quick_gelu", False),
          ("fc2", 1024, 4096, None, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=577)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tiles", default="-1", help="comma list of forced tile codes (ops.linear tile=)")
    a = ap.parse_args()
    load_hip(required=True)
    dev = "cuda"
    tot = 0.0
    res = {"M": a.M}

    def med_us(f):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                f()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / a.iters * 1e3)
        return statistics.median(ts)

    for name, N, K, act, resid in SHAPES:
        x = torch.randn(a.M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        r = torch.randn(a.M, N, device=dev).bfloat16() if resid else None
        out = torch.empty(a.M, N, device=dev, dtype=torch.bfloat16)
        for t in [int(v) for v in a.tiles.split(",")][1:]:
            g = lambda: ops.linear(x, w, b, act=act, residual=r, out=out, tile=t)  # noqa: E731
            res[f"{name}_t{t}_us"] = round(med_us(g), 2)
        t0 = int(a.tiles.split(",")[0])
        f = lambda: ops.linear(x, w, b, act=act, residual=r, out=out, tile=t0)  # noqa: E731

        def lib():
            y = torch.nn.functional.linear(x, w, b)
            if act:
                y = y * torch.sigmoid(1.702 * y)
            return y + r if resid else y

        us = med_us(f)
        res[f"{name}_torch_us"] = round(med_us(lib), 2)
        tot += us
        res[f"{name}_us"] = round(us, 2)
        res[f"{name}_tf"] = round(2 * a.M * N * K / us / 1e6, 1)
    res["layer_us"] = round(tot, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
