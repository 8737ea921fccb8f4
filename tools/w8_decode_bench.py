"""Decode-shaped fp8 weight GEMMs on the Llama-3-8B layer shapes, HBM-cold.

Each shape gets enough weight copies (>= 1 GiB in all, 4x the 256 MiB Infinity Cache) that
every GEMM of the graph-replayed chain streams its weights from HBM, as in a real decode
step; reports us per GEMM and achieved weight TB/s for M = 1 and 16 rows through
ops.linear_dec (the decode epilogue: rstd row scale for qkv / gate|up, residual + ssq for
o / down, fp32 logits for lm_head).

    python tools/w8_decode_bench.py [--m 1,16] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402

H, I, V = 4096, 14336, 128256
# name: (N, K, kind)
SHAPES = {"qkv": (6144, H, "norm"), "o": (H, H, "resid"), "gate_up": (2 * I, H, "glu"),
          "down": (H, I, "resid"), "lm_head": (V, H, "logits")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1,16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    out = {}
    for name in args.shapes.split(","):
        N, K, kind = SHAPES[name]
        copies = max(2, (1 << 30) // (N * K))
        ws = []
        for _ in range(copies):
            w8, s = ops.quantize_fp8_rows(torch.randn(N, K, device=dev) * K ** -0.5)
            ws.append((w8, s))
        for M in [int(m) for m in args.m.split(",")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            res = torch.randn(M, N, device=dev).bfloat16() if kind == "resid" else None
            ssq_in = torch.rand(M, K // 16, device=dev) if kind in ("norm", "glu", "logits") else None
            ssq_out = torch.zeros(M, N // 16, device=dev) if kind == "resid" else None

            def chain():
                for w8, s in ws:
                    if kind == "resid":
                        ops.linear_dec(x, w8, s, residual=res, out=res, ssq_out=ssq_out)
                    elif kind == "glu":
                        ops.linear_dec(x, w8, s, glu=True, norm_eps=1e-5, ssq_in=ssq_in)
                    elif kind == "logits":
                        ops.linear_dec(x, w8, s, norm_eps=1e-5, ssq_in=ssq_in, out_dtype=torch.float32)
                    else:
                        ops.linear_dec(x, w8, s, norm_eps=1e-5, ssq_in=ssq_in)

            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                chain()
            torch.cuda.current_stream().wait_stream(st)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                chain()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters / copies
            out[f"{name}_M{M}_us"] = round(us, 2)
            out[f"{name}_M{M}_TBs"] = round(N * K / us / 1e6, 2)
        del ws
        torch.cuda.empty_cache()
    for M in [int(m) for m in args.m.split(",")]:
        layer = sum(out.get(f"{n}_M{M}_us", 0.0) for n in ("qkv", "o", "gate_up", "down"))
        if layer:
            out[f"layer_M{M}_us"] = round(layer, 2)
            out[f"layer_M{M}_TBs"] = round(sum(SHAPES[n][0] * SHAPES[n][1] for n in ("qkv", "o", "gate_up", "down"))
                                           / layer / 1e6, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
