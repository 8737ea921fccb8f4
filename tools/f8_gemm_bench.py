"""Prefill-shaped decoder projections: W8A8 fp8 MFMA (ops.linear_f8) vs the weight-only fp8
kernel (bf16 MFMA), hipBLASLt bf16 (torch.mm) and hipBLASLt fp8 (torch._scaled_mm, when the
build exposes it).  One JSON line per shape; times are medians of interleaved rounds.

  python tools/f8_gemm_bench.py [--M 624] [--shapes llama8b|qwen05b|NxK,...]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lumen_amd import ops  # noqa: E402

SHAPES = {
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gu", 28672, 4096), ("down", 4096, 14336)],
    "qwen05b": [("qkv", 1152, 896), ("o", 896, 896), ("gu", 9728, 896), ("down", 896, 4864)],
}


def _time(fn, iters, graph=False):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:       # decode-shaped launches replay from a hipGraph in serving: time them that way
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
    else:
        s.record()
        for _ in range(iters):
            fn()
        e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=624)
    ap.add_argument("--shapes", default="llama8b")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    shapes = []
    for s in a.shapes.split(","):
        if s in SHAPES:
            shapes += SHAPES[s]
        else:
            n, k = s.split("x")
            shapes.append((s, int(n), int(k)))
    dev = "cuda"
    M = a.M
    for name, N, K in shapes:
        glu = name == "gu"
        x = torch.randn(M, K, device=dev).bfloat16()
        w8, ws = ops.quantize_fp8_rows(torch.randn(N, K, device=dev) * K ** -0.5)
        wb = (w8.float() * ws[:, None]).bfloat16()
        x8, xs = ops.quant_rows_fp8(x)
        out = torch.empty(M, N // 2 if glu else N, device=dev, dtype=torch.bfloat16)
        outf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if M <= 32:     # decode: the weight-only fp8 skinny kernel (bf16 activations), graph-replayed
            f = lambda: ops.linear(x, w8, w_scale=ws, out=out, glu=glu)  # noqa: E731
            f()
            torch.cuda.synchronize()
            us = statistics.median(_time(f, a.iters, graph=True) for _ in range(a.rounds))
            nbytes = N * K + M * K * 2
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "w8_skinny_us": round(us, 2),
                              "GBs": round(nbytes / us / 1e3, 1)}), flush=True)
            continue
        cands = {
            "f8f8": lambda: ops.linear_f8(x8, xs, w8, ws, out=out, glu=glu),
            "f8f8_s1": lambda: ops.linear_f8(x8, xs, w8, ws, out=out, glu=glu, splits=1),
            "f8f8_s2": lambda: ops.linear_f8(x8, xs, w8, ws, out=out, glu=glu, splits=2),
            "f8f8_s4": lambda: ops.linear_f8(x8, xs, w8, ws, out=out, glu=glu, splits=4),
            "f8f8+quant": lambda: ops.linear_f8(*ops.quant_rows_fp8(x), w8, ws, out=out, glu=glu),
            "w8_bf16mfma": lambda: ops.linear(x, w8, w_scale=ws, out=out, glu=glu),
            "blas_bf16": lambda: torch.mm(x, wb.t(), out=outf),
        }
        if hasattr(torch, "_scaled_mm"):
            one = torch.ones((), device=dev)
            try:
                torch._scaled_mm(x8, w8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                cands["blas_f8"] = lambda: torch._scaled_mm(x8, w8.t(), scale_a=one, scale_b=one,
                                                            out_dtype=torch.bfloat16)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"note": f"_scaled_mm unavailable: {type(e).__name__}"}))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, f in cands.items():
                res[k].append(_time(f, a.iters))
        flop = 2.0 * M * N * K
        row = {"shape": name, "M": M, "N": N, "K": K}
        for k, v in res.items():
            us = statistics.median(v)
            row[k + "_us"] = round(us, 2)
            row[k + "_tflops"] = round(flop / us / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
