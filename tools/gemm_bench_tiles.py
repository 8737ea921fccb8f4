"""A/B of GEMM tile configurations (``ops.linear(tile=...)``) against hipBLASLt on given shapes.

Interleaved rounds in one process (cdna guide §5.4 rule 24): each round times every variant
once, the reported figure is the median over rounds.  Random normal operands.

  python tools/gemm_bench_tiles.py --tiles 47,5,9,109 --epi plain,bias_res [--shapes vit]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops

SHAPES = {
    "vit": [(131584, 3072, 1024), (131584, 1024, 1024), (131584, 4096, 1024), (131584, 1024, 4096)],
    "sq": [(4096, 4096, 4096), (8192, 8192, 8192)],
    "llm": [(624, 6144, 4096), (624, 4096, 4096), (624, 28672, 4096), (624, 4096, 14336)],
}


def timeit(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="-1,9")
    ap.add_argument("--epi", default="plain")
    ap.add_argument("--shapes", default="vit")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    shapes = []
    for s in a.shapes.split(","):
        shapes += SHAPES[s] if s in SHAPES else [tuple(int(v) for v in s.split("x"))]
    torch.manual_seed(0)
    for M, N, K in shapes:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        res = torch.randn(M, N, device="cuda").bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = None
        rows = torch.randint(0, M, (256,), device="cuda")
        variants = {}
        for epi in a.epi.split(","):
            kw = {}
            if epi in ("bias", "bias_res", "bias_gelu", "bias_qgelu"):
                kw["bias"] = b
            if epi == "bias_res":
                kw["residual"] = res
            if epi == "bias_gelu":
                kw["act"] = "gelu"
            if epi == "bias_qgelu":
                kw["act"] = "quick_gelu"
            # numerics vs fp32 on 256 sampled rows
            y = (x[rows].float() @ w.float().t())
            if "bias" in kw:
                y = y + b.float()
            if epi == "bias_gelu":
                y = torch.nn.functional.gelu(y)
            if epi == "bias_qgelu":
                y = y * torch.sigmoid(1.702 * y)
            if "residual" in kw:
                y = y + res[rows].float()
            for t in tiles:
                variants[f"t{t}_{epi}"] = (lambda t=t, kw=kw: ops.linear(x, w, out=out, tile=t, **kw), y)
        variants["hipblaslt"] = (lambda: torch.matmul(x, w.t(), out=out), None)
        r = {"M": M, "N": N, "K": K}
        for name, (fn, yref) in variants.items():
            fn()
            torch.cuda.synchronize()
            if yref is not None:
                got = out[rows].float()
                r[name + "_relerr"] = float((got - yref).norm() / yref.norm())
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for name, (fn, _) in variants.items():
                fn()
                times[name].append(timeit(fn, a.iters))
        for name, ts in times.items():
            ms = statistics.median(ts)
            r[name + "_ms"] = round(ms, 4)
            r[name + "_tf"] = round(2 * M * N * K / ms / 1e9, 1)
        print(json.dumps(r), flush=True)
        del x, w, res, out


if __name__ == "__main__":
    main()
