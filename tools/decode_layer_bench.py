"""One Llama-3-8B decode layer's projections (fp8 weights, M = 1 / 16 rows), graph-replayed:
RMSNorm kernel + plain skinny GEMMs (unfused) vs the norm-folded chain (ops.linear_dec: rstd
row scale from the producer's sums of squares, no norm launch).  Attention / RoPE are left
out -- this isolates what the folding changes.

    python tools/decode_layer_bench.py [--layers 8] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402

H, QKV, I = 4096, 6144, 14336


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    L = args.layers
    q = lambda n, k: ops.quantize_fp8_rows(torch.randn(n, k, device=dev) * k ** -0.5)  # noqa: E731
    layers = [dict(qkv=q(QKV, H), o=q(H, H), gu=q(2 * I, H), down=q(H, I),
                   ln1=torch.ones(H, device=dev, dtype=torch.bfloat16),
                   ln2=torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(L)]
    res = {"layers": L}
    for M in (1, 16):
        x = torch.randn(M, H, device=dev).bfloat16()
        h = torch.empty_like(x)
        att = torch.randn(M, H, device=dev).bfloat16()
        ssq = torch.zeros(32, H // 16, device=dev)

        def unfused():
            for l in layers:
                ops.rms_norm(x, l["ln1"], 1e-5, out=h)
                ops.linear(h, l["qkv"][0], w_scale=l["qkv"][1])
                ops.linear(att, l["o"][0], w_scale=l["o"][1], residual=x, out=x)
                ops.rms_norm(x, l["ln2"], 1e-5, out=h)
                g = ops.linear(h, l["gu"][0], w_scale=l["gu"][1], glu=True)
                ops.linear(g, l["down"][0], w_scale=l["down"][1], residual=x, out=x)

        def fused():
            for i, l in enumerate(layers):
                ops.linear_dec(x, l["qkv"][0], l["qkv"][1], norm_eps=1e-5, ssq_in=ssq if i else None)
                ops.linear_dec(att, l["o"][0], l["o"][1], residual=x, out=x, ssq_out=ssq)
                g = ops.linear_dec(x, l["gu"][0], l["gu"][1], glu=True, norm_eps=1e-5, ssq_in=ssq)
                ops.linear_dec(g, l["down"][0], l["down"][1], residual=x, out=x, ssq_out=ssq)

        for name, fn in (("unfused", unfused), ("fused", fused), ("unfused2", unfused), ("fused2", fused)):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                fn()
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            res[f"M{M}_{name}_us_per_layer"] = round(e0.elapsed_time(e1) * 1e3 / args.iters / L, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
