"""Implicit-GEMM conv timing on the IResNet-100 / SCRFD layer shapes (face pipeline, batch of
128 aligned faces = 32 images x 4): every conv_lds variant (tile 10 + v) per shape, cold-ish
(inputs rotate over 4 buffers), HIP-event timed; prints us and TFLOP/s per (shape, variant).

  python tools/conv_bench.py [--faces 128] [--variants 0,1,2,5,6] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lumen_amd.ops import cnn

SHAPES = {  # name: (H, W, Cin, Cout, K, stride)
    "ires_s1_112": (112, 112, 64, 64, 3, 1),
    "ires_s1_56": (56, 56, 64, 64, 3, 1),
    "ires_s2_28": (28, 28, 128, 128, 3, 1),
    "ires_s3_14": (14, 14, 256, 256, 3, 1),
    "ires_s4_7": (7, 7, 512, 512, 3, 1),
    "ires_s3_down": (28, 28, 128, 256, 3, 2),
    "ires_stem": (112, 112, 8, 64, 3, 1),
    "scrfd_stem1": (640, 640, 8, 32, 3, 2),
    "scrfd_stem2": (320, 320, 32, 32, 3, 1),
    "scrfd_stem3": (320, 320, 32, 64, 3, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--faces", type=int, default=128)
    ap.add_argument("--variants", default="0,1,2,5,6,8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--tiles", default=None,
                    help="raw conv tile codes instead of --variants (-1 auto, 0..2 register-staged igemm, "
                         "10 + v the LDS pipeline variant v)")
    ap.add_argument("--epi", default="prelu_res", choices=["prelu_res", "res_aff"],
                    help="prelu_res: bias + PReLU + residual; res_aff: IResNet conv2 -- bias + residual + the "
                         "next block's BN as a second output")
    a = ap.parse_args()
    dev = "cuda"
    out = []
    for name in a.shapes.split(","):
        H, W, Cin, Cout, K, s = SHAPES[name]
        nb = a.faces // 4 if name.startswith("scrfd") else a.faces      # detector: 32 images per 128 faces
        xs = [torch.randn(nb, H, W, Cin, device=dev).bfloat16() for _ in range(4)]
        w = (torch.randn(Cout, K, K, Cin, device=dev) * (K * K * Cin) ** -0.5).bfloat16()
        b = torch.randn(Cout, device=dev).bfloat16()
        pr = (torch.rand(Cout, device=dev) * 0.3).bfloat16()
        Ho, Wo = cnn.conv_out_hw(H, W, K, K, s, K // 2, 1)
        res = torch.randn(nb, Ho, Wo, Cout, device=dev).bfloat16()
        flops = 2.0 * nb * Ho * Wo * Cout * K * K * Cin
        sc, sh = 1 + 0.1 * torch.randn(Cout, device=dev), 0.1 * torch.randn(Cout, device=dev)
        ao = torch.empty_like(res)
        kw = dict(prelu=pr, residual=res) if a.epi == "prelu_res" else dict(residual=res, aff=(sc, sh), aff_out=ao)
        ref = None
        codes = [int(t) for t in a.tiles.split(",")] if a.tiles else \
            [-1 if int(v) == 0 else 10 + int(v) for v in a.variants.split(",")]
        for tile in codes:
            v = tile
            y = cnn.conv2d(xs[0], w, b, s, K // 2, 1, tile=tile, **kw)
            if ref is None:
                ref = y.float()
            err = ((y.float() - ref).norm() / ref.norm()).item()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                cnn.conv2d(xs[i % 4], w, b, s, K // 2, 1, tile=tile, out=y, **kw)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            r = {"shape": name, "variant": v, "epi": a.epi, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                 "rel_err_vs_first": round(err, 5)}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
