"""GEMM epilogue cost on the ViT-L/14 b512 shapes: plain vs +bias vs +bias+GELU vs +bias+residual
(auto tile selection, i.e. what the model runs), random data, vs hipBLASLt plain."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


for M, N, K in [(131584, 3072, 1024), (131584, 1024, 1024), (131584, 4096, 1024), (131584, 1024, 4096)]:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    b = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    r = {"M": M, "N": N, "K": K}
    tiles = [int(t) for t in os.environ.get("GEMM_TILES", "").split(",") if t]
    extra = []
    for tl in tiles:
        extra += [(f"t{tl}_plain", lambda tl=tl: ops.linear(x, w, out=out, tile=tl)),
                  (f"t{tl}_bias_res", lambda tl=tl: ops.linear(x, w, b, residual=res, out=out, tile=tl))]
    for name, fn in extra + [("plain", lambda: ops.linear(x, w, out=out)),
                     ("bias", lambda: ops.linear(x, w, b, out=out)),
                     ("bias_gelu", lambda: ops.linear(x, w, b, act="gelu", out=out)),
                     ("bias_res", lambda: ops.linear(x, w, b, residual=res, out=out)),
                     ("torch", lambda: torch.matmul(x, w.t(), out=out))]:
        ms = t(fn)
        r[name + "_ms"] = round(ms, 3)
        r[name + "_tf"] = round(2 * M * N * K / ms / 1e9, 1)
    print(json.dumps(r), flush=True)
