"""Microbenchmark: lumen HIP GEMM vs torch.matmul (hipBLASLt) on the ViT-L/14 shapes (random data)."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops

shapes = [(131584, 3072, 1024), (131584, 1024, 1024), (131584, 4096, 1024), (131584, 1024, 4096),
          (8192, 8192, 8192), (4096, 4096, 4096), (39424, 2304, 768)]
res = []
for M, N, K in shapes:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    def run_t():
        torch.matmul(x, w.t(), out=out)
    r = {"M": M, "N": N, "K": K}
    variants = [("g1", lambda: ops.linear(x, w, out=out, tile=15)), ("g2", lambda: ops.linear(x, w, out=out, tile=25)),
                ("g4", lambda: ops.linear(x, w, out=out, tile=45)), ("g8", lambda: ops.linear(x, w, out=out, tile=85)),
                ("torch", run_t), ("ns4", lambda: ops.linear(x, w, out=out, tile=1045)),
                ("g4b", lambda: ops.linear(x, w, out=out, tile=45)), ("ns8", lambda: ops.linear(x, w, out=out, tile=1085)),
                ("g16", lambda: ops.linear(x, w, out=out, tile=165))]
    for name, fn in variants:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        n = 10
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / n
        r[name + "_ms"] = round(ms, 3)
        r[name + "_tflops"] = round(2 * M * N * K / ms / 1e9, 1)
    ref = (x[:256].float() @ w.float().t())
    ops.linear(x, w, out=out, tile=4)
    r["rel_err"] = float(((out[:256].float() - ref).norm() / ref.norm()).item())
    print(json.dumps(r), flush=True)
    res.append(r)
