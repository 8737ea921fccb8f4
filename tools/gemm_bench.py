"""Microbenchmark: lumen HIP GEMM vs torch.matmul (hipBLASLt) on the ViT-L/14 shapes (random data)."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops

shapes = [(131584, 3072, 1024), (131584, 1024, 1024), (131584, 4096, 1024), (131584, 1024, 4096),
          (8192, 8192, 8192), (4096, 4096, 4096), (39424, 2304, 768)]
if os.environ.get("GEMM_SHAPES") == "ksweep":
    shapes = [(65536, 2048, k) for k in (64, 128, 256, 512, 1024, 2048, 4096)]
if os.environ.get("GEMM_SHAPES") == "probe":
    shapes = [(8192, 8192, 1024), (8192, 8192, 2048), (32768, 4096, 1024), (131584, 1024, 1024), (16384, 16384, 1024)]
res = []
for M, N, K in shapes:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    def run_t():
        torch.matmul(x, w.t(), out=out)
    r = {"M": M, "N": N, "K": K}
    variants = [("e0", lambda: ops.linear(x, w, out=out, tile=45)), ("torch", run_t),
                ("e1", lambda: ops.linear(x, w, out=out, tile=145)), ("e2", lambda: ops.linear(x, w, out=out, tile=245)),
                ("e3", lambda: ops.linear(x, w, out=out, tile=345)), ("p4", lambda: ops.linear(x, w, out=out, tile=47)),
                ("e0b", lambda: ops.linear(x, w, out=out, tile=45))]
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
    for tname, t in (("rel_err_e0", 45), ("rel_err_e1", 145), ("rel_err_e2", 245), ("rel_err_e3", 345)):
        out.zero_()
        ops.linear(x, w, out=out, tile=t)
        rows = torch.cat([torch.arange(0, 256), torch.arange(M - 256, M)]).cuda()
        ref = x[rows].float() @ w.float().t()
        r[tname] = float(((out[rows].float() - ref).norm() / ref.norm()).item())
    print(json.dumps(r), flush=True)
    res.append(r)
