"""Target for rocprofv3 PMC passes: a few GEMM launches per shape/config (random data)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops

cfgs = [int(t) for t in os.environ.get("GEMM_TILES", "47,45").split(",")]
shapes = [(131584, 1024, 1024), (8192, 8192, 8192)]
for M, N, K in shapes:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for t in cfgs:
        for _ in range(3):
            ops.linear(x, w, out=out, tile=t)
    torch.cuda.synchronize()
print("done")
