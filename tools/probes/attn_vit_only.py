"""ViT-L/14 attention only (b512, S 257, 16 heads x 64), 40 launches: the subject of a PMC pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lumen_amd import ops  # noqa: E402

qkv = torch.randn(512, 257, 3, 16, 64, device="cuda").bfloat16()
out = torch.empty(512, 257, 16, 64, device="cuda", dtype=torch.bfloat16)
for _ in range(40):
    ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], out=out)
torch.cuda.synchronize()
print("done")
