"""Per-workgroup timeline of the 256x256 GEMM (s_memrealtime, 100 MHz): prologue / K-loop / epilogue."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd._native import hip_ops

ops = hip_ops()
for M, N, K in [(65536, 2048, 64), (65536, 2048, 1024), (8192, 8192, 1024)]:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nt = ((M + 255) // 256) * ((N + 255) // 256)
    dbg = torch.zeros(nt * 4, dtype=torch.int64, device="cuda")
    for _ in range(3):
        ops.gemm_probe(x, w, out, dbg, 1005)
    torch.cuda.synchronize()
    d = dbg.view(nt, 4).cpu().double() * 10e-3   # us
    t0 = d[:, 0].min()
    pro = (d[:, 1] - d[:, 0]).median().item()
    loop = (d[:, 2] - d[:, 1]).median().item()
    epi = (d[:, 3] - d[:, 2]).median().item()
    span = (d[:, 3].max() - t0).item()
    starts = (d[:, 0] - t0).sort().values
    print(f"M={M} N={N} K={K} tiles={nt}: median prologue {pro:.2f} us, K-loop {loop:.2f} us, epilogue {epi:.2f} us, "
          f"span {span:.1f} us; start of tile 256 at {starts[256].item():.2f} us, tile 512 at {starts[min(512, nt-1)].item():.2f}",
          flush=True)
