"""Does a small pageable H2D copy (torch.tensor(...).to(dev, non_blocking=True)) block the host
until the stream's queued work finishes?  Queues ~50 ms of GEMMs, then times the copy call."""
import time

import torch

dev = torch.device("cuda:0")
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    a @ a
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    a @ a
torch.cuda.synchronize()
gemm_ms = (time.perf_counter() - t) * 1e3
for name, mk in [("pageable", lambda: torch.arange(8192, dtype=torch.long)),
                 ("pinned", lambda: torch.arange(8192, dtype=torch.long).pin_memory())]:
    src = mk()
    torch.cuda.synchronize()
    for _ in range(20):
        a @ a
    t = time.perf_counter()
    d = src.to(dev, non_blocking=True)
    host_ms = (time.perf_counter() - t) * 1e3
    torch.cuda.synchronize()
    print(f"{name}: queued gemm work {gemm_ms:.1f} ms, host time of the copy call {host_ms:.2f} ms", flush=True)
