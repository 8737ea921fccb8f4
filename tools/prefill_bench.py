"""LLM prefill alone (Llama-3-8B shapes, fp8 W8A8 or bf16, random weights): GPU time (hipEvents)
vs host issue time of one ``LLM.prefill`` call -- tells whether prefill is launch-bound.

    python tools/prefill_bench.py [--preset llama3-8b] [--tokens 624] [--fp8]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd._native import load_hip  # noqa: E402
from lumen_amd.models.llm import LLM, LLM_PRESETS  # noqa: E402
from lumen_amd.runtime.kv_cache import PagedKVCache  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=624)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    cfg = LLM_PRESETS[a.preset]
    m = LLM(cfg, device=dev)
    m.random_init(0)
    if a.fp8:
        m.quantize_fp8()
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=64, device=dev)
    T = a.tokens
    slots = torch.arange(T, device=dev, dtype=torch.long)
    x0 = (torch.randn(T, cfg.hidden_size, device=dev) * 0.5).bfloat16()
    for _ in range(3):
        m.prefill(x0.clone(), kv, slots)
    torch.cuda.synchronize()
    gpu, issue = [], []
    for _ in range(a.iters):
        x = x0.clone()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        m.prefill(x, kv, slots)
        issue.append((time.perf_counter() - t0) * 1e3)
        e1.record()
        e1.synchronize()
        gpu.append(e0.elapsed_time(e1))
    print(json.dumps({"preset": a.preset, "tokens": T, "fp8": a.fp8, "gpu_ms": round(statistics.median(gpu), 3),
                      "host_issue_ms": round(statistics.median(issue), 3)}))


if __name__ == "__main__":
    main()
