"""Paged decode attention alone (Llama-3-8B geometry: 32 q / 8 kv heads x 128, bf16 cache), graph-
timed per launch between cache-flushing writes (run under rocprofv3 --kernel-trace for
kernel-only durations), over split configurations (nsplit:min blocks per split) and an
optional weight prefetch of the o projection (16.8 MB fp8) in the same launch.

    python tools/decode_attn_bench.py [--ctx 650] [--batch 1] [--iters 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd._native import load_hip  # noqa: E402
from lumen_amd.ops import llm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=650)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--width", type=int, default=32, help="block-table width (blocks)")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--configs", default="8:1,8:4,3:4,11:1,32:1,1:32")
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    H, Hkv, D, B = 32, 8, 128, args.batch
    NB = B * args.width + 4
    kc = torch.randn(NB, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.randn(NB, Hkv, D, 64, device=dev).bfloat16()
    bt = torch.randperm(NB, device=dev)[:B * args.width].view(B, args.width).int()
    ctx = torch.full((B,), args.ctx, device=dev, dtype=torch.int32)
    q = torch.randn(B, (H + 2 * Hkv) * D, device=dev).bfloat16()
    ow = torch.empty(4096 * 4096, device=dev, dtype=torch.uint8)
    flush = [torch.empty(64 << 20, device=dev, dtype=torch.uint8) for _ in range(8)]   # > MALL between replays
    ref = llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv)
    out = {}
    for cfg in args.configs.split(","):
        ns, bps = (int(v) for v in cfg.split(":"))
        for pf in ((), (ow,)):
            ws = {}
            o = llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv, workspace=ws, splits=(ns, bps), prefetch=pf)
            err = float((o.float() - ref.float()).abs().max())
            ts = []
            for _ in range(args.iters):
                flush[0].add_(1)             # 64 MiB written: the K / V of this launch come from HBM / MALL
                flush[1].add_(1)
                flush[2].add_(1)
                flush[3].add_(1)
                flush[4].add_(1)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv, workspace=ws, splits=(ns, bps), prefetch=pf, out=o)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1000)
            ts.sort()
            out[f"{cfg}{'+pf' if pf else ''}"] = {"us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                                                  "max_abs_err": round(err, 4)}
    print(json.dumps({"ctx": args.ctx, "batch": B, "results": out}))


if __name__ == "__main__":
    main()
