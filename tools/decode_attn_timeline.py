"""Per-workgroup timeline of the paged decode attention (Llama-3-8B geometry: 32 q / 8 kv heads x 128,
bf16 cache), s_memrealtime stamps (100 MHz): start, each wave's block-loop end, partials published,
split ticket back, combine done -- medians over launches between cache-flushing writes.

    python tools/decode_attn_timeline.py [--ctx 650] [--configs 8:1,3:4,1:16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd._native import hip_ops, load_hip  # noqa: E402
from lumen_amd.ops import llm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=650)
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--configs", default="8:1,3:4,1:16")
    a = ap.parse_args()
    load_hip(required=True)
    h = hip_ops()
    dev = torch.device("cuda")
    H, Hkv, D, B = 32, 8, 128, 1
    NB = B * a.width + 4
    kc = torch.randn(NB, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.randn(NB, Hkv, D, 64, device=dev).bfloat16()
    bt = torch.randperm(NB, device=dev)[:B * a.width].view(B, a.width).int()
    ctx = torch.full((B,), a.ctx, device=dev, dtype=torch.int32)
    q = torch.randn(B, (H + 2 * Hkv) * D, device=dev).bfloat16()
    flush = torch.empty(256 << 20, device=dev, dtype=torch.uint8)
    for cfg in a.configs.split(","):
        ns, bps = (int(v) for v in cfg.split(":"))
        ws = {}
        o = llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv, workspace=ws, splits=(ns, bps))
        dbg = torch.zeros(B * Hkv * ns * 8, dtype=torch.int64, device=dev)
        rows = []
        ev = []
        for _ in range(a.iters):
            flush.add_(1)
            dbg.zero_()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            h.decode_set_dbg(dbg)
            s.record()
            llm.paged_decode(q, kc, vc, bt, ctx, H, Hkv, workspace=ws, splits=(ns, bps), out=o)
            e.record()
            h.decode_set_dbg(dbg[:0])
            e.synchronize()
            ev.append(s.elapsed_time(e) * 1000)
            d = dbg.view(-1, 8).cpu().double() * 10e-3
            t0 = d[:, 0][d[:, 0] > 0].min()
            live = d[:, 0] > 0
            dd = d[live]
            loop_end = dd[:, 1:5].max(1).values - t0
            pub = dd[:, 5] - t0
            tick = dd[:, 6] - t0
            comb = dd[:, 7][dd[:, 7] > 0] - t0
            rows.append([(dd[:, 0] - t0).max().item(), loop_end.median().item(), loop_end.max().item(),
                         pub.max().item(), tick.max().item() if ns > 1 else 0.0,
                         comb.max().item() if comb.numel() else 0.0])
        r = torch.tensor(rows).median(0).values.tolist()
        ev.sort()
        print(f"{cfg}: event {ev[len(ev) // 2]:.2f} us | stamps rel. first WG start (us): last WG start {r[0]:.2f}, "
              f"block loops end median {r[1]:.2f} / max {r[2]:.2f}, partials published {r[3]:.2f}, ticket back {r[4]:.2f}, "
              f"combine done {r[5]:.2f}", flush=True)


if __name__ == "__main__":
    main()
