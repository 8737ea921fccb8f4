"""Per-workgroup timeline of the production ping-pong GEMM (tile 1629) on the ViT-L/14 b512 micro-batch
shapes (M = 256 * 257 rows), s_memrealtime (100 MHz): prologue (first K-tile landed), K-loop, epilogue, and
the gaps between a CU's consecutive tiles.  Epilogues: the LN-folded qkv / fc1 form (gemm_lnf, fc1 with
quick-GELU) and the bias + residual out-proj / fc2 form, as clip._block_steps issues them.

    python tools/gemm_pp_timeline.py [--tiles 1629,1829]

Several tile codes: each is timed and stamped in turn and its output compared with the first one's.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd import ops
from lumen_amd._native import hip_ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1629")
    ap.add_argument("--M", type=int, default=256 * 257)
    a = ap.parse_args()
    h = hip_ops()
    M = a.M
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
    st = torch.stack([torch.full((M,), 0.9, device=dev), torch.full((M,), -0.01, device=dev)], 1).contiguous()
    for name, N, K, kind in [("qkv_lnf", 3072, 1024, "lnf"), ("out_res", 1024, 1024, "res"),
                             ("fc1_lnf_gelu", 4096, 1024, "lnf_gelu"), ("fc2_res", 1024, 4096, "res")]:
        xa = x if K == 1024 else torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        nt = ((M + 255) // 256) * ((N + 255) // 256)
        ca = torch.randn(2, N, device=dev, generator=g).contiguous()
        b = torch.randn(N, device=dev, generator=g).bfloat16()
        res = torch.randn(M, N, device=dev, generator=g).bfloat16() if not kind.startswith("lnf") else None
        first = None
        for tile in [int(t) for t in a.tiles.split(",")]:
            first = probe(h, name, M, N, K, kind, xa, w, st, ca, b, res, tile, nt, first)


def probe(h, name, M, N, K, kind, xa, w, st, ca, b, res, tile, nt, first):
        dev = "cuda"
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dbg = torch.zeros(nt * 4, dtype=torch.int64, device=dev)
        if kind.startswith("lnf"):
            act = "quick_gelu" if kind == "lnf_gelu" else None

            def run():
                ops.linear_lnf(xa, w, ca, st, act=act, tile=tile, out=out)
        else:
            def run():
                ops.linear(xa, w, b, residual=res, out=out, tile=tile)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            run()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / 5
        h.gemm_set_dbg(dbg)
        run()
        torch.cuda.synchronize()
        h.gemm_set_dbg(dbg[:0])
        d = dbg.view(nt, 4).cpu().double() * 10e-3   # us
        t0 = d[:, 0].min()
        pro = (d[:, 1] - d[:, 0])
        loop = (d[:, 2] - d[:, 1])
        epi = (d[:, 3] - d[:, 2])
        span = (d[:, 3].max() - t0).item()
        # gap: sort tile ends; each later start pairs with the earliest unclaimed end (the CU it reuses)
        ends = (d[:, 3] - t0).sort().values
        starts = (d[:, 0] - t0).sort().values
        gaps = (starts[256:] - ends[:nt - 256]) if nt > 256 else torch.zeros(1)
        tiles_per_cu = nt / 256
        busy = (d[:, 3] - d[:, 0]).sum().item() / 256
        tf = 2 * M * N * K / (ms * 1e-3) / 1e12
        diff = 0.0 if first is None else ((out.float() - first.float()).abs().max() /
                                          first.float().abs().max()).item()
        print(f"{name:14s} tile {tile} diff {diff:.2e} M={M} N={N} K={K} tiles={nt} ({tiles_per_cu:.2f}/CU): {ms * 1e3:.1f} us ({tf:.0f} TF); "
              f"per tile median prologue {pro.median():.2f} / K-loop {loop.median():.2f} / epilogue {epi.median():.2f} us "
              f"(p90 {pro.quantile(.9):.2f} / {loop.quantile(.9):.2f} / {epi.quantile(.9):.2f}); "
              f"dispatch gap median {gaps.median():.2f} us; span {span:.1f} us, CU-busy {busy:.1f} us", flush=True)
        return out.clone() if first is None else first


if __name__ == "__main__":
    main()
