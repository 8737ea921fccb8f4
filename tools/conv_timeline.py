"""Per-workgroup timeline of the implicit-GEMM conv kernels (csrc/conv_lds.hip) on the face pipeline's
heaviest shapes -- the SCRFD 640 px stem (32 images, 8 -> 32 ch, 3x3 s2), the IResNet stem (128 faces,
8 -> 64 ch, 3x3 s1) and an IResNet stage-3 conv (128 faces, 256 -> 256 ch at 14x14) -- s_memrealtime stamps
(100 MHz): prologue (first K-stage landed), K-loop, epilogue (to the last store's completion), tile-to-tile
dispatch gaps.

    python tools/conv_timeline.py [--tiles -1,19,20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd.ops import cnn
from lumen_amd._native import hip_ops

SHAPES = [("scrfd_stem", 32, 640, 640, 8, 32, 2), ("iresnet_stem", 128, 112, 112, 8, 64, 1),
          ("iresnet_s3", 128, 14, 14, 256, 256, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="-1")
    ap.add_argument("--shapes", default=",".join(s[0] for s in SHAPES))
    a = ap.parse_args()
    h = hip_ops()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, H, W, Cin, Cout, s in SHAPES:
        if name not in a.shapes.split(","):
            continue
        x = torch.randn(N, H, W, Cin, device=dev, generator=g).bfloat16()
        w = (torch.randn(Cout, 3, 3, Cin, device=dev, generator=g) * 0.1).bfloat16()
        b = torch.randn(Cout, device=dev, generator=g).bfloat16()
        ref = None
        for tile in [int(t) for t in a.tiles.split(",")]:
            def run():
                return cnn.conv2d(x, w, b, stride=s, padding=1, act="relu", tile=tile)
            try:
                y = run()
            except RuntimeError as e:
                print(f"{name} tile {tile}: {str(e).splitlines()[0]}", flush=True)
                continue
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                run()
            ev[1].record()
            torch.cuda.synchronize()
            us = ev[0].elapsed_time(ev[1]) / 10 * 1e3
            M = N * y.shape[1] * y.shape[2]
            nwg = 1 << 20
            dbg = torch.zeros(nwg * 4, dtype=torch.int64, device=dev)
            h.gemm_set_dbg(dbg)
            y = run()
            torch.cuda.synchronize()
            h.gemm_set_dbg(dbg[:0])
            d = dbg.view(nwg, 4).cpu().double()
            d = d[d[:, 0] > 0] * 10e-3
            diff = 0.0 if ref is None else ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            ref = y if ref is None else ref
            gb = (x.numel() + y.numel()) * 2 / 1e9
            tf = 2 * M * Cout * 9 * Cin / (us * 1e-6) / 1e12
            if d.numel():
                t0 = d[:, 0].min()
                pro, loop, epi = d[:, 1] - d[:, 0], d[:, 2] - d[:, 1], d[:, 3] - d[:, 2]
                ends, starts = (d[:, 3] - t0).sort().values, (d[:, 0] - t0).sort().values
                k = min(256 * 3, len(starts) - 1)
                gaps = starts[k:] - ends[:len(starts) - k]
                stats = (f"{len(d)} WGs: prologue {pro.median():.2f} / K-loop {loop.median():.2f} / epilogue "
                         f"{epi.median():.2f} us per tile, gap {gaps.median():.2f} us, span {(d[:, 3].max() - t0).item():.1f} us")
            else:
                stats = "no stamps (kernel without them)"
            print(f"{name} tile {tile}: {us:.1f} us ({tf:.0f} TF, {gb / (us * 1e-6) / 1e3:.2f} TB/s of x+y) diff {diff:.1e}; "
                  f"{stats}", flush=True)


if __name__ == "__main__":
    main()
