"""ViT prep timing: b512 uint8 256x256 -> 224x224 PIL-bicubic patch rows (ViT-L/14: patch 14, kpad of the tower)
through ops.image_prep (geometry precomputed), HIP-event timed (best of 3 windows of 20): the fused
per-band kernel against the two-pass path."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402


def main():
    load_hip(required=True)
    dev = torch.device("cuda")
    res = {}
    for B, side, out, patch, kpad in [(512, 256, 224, 14, 640), (512, 256, 224, 32, 3072), (16, 1024, 336, 14, 640)]:
        imgs = torch.randint(0, 256, (B, side, side, 3), dtype=torch.uint8, device=dev)
        kw = dict(mean=(0.48, 0.46, 0.41), std=(0.27, 0.26, 0.28), filter="pil_bicubic", layout="patches",
                  patch=patch, kpad=kpad, out_dtype=torch.bfloat16, device=dev)
        geoms = [ops.ImageGeom.resize(side, side, i * side * side * 3, out, out) for i in range(B)]
        flat = imgs.reshape(-1)
        shapes = [torch.empty((side, side, 3), dtype=torch.uint8, device="meta")] * B
        band_fn = ops._prep_band_bounds
        for arm in ("two_pass", "band", "two_pass", "band"):
            ops._prep_band_bounds = band_fn if arm == "band" else (lambda *a, **k: None)
            for _ in range(3):
                ops.image_prep(shapes, (out, out), geoms=geoms, src=flat, **kw)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    ops.image_prep(shapes, (out, out), geoms=geoms, src=flat, **kw)
                e.record()
                torch.cuda.synchronize()
                best = min(best, s.elapsed_time(e) / 20)
            key = f"b{B}_{side}to{out}_p{patch}_{arm}_ms"
            res[key] = min(res.get(key, 1e9), round(best, 4))
        ops._prep_band_bounds = band_fn
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
