"""JPEG decode latency on the bench images: Pillow (full / DCT-scaled) vs the parallel entropy
decoder (host threads) + GPU reconstruction (utils/jpeg.py), per image, median of N.

    python tools/jpeg_bench.py [--n 30]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd._native import load_hip  # noqa: E402
from lumen_amd.utils import jpeg as J  # noqa: E402
from lumen_amd.utils.image import decode_rgb, encode_jpeg  # noqa: E402
from tools.face_ocr_bench import synth_image  # noqa: E402


def med(f, n):
    f()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(statistics.median(ts), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=30)
    a = ap.parse_args()
    load_hip(required=True)
    rng = np.random.default_rng(0)
    out = {"cpus": os.cpu_count(), "default_threads": J.default_threads()}
    for kind, (h, w) in [("noise", (768, 1024)), ("photo", (768, 1024)), ("noise", (256, 256))]:
        data = encode_jpeg(synth_image(rng, h, w, kind))
        key = f"{kind}_{w}x{h}_{len(data) // 1024}KiB"
        r = {"pil_full_ms": med(lambda: decode_rgb(data), a.n),
             "pil_draft_half_ms": med(lambda: decode_rgb(data, draft_to=(w // 2, h // 2)), a.n)}
        for th in (1, 4, 8, 16):
            r[f"coefs_{th}t_ms"] = med(lambda: J.decode_coefs(data, threads=th), a.n)

        def dev():
            J.decode_to_device(data, "cuda")
            torch.cuda.synchronize()

        r["device_decode_ms"] = med(dev, a.n)
        st = {}
        J.decode_to_device(data, "cuda", stats=st)
        r["stats"] = st
        out[key] = r
        print(key, r, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
