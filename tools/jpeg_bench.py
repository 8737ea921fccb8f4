"""JPEG decode latency on the bench images: Pillow (full / DCT-scaled) vs the parallel entropy
decoder (host threads) + GPU reconstruction vs the GPU entropy decoder (csrc/jpeg_huff.hip) + GPU
reconstruction (utils/jpeg.py), per image and per batch of 32, median of N.

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

        def batch():
            J.decode_batch_to_device([data] * 32, "cuda")
            torch.cuda.synchronize()

        for mode in ("1", "0"):        # GPU entropy decode, then the host thread-pool decoder
            os.environ["LUMEN_JPEG_GPU_ENTROPY"] = mode
            tag = "gpu_entropy" if mode == "1" else "host_entropy"
            r[f"device_decode_{tag}_ms"] = med(dev, a.n)
            b = med(batch, max(5, a.n // 4))
            r[f"batch32_{tag}_ms"] = b
            r[f"batch32_{tag}_img_s"] = round(32e3 / b, 1)
        os.environ.pop("LUMEN_JPEG_GPU_ENTROPY")
        img = J.decode_to_device_gpu(data, "cuda")
        torch.cuda.synchronize()
        r["gpu_rounds"] = int(img.jpeg_err[1])
        st = {}
        J.decode_to_device(data, "cuda", stats=st)
        r["stats"] = st
        out[key] = r
        print(key, r, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
