"""FastViT-family towers on one MI355X: MobileCLIP2-S2 / -S4 image embeddings/s (batched, incl.
resize/normalise from uint8) and FastViTHD (FastVLM) single-image encode latency.
Synthetic data, random-init weights."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd.models.clip import CLIPModel
from lumen_amd.models.vlm import VLM, VLM_PRESETS


def timeit(fn, n, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    for preset in ("MobileCLIP2-S2", "MobileCLIP2-S4"):
        m = CLIPModel.random(preset, seed=0, device="cuda", with_text=False)
        imgs = torch.randint(0, 256, (args.batch, 256, 256, 3), dtype=torch.uint8, device="cuda")
        dt = timeit(lambda: m.encode_image_uint8(imgs), args.steps)
        print(json.dumps({"model": preset, "batch": args.batch, "images_per_s": round(args.batch / dt, 1),
                          "ms_per_batch": round(dt * 1e3, 3), "dtype": "bf16", "data": "synthetic"}), flush=True)
        del m
    v = VLM(VLM_PRESETS["fastvlm-0.5b"], device="cuda")
    v.random_init(0)
    img = [torch.randint(0, 256, (768, 1024, 3), dtype=torch.uint8, device="cuda")]
    dt = timeit(lambda: v.encode_images(img), 10)
    print(json.dumps({"model": "FastViTHD (fastvlm-0.5b vision + projector)", "batch": 1,
                      "encode_ms": round(dt * 1e3, 3), "tokens": 256}), flush=True)


if __name__ == "__main__":
    main()
