"""GPU entropy decode timing breakdown on the bench images (run under rocprofv3 --kernel-trace
--stats for the per-kernel times): host prepare (parse + unstuff), then the full single-image
device decode, N times each.

    python tools/jpeg_huff_prof.py [--n 20] [--kind photo]
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
from lumen_amd.utils.image import encode_jpeg  # noqa: E402
from tools.face_ocr_bench import synth_image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--kind", default="photo")
    ap.add_argument("--hw", default="768,1024")
    ap.add_argument("--lanes", default="256,512,1024,2048,4096")
    a = ap.parse_args()
    load_hip(required=True)
    h, w = map(int, a.hw.split(","))
    data = encode_jpeg(synth_image(np.random.default_rng(0), h, w, a.kind))
    ji = J.info(data)
    blob = np.zeros(J.blob_capacity([data], [ji]), np.uint8)
    qt = np.zeros((1, 192), np.uint16)
    prep = []
    for _ in range(a.n):
        t = time.perf_counter()
        J.prepare_blob([data], [ji], blob, qt)
        prep.append((time.perf_counter() - t) * 1e3)
    res = {"kind": a.kind, "bytes": len(data), "prepare_ms": round(statistics.median(prep), 4)}
    for lanes in map(int, a.lanes.split(",")):
        full, rounds = [], 0
        for _ in range(a.n + 2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            img = J.decode_to_device_gpu(data, "cuda", ji, lanes=lanes)
            torch.cuda.synchronize()
            full.append((time.perf_counter() - t) * 1e3)
            rounds = int(img.jpeg_err[1])
            assert int(img.jpeg_err[0]) == 0
        res[f"lanes{lanes}"] = {"device_decode_ms": round(statistics.median(full[2:]), 4), "rounds": rounds}
    # phase timing of one decode per lane count (wall-clock stamps of workgroup 0, 100 MHz)
    from lumen_amd.ops import hip_ops
    for lanes in map(int, a.lanes.split(",")):
        hb = torch.zeros(J.blob_capacity([data], [ji]), dtype=torch.uint8).pin_memory()
        used, ok = J.prepare_blob([data], [ji], hb.numpy(), np.zeros((1, 192), np.uint16), lanes=lanes)
        coef = torch.empty(ji.coef_count, dtype=torch.int16, device="cuda")
        err = torch.zeros(2, dtype=torch.int32, device="cuda")
        ticks = torch.zeros(128, dtype=torch.int64, device="cuda")
        hip_ops().jpeg_huff_decode(hb[:used].cuda(), hb[:used], 1, coef, err, ticks)
        t = ticks.cpu().numpy()
        t0 = t[0]
        us = lambda v: round((int(v) - int(t0)) / 100.0, 1) if v else None   # noqa: E731
        rounds = int(err[1])
        res[f"phases_lanes{lanes}"] = {"staged": us(t[1]), "round0": us(t[2]), "round0_bar": us(t[3]),
                                       "rounds": [us(t[3 + r]) for r in range(1, min(rounds, 100))],
                                       "scan": us(t[120]), "end": us(t[121])}
    # batches of 32 / 128 (lanes per image from the co-residency rule)
    for nb in (32, 128):
        ts = []
        for _ in range(max(3, a.n // 4)):
            torch.cuda.synchronize()
            t = time.perf_counter()
            J.decode_batch_to_device([data] * nb, "cuda")
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        res[f"batch{nb}_ms"] = round(statistics.median(ts[1:]), 3)
        res[f"batch{nb}_img_s"] = round(nb * 1e3 / statistics.median(ts[1:]), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
