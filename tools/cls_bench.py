"""Microbenchmark: the OCR recogniser classifier fused with the CTC arg-max (csrc/postproc.hip
cls_argmax_kernel via hip_ops().cls_ctc) on the OCR bench's two recogniser chunks per batch
(256 crops x 96 steps, 64 crops x 108 steps; K 128, 6625 classes padded to 6640).

    python tools/cls_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lumen_amd._native import hip_ops, load_hip


def main():
    load_hip(required=True)
    hip = hip_ops()
    dev = torch.device("cuda")
    K, N, C = 128, 6640, 6625
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(N, K, generator=g) * 0.3).bfloat16().to(dev)
    b = (torch.randn(N, generator=g) * 0.5).to(dev)
    out = []
    for B, T in ((256, 96), (64, 108)):
        M = B * T
        h = torch.randn(M, K, generator=g).bfloat16().to(dev)
        i1 = torch.empty(M, dtype=torch.int32, device=dev)
        c1 = torch.empty(M, dtype=torch.float32, device=dev)
        ids = torch.empty((B, T), dtype=torch.int32, device=dev)
        ln = torch.empty((B,), dtype=torch.int32, device=dev)
        cf = torch.empty((B,), dtype=torch.float32, device=dev)

        def run():
            hip.cls_ctc(h, w, b, C, B, T, 0, None, i1, c1, ids, ln, cf)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        out.append({"rows": M, "us": round(us, 1), "tflops": round(2 * M * N * K / us / 1e6, 1),
                    "glogits_per_s": round(M * N / us / 1e3, 1)})
    print(json.dumps({"kernel": "cls_ctc (classifier + CTC arg-max fused)", "K": K, "classes": C, "runs": out}))


if __name__ == "__main__":
    main()
