"""Where does a GEMM's time go: per-K-step slope and fixed per-launch cost, with operands from
memory as in the model ("real") or from a small, cache-resident footprint ("resident": rows
viewed with a 128-byte row stride, so every K-step still reads distinct bytes per row but the
whole operand is a few hundred KiB to a few MiB).

If the resident slope is much lower than the real one, the main loop waits on memory (latency /
intake); if they are equal, the kernel's own instruction stream and synchronisation set the pace.

    python tools/gemm_floor_probe.py --what f8   # W8A8 prefill shapes (M = 624)
    python tools/gemm_floor_probe.py --what bf16 # ViT-L/14 b512 shapes (M = 131584)
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402


def timed(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps * 1e3)
    return statistics.median(ts)


def resident(rows, K, dtype, dev, row_bytes=128):
    """[rows, K] view whose row r starts row_bytes * r into a small buffer."""
    es = torch.empty((), dtype=dtype).element_size()
    st = row_bytes // es
    buf = torch.empty(rows * st + K, dtype=torch.float32 if dtype == torch.float8_e4m3fn else dtype, device=dev)
    if dtype == torch.float8_e4m3fn:
        buf = (torch.randn(rows * st + K, device=dev) * 0.5).to(dtype)
    else:
        buf.normal_()
    return torch.as_strided(buf, (rows, K), (st, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["f8", "bf16"], default="f8")
    ap.add_argument("--variants", default="")
    ap.add_argument("--Ks", default="")
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--M", type=int, default=0)
    a = ap.parse_args()
    load_hip(required=True)
    dev = "cuda"
    torch.manual_seed(0)
    out = {"what": a.what}
    if a.what == "f8":
        M, N = a.M or 624, a.N or 4096
        Ks = [int(k) for k in (a.Ks or "1024,4096,16384").split(",")]
        variants = [int(v) for v in (a.variants or "2,1,3,12,13").split(",")]
        for K in Ks:
            sw = torch.rand(N, device=dev) + 0.5
            sx = torch.rand(M, device=dev) + 0.5
            real_w = (torch.randn(N, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
            real_x = (torch.randn(M, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
            res_w, res_x = resident(N, K, torch.float8_e4m3fn, dev), resident(M, K, torch.float8_e4m3fn, dev)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for v in variants:
                for tag, x, w in (("real", real_x, real_w), ("resident", res_x, res_w)):
                    try:
                        t = timed(lambda: ops.linear_f8(x, sx, w, sw, out=y, splits=1, variant=v))
                    except RuntimeError as e:
                        out[f"K{K}_v{v}_{tag}"] = str(e)[:60]
                        continue
                    out[f"K{K}_v{v}_{tag}"] = {"us": round(t, 2), "tflops": round(2 * M * N * K / t / 1e6, 1),
                                               "us_per_kstep": round(t / (K // 128), 4)}
                    print(f"K{K}_v{v}_{tag}", out[f"K{K}_v{v}_{tag}"], flush=True)
    else:
        M, N = a.M or 131584, a.N or 3072
        Ks = [int(k) for k in (a.Ks or "1024,2048,4096").split(",")]
        variants = [int(v) for v in (a.variants or "-1").split(",")]
        for K in Ks:
            b = torch.randn(N, device=dev).bfloat16()
            real_w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
            real_x = torch.randn(M, K, device=dev).bfloat16()
            res_w, res_x = resident(N, K, torch.bfloat16, dev), resident(M, K, torch.bfloat16, dev)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for v in variants:
                for tag, x, w in (("real", real_x, real_w), ("resident", res_x, res_w)):
                    try:
                        t = timed(lambda: ops.linear(x, w, b, out=y, tile=v), reps=5)
                    except RuntimeError as e:
                        out[f"K{K}_t{v}_{tag}"] = str(e)[:60]
                        continue
                    out[f"K{K}_t{v}_{tag}"] = {"us": round(t, 2), "tflops": round(2 * M * N * K / t / 1e6, 1)}
                    print(f"K{K}_t{v}_{tag}", out[f"K{K}_t{v}_{tag}"], flush=True)
            try:
                t = timed(lambda: torch.nn.functional.linear(real_x, real_w, b), reps=5)
                out[f"K{K}_hipblaslt"] = {"us": round(t, 2), "tflops": round(2 * M * N * K / t / 1e6, 1)}
                print(f"K{K}_hipblaslt", out[f"K{K}_hipblaslt"], flush=True)
            except RuntimeError as e:
                out[f"K{K}_hipblaslt"] = str(e)[:60]
            del real_x, real_w
    print(json.dumps(out))


if __name__ == "__main__":
    main()
