"""Prefill-shaped GEMMs of Llama-3-8B (M = 624 prompt tokens) on every available path:
lumen bf16 MFMA, lumen fp8-weight MFMA, hipBLASLt bf16 (torch.matmul) and hipBLASLt fp8
x fp8 (torch._scaled_mm, per-token activation scales x per-channel weight scales)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lumen_amd import ops  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, it=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def main():
    load_hip(required=True)
    dev = torch.device("cuda")
    M = int(os.environ.get("M", "624"))
    res = {"M": M}
    for name, (N, K) in SHAPES.items():
        x = torch.randn(M, K, device=dev).bfloat16()
        wf = torch.randn(N, K, device=dev) * K ** -0.5
        wb = wf.bfloat16()
        w8, s = ops.quantize_fp8_rows(wf)
        fl = 2 * M * N * K
        r = {}
        r["lumen_bf16"] = timeit(lambda: ops.linear(x, wb))
        r["lumen_w8"] = timeit(lambda: ops.linear(x, w8, w_scale=s))
        r["blas_bf16"] = timeit(lambda: torch.matmul(x, wb.t()))
        try:
            def sm():
                amax = x.abs().amax(dim=1, keepdim=True).float().clamp_min(1e-6)
                sa = amax / 448.0
                x8 = (x.float() / sa).to(torch.float8_e4m3fn)
                return torch._scaled_mm(x8, w8.t(), scale_a=sa, scale_b=s.view(1, -1), out_dtype=torch.bfloat16)
            r["blas_fp8_rowwise_incl_quant"] = timeit(sm)
            amax = x.abs().amax(dim=1, keepdim=True).float().clamp_min(1e-6)
            sa = amax / 448.0
            x8 = (x.float() / sa).to(torch.float8_e4m3fn)
            r["blas_fp8_rowwise_gemm_only"] = timeit(
                lambda: torch._scaled_mm(x8, w8.t(), scale_a=sa, scale_b=s.view(1, -1), out_dtype=torch.bfloat16))
            ref = ops.linear(x, w8, w_scale=s).float()
            got = sm().float()
            r["fp8_rowwise_rel_err"] = ((got - ref).norm() / ref.norm()).item()
        except Exception as e:  # noqa: BLE001
            r["blas_fp8_error"] = str(e)[:200]
        for k in list(r):
            if isinstance(r[k], float) and not k.endswith("err"):
                r[k + "_TF"] = round(fl / r[k] / 1e6, 1)
                r[k] = round(r[k], 1)
        res[name] = r
        print(json.dumps({name: r}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
