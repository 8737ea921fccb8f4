"""Mid-M GEMMs in the regime a layer stack runs them: weights cold (HBM), activations fresh.

The VLM time-to-first-token runs two layer stacks at a few hundred rows: the LLaVA vision
tower (ViT-L/14-336, 577 tokens, bf16) and the Llama-3-8B W8A8 prefill (624 tokens, fp8).
Benchmarked in a loop over ONE weight matrix, these GEMMs read their weights from the
Infinity Cache and look twice as fast as they run in the model (profiles/r4_ttft_*), so
here every launch of a timed loop reads a different weight matrix (enough of them that the
set exceeds the 256 MiB Infinity Cache) and a different activation matrix.

    python tools/cold_gemm_bench.py --what vit --variants -1,20002,20013
    python tools/cold_gemm_bench.py --what prefill --variants 0,1,2,3,6 --splits -1,1,2
    python tools/cold_gemm_bench.py --what mx --epi full      # the fused MX chain's GEMMs (ops.linear_mx)

Variant codes: bf16 (--what vit) are ops.linear tile codes (-1 auto; 20000 + v: the LDS-DMA
pipeline of csrc/gemm_f8.hip, v = 2 / 3 / 5 r2 shapes, 10 + c: launch_variant code c);
fp8 (--what prefill) are launch_variant codes (0 = auto).
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

VIT = [("qkv", 3072, 1024, None, False), ("out", 1024, 1024, None, True), ("fc1", 4096, 1024, "quick_gelu", False),
       ("fc2", 1024, 4096, None, True)]
PREFILL = [("qkv", 6144, 4096, False, False), ("o", 4096, 4096, False, True), ("gu", 28672, 4096, True, False),
           ("down", 4096, 14336, False, True)]


def timed(fn, L, reps=3):
    fn(0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for l in range(L):
            fn(l)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / L * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["vit", "prefill", "mx", "mxvit"], default="vit")
    ap.add_argument("--epi", choices=["full", "plain"], default="full",
                    help="mx: the chain's epilogues (rstd, MX outputs, sums of squares) or a plain store")
    ap.add_argument("--M", type=int, default=0)
    ap.add_argument("--variants", default="")
    ap.add_argument("--splits", default="-1")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default all)")
    ap.add_argument("--cold-mb", type=int, default=768, help="weight bytes per timed loop")
    a = ap.parse_args()
    load_hip(required=True)
    dev = "cuda"
    torch.manual_seed(0)
    vit = a.what == "vit"
    mx = a.what in ("mx", "mxvit")
    mxvit = a.what == "mxvit"
    M = a.M or (577 if vit or mxvit else 624)
    variants = [int(v) for v in (a.variants or ("-1,20002,20003,20005" if vit else "0,1,2")).split(",")]
    splits = [int(s) for s in a.splits.split(",")]
    shapes = VIT if vit else PREFILL
    if mxvit:   # the W8A8 vision chain's GEMMs (clip.run_blocks_mx): act -> MX output for fc1
        shapes = [("qkv", 3072, 1024, False, False), ("out", 1024, 1024, False, True), ("fc1", 4096, 1024, False, False),
                  ("fc2", 1024, 4096, False, True)]
    if a.shapes:
        shapes = [s for s in shapes if s[0] in a.shapes.split(",")]
    res = {"what": a.what, "M": M}
    best_total = 0.0
    for name, N, K, x4, resid in shapes:
        wbytes = N * K * (2 if vit else 1)
        L = max(4, -(-a.cold_mb * (1 << 20) // wbytes))
        if vit:
            ws = [(torch.randn(N, K, device=dev) * K ** -0.5).bfloat16() for _ in range(L)]
            xs = [torch.randn(M, K, device=dev).bfloat16() for _ in range(L)]
            b = torch.randn(N, device=dev).bfloat16()
        else:
            ws, sws = [], []
            for _ in range(L):
                w8, sw = ops.quantize_fp8_rows((torch.randn(N, K, device=dev) * K ** -0.5).bfloat16())
                ws.append(w8)
                sws.append(sw)
            xs, sxs = [], []
            for _ in range(L):
                if mx:
                    x8, sx = ops.quant_rows_mx(torch.randn(M, K, device=dev).bfloat16())
                else:
                    x8, sx = ops.quant_rows_fp8(torch.randn(M, K, device=dev).bfloat16())
                xs.append(x8)
                sxs.append(sx)
            NO_ = N // 2 if x4 else N
            q8 = torch.empty(M, NO_, device=dev, dtype=torch.float8_e4m3fn)
            qs = torch.empty(NO_ // 128, M, 4, device=dev, dtype=torch.uint8)
            ssq_in = torch.rand(M, K // 128, device=dev) + 1.0
            ssq_out = torch.empty(M, N // 128, device=dev)
        r = torch.randn(M, N, device=dev).bfloat16() if resid else None
        NO = N // 2 if (not vit and x4) else N
        out = torch.empty(M, NO, device=dev, dtype=torch.bfloat16)
        best = None
        for v in variants:
            wv = ws
            for sp in splits:
                if vit:
                    f = lambda l, v=v: ops.linear(xs[l], ws[l], b, act=x4, residual=r, out=out, tile=v)  # noqa: E731
                    fw = lambda l, v=v: ops.linear(xs[0], ws[0], b, act=x4, residual=r, out=out, tile=v)  # noqa: E731
                    key = f"{name}_t{v}"
                elif mx:
                    full = a.epi == "full"
                    kw = dict(residual=r, glu=x4, variant=v)
                    if full:
                        kw.update(q_out=(q8, qs) if (x4 or resid) else None, ssq_out=ssq_out if resid else None,
                                  ssq_in=ssq_in if not resid else None, norm_eps=1e-5, write_out=not x4)
                    f = lambda l, v=v, kw=kw: ops.linear_mx(xs[l], sxs[l], ws[l], sws[l], out=out, **kw)  # noqa: E731
                    fw = lambda l, v=v, kw=kw: ops.linear_mx(xs[0], sxs[0], ws[0], sws[0], out=out, **kw)  # noqa: E731
                    key = f"{name}_mx{a.epi}_v{v}"
                else:
                    f = lambda l, v=v, sp=sp, wv=wv: ops.linear_f8(xs[l], sxs[l], wv[l], sws[l], residual=r,  # noqa: E731
                                                                   out=out, glu=x4, splits=sp, variant=v)
                    fw = lambda l, v=v, sp=sp, wv=wv: ops.linear_f8(xs[0], sxs[0], wv[0], sws[0], residual=r,  # noqa: E731
                                                                    out=out, glu=x4, splits=sp, variant=v)
                    key = f"{name}_v{v}_s{sp}"
                try:
                    cold = timed(f, L)
                    warm = timed(fw, L)
                except RuntimeError as e:   # an unsupported combination: record and go on
                    res[key] = str(e)[:80]
                    continue
                tf = 2 * M * N * K / cold / 1e6
                res[key] = {"cold_us": round(cold, 2), "warm_us": round(warm, 2), "cold_tflops": round(tf, 1)}
                if best is None or cold < best[1]:
                    best = (key, cold)
                print(key, res[key], flush=True)
        if best:
            res[f"{name}_best"] = best[0]
            best_total += best[1]
    res["layer_best_us"] = round(best_total, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
