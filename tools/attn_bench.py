"""Microbenchmark: lumen fused attention vs torch SDPA on the ViT-L/14 shape (B=512, S=257, H=16, D=64)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from lumen_amd import ops

for (B, S, H, D, causal) in [(512, 257, 16, 64, False), (512, 77, 12, 64, True), (8, 1024, 28, 128, True)]:
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    out = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    def run_l():
        ops.attention(q, k, v, causal=causal, out=out)
    qt, kt, vt = (t.transpose(1, 2).contiguous() for t in (q, k, v))
    def run_t():
        F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
    r = {"B": B, "S": S, "H": H, "D": D, "causal": causal}
    flops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    for name, fn in (("lumen", run_l), ("sdpa", run_t)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        ms = 1e9
        for _ in range(3):     # best of 3 windows of 30 launches (clock / warm-up noise)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(30):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = min(ms, s.elapsed_time(e) / 30)
        r[name + "_ms"] = round(ms, 3)
        r[name + "_tflops"] = round(flops / ms / 1e9, 1)
    # csrc/tuning.h A/B of the K/V-resident kernel: TUNE_ATTN_CLEAN_CHUNKS (1) mask-free clean chunks
    # (a hashed rotation of the query-block walk, switch 2, lost: profiles/r6_attn_rotate_ab_v1.txt)
    for flag, name in ((1, "clean_chunks"),):
        if not (S in (197, 257, 577) and not causal):
            continue
        hip = ops.hip_ops()
        base = hip.set_tuning(flag, 1)
        for val in (0, 1, 0, 1, 0, 1):
            hip.set_tuning(flag, val)
            for _ in range(5):
                run_l()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(30):
                run_l()
            e.record()
            torch.cuda.synchronize()
            key = name + ("_on" if val else "_off") + "_ms"
            r[key] = min(r.get(key, 1e9), round(s.elapsed_time(e) / 30, 4))
        hip.set_tuning(flag, base)
    ref = F.scaled_dot_product_attention(qt[:2].float(), kt[:2].float(), vt[:2].float(), is_causal=causal).transpose(1, 2)
    run_l()
    r["rel_err"] = float(((out[:2].float() - ref).norm() / ref.norm()).item())
    print(json.dumps(r), flush=True)
