"""ViT-L/14 b512 patch-embedding GEMM (M 131,072 patches x N 1,024 x K 640, positional-table epilogue with the
token-row remap) under each candidate tile code of ops.linear, HIP-event timed, output checked against tile -1."""
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
    B, P, S, W, K = 512, 256, 257, 1024, 640
    patches = (torch.randn(B * P, K, device=dev) * 0.5).bfloat16()
    w = (torch.randn(W, K, device=dev) * K ** -0.5).bfloat16()
    pos = (torch.randn(S, W, device=dev) * 0.02).bfloat16()
    outs = {}
    res = {}
    for tile in (-1, 609, 709, 209, 245, 1609, 20000, 20003, 1, 9, 1009):
        x = torch.zeros(B * S, W, device=dev, dtype=torch.bfloat16)

        def run():
            ops.linear(patches, w, table=pos, table_period=P, table_offset=1, out=x, out_group=P,
                       out_group_stride=S, out_row_offset=1, tile=tile)
        try:
            run()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 - a code this shape cannot take
            res[str(tile)] = f"error: {str(e)[:60]}"
            continue
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) / 20)
        outs[tile] = x.clone()
        same = bool(torch.equal(outs[tile], outs[-1])) if -1 in outs else None
        res[str(tile)] = {"ms": round(best, 4), "same_as_auto": same,
                          "max_diff": float((outs[tile].float() - outs[-1].float()).abs().max()) if -1 in outs else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
