"""Marginal cost of the LayerNorm row-statistics passes inside the ViT-L/14 b512 tower step.

Arm "x2" runs every ops.ln_row_stats call twice (the second pass recomputes the same statistics),
arm "x1" is the production step; interleaved rounds in one process.  The difference bounds what
fusing the statistics into the residual GEMM epilogues could save.

    python tools/probes/ln_stats_cost.py [--op ln_row_stats | attention] [--rounds 5] [--steps 10]
    python tools/probes/ln_stats_cost.py --op linear_lnf --drop-act     # cost of the fc1 activation epilogue
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lumen_amd.models.clip as clip_mod  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--op", default="ln_row_stats", help="lumen_amd.ops function to double (ln_row_stats | attention)")
    ap.add_argument("--drop-act", action="store_true",
                    help="arm x2 runs the op (linear_lnf) WITHOUT its activation instead: the epilogue's activation cost")
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    m = clip_mod.CLIPModel.random(clip_mod.PRESETS["ViT-L-14"], seed=0, device=dev, with_text=False)
    imgs = torch.randint(0, 256, (512, 256, 256, 3), dtype=torch.uint8, device=dev)
    orig = getattr(clip_mod.ops, args.op)
    state = {"n": 1}

    def stats(*a, **k):
        if args.drop_act:
            if state["n"] == 2:
                k = dict(k, act=None)
            return orig(*a, **k)
        for _ in range(state["n"] - 1):
            orig(*a, **k)
        return orig(*a, **k)

    setattr(clip_mod.ops, args.op, stats)
    res = {"x1": [], "x2": []}
    try:
        for r in range(args.rounds + 1):
            for name, n in (("x1", 1), ("x2", 2)):
                state["n"] = n
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    m.encode_image_uint8(imgs)
                torch.cuda.synchronize()
                if r > 0:
                    res[name].append(512 * args.steps / (time.perf_counter() - t0))
    finally:
        setattr(clip_mod.ops, args.op, orig)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    ms = {k: 512 / v * 1e3 for k, v in med.items()}
    print(json.dumps({"op": args.op, "drop_act": args.drop_act, "images_per_s": {k: [round(x, 1) for x in v] for k, v in res.items()},
                      "median": {k: round(v, 1) for k, v in med.items()},
                      "ms_per_step": {k: round(v, 3) for k, v in ms.items()},
                      "extra_pass_cost_ms_per_step": round(ms["x2"] - ms["x1"], 3)}))


if __name__ == "__main__":
    main()
