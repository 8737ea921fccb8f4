"""A/B of a CLIP image-tower code path in ONE process (interleaved rounds, cdna_hip_programming.md
§5.4 rule 24): the bench.py step (uint8 256x256 batch -> prep -> ViT tower -> L2) timed with a
module flag of lumen_amd.models.clip off and on.

    python tools/tower_ab.py --flag _LN_FOLD [--model ViT-L-14] [--batch 512] [--rounds 5] [--steps 10]
    python tools/tower_ab.py --tuning ln_multi_row        # a kernel-variant switch (csrc/tuning.h) instead
    python tools/tower_ab.py --flag ops._PREP_BAND_LDS --values 0,54272   # a lumen_amd.ops module flag
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lumen_amd.models.clip as clip_mod  # noqa: E402
from lumen_amd._native import load_hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flag", default="_LN_FOLD")
    ap.add_argument("--model", default="ViT-L-14")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--values", default="", help="the two arms of an int flag, e.g. 2,3 (default off / on)")
    ap.add_argument("--tuning", default=None, help="csrc/tuning.h switch: ln_multi_row | attn_clean_chunks")
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    m = clip_mod.CLIPModel.random(clip_mod.PRESETS[args.model], seed=0, device=dev, with_text=False)
    imgs = torch.randint(0, 256, (args.batch, 256, 256, 3), dtype=torch.uint8, device=dev)
    tune = {"ln_multi_row": 0, "attn_clean_chunks": 1}.get(args.tuning) if args.tuning else None
    ops = load_hip(required=True) if tune is not None else None
    if tune is not None:
        from lumen_amd._native import hip_ops

        def setter(v):
            hip_ops().set_tuning(tune, int(v))
        base = True
        args.flag = f"tuning:{args.tuning}"
    else:
        from lumen_amd import ops as ops_mod
        mod, name = (ops_mod, args.flag[4:]) if args.flag.startswith("ops.") else (clip_mod, args.flag)
        base = getattr(mod, name)

        def setter(v):
            setattr(mod, name, v)
    arms = {"off": False if isinstance(base, bool) else 0, "on": True if isinstance(base, bool) else 1}
    if args.values:       # two explicit values of an int flag (e.g. --flag _VIT_MICRO --values 2,3)
        a, b = (int(v) for v in args.values.split(","))
        arms = {f"v{a}": a, f"v{b}": b}
    res = {k: [] for k in arms}
    outs = {}
    for r in range(args.rounds + 1):
        for name, val in arms.items():
            setter(val)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                e = m.encode_image_uint8(imgs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r > 0:                                   # round 0 = warm-up of both arms
                res[name].append(args.batch * args.steps / dt)
            outs[name] = e.float().cpu()
    setter(base)
    o1, o2 = (outs[k] for k in arms)
    cos = float((o1 * o2).sum(-1).min())
    print(json.dumps({"flag": args.flag, "model": args.model, "batch": args.batch,
                      "images_per_s": {k: [round(x, 1) for x in v] for k, v in res.items()},
                      "median": {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()},
                      "min_cos_off_vs_on": round(cos, 6)}))


if __name__ == "__main__":
    main()
