#!/usr/bin/env python
"""Headline benchmark: CLIP ViT-L/14 image embedding throughput (whole node).

One step = one serving batch per GPU: host-pinned decoded uint8 images (256x256
RGB, synthetic) -> H2D -> fused resize/normalise/patchify kernel -> ViT-L/14
image tower (bf16, random-init weights of the real architecture: 24 layers,
width 1024, 16 heads, patch 14, 224x224) -> fp32 L2-normalised 768-d
embeddings -> RCCL all-gather of every rank's embeddings (the DP result
gather).  Weak scaling: the per-GPU batch is fixed, so the global batch grows
with N.  JPEG decode is not in the headline timed region.  After it, two side windows
run by default: a >= 30 s steady-state window of the same step (``--seconds``,
``steady_state``) and two end-to-end windows that include JPEG decode (``--include-decode``):
``e2e_with_jpeg_decode`` = the framework's device JPEG path (host entropy decode + one batched GPU
IDCT/colour launch, utils/jpeg.py) and ``e2e_with_pillow_decode`` = Pillow on the CPU pool; then
the text tower (``texts_per_s``).

Launch: ``python bench.py --gpus 1`` or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lumen_amd.models.clip import CLIPModel, PRESETS  # noqa: E402
from lumen_amd.parallel import Communicator, destroy, init_distributed  # noqa: E402

METRIC = "CLIP ViT-L/14 images/sec (whole node)"


def _decode_window(model, B, side, dev, world, steps, g):
    """End-to-end side metric: B JPEG files per step decoded on the CPU decode pool into a
    pinned staging buffer (while the previous batch runs on the GPU), H2D, tower."""
    from lumen_amd.utils.image import decode_many, encode_jpeg

    rng = torch.randint(0, 256, (16, side, side, 3), generator=g, dtype=torch.uint8).numpy()
    jpegs = [encode_jpeg(rng[i % 16]) for i in range(B)]
    pinned = [torch.empty((B, side, side, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]
    dbuf = torch.empty((B, side, side, 3), dtype=torch.uint8, device=dev)
    done = [None, None]

    def run(i):
        arrs = decode_many(jpegs)          # overlaps the previous batch's tower on the GPU
        if done[i % 2] is not None:
            done[i % 2].synchronize()      # its H2D from this staging buffer has finished
        hb = pinned[i % 2]
        for k, a in enumerate(arrs):
            hb[k].copy_(torch.from_numpy(a))
        dbuf.copy_(hb, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        done[i % 2] = ev
        return model.encode_image_uint8(dbuf)

    run(0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        run(i)
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return {"images_per_s": round(world * B * steps / float(el.item()), 2), "steps": steps,
            "jpeg": f"{side}x{side} q90", "decode": "CPU thread pool (Pillow/libjpeg-turbo), draft off"}


def _device_decode_window(model, B, side, dev, world, steps, g):
    """End-to-end side metric, device JPEG path (utils/jpeg.py decode_batch_to_device): per step the
    batch's entropy decode on the host decode pool (one image per thread), one pinned H2D of the
    coefficients, ONE IDCT + ONE colour launch for the whole batch, then the tower's preprocessing
    reads the decoded pixels in place.  Host decode of step i overlaps the tower of step i - 1."""
    from lumen_amd.utils.image import encode_jpeg
    from lumen_amd.utils.jpeg import decode_batch_to_device

    rng = torch.randint(0, 256, (16, side, side, 3), generator=g, dtype=torch.uint8).numpy()
    jpegs = [encode_jpeg(rng[i % 16]) for i in range(B)]

    def run():
        flat, _offs, shapes, errs = decode_batch_to_device(jpegs, dev)
        assert not errs
        return model.encode_image_uint8(shapes, src=flat)

    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return {"images_per_s": round(world * B * steps / float(el.item()), 2), "steps": steps,
            "jpeg": f"{side}x{side} q90", "decode": "device JPEG (host entropy decode pool + batched GPU IDCT)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="images per GPU per step")
    ap.add_argument("--model", default="ViT-L-14")
    ap.add_argument("--src-size", type=int, default=256, help="synthetic decoded image side")
    ap.add_argument("--graph", action="store_true", help="capture the step in a HIP graph")
    ap.add_argument("--text-steps", type=int, default=None,
                    help="text-tower steps timed separately for the texts/s side metric (default = --steps; 0 = skip)")
    ap.add_argument("--seconds", type=float, default=30.0,
                    help="after the K-step window, run a steady-state window of at least this many seconds "
                         "(BASELINE.md asks >= 30 s) and report it as a side metric (0 = skip)")
    ap.add_argument("--include-decode", action=argparse.BooleanOptionalAction, default=True,
                    help="side metric: end-to-end images/s with JPEG decode (CPU thread pool, libjpeg-turbo) "
                         "+ pinned staging + H2D + tower, timed after the headline window (--no-include-decode "
                         "skips it)")
    args = ap.parse_args()

    local = int(os.environ.get("LOCAL_RANK", "0"))
    st = init_distributed(tp_size=1, device=torch.device("cuda", local))   # one process per GPU, RCCL
    world, rank, dev = st.world, st.rank, st.device
    comm = Communicator(st.dp_group, dev, ipc=False)                      # DP result gather over RCCL

    cfg = PRESETS[args.model]
    text_steps = args.steps if args.text_steps is None else args.text_steps
    model = CLIPModel.random(cfg, seed=0, device=dev, with_text=text_steps > 0)
    B = args.batch
    g = torch.Generator().manual_seed(1234 + rank)
    host = torch.randint(0, 256, (B, args.src_size, args.src_size, 3), generator=g, dtype=torch.uint8).pin_memory()
    gathered = torch.empty((world * B, cfg.embed_dim), device=dev, dtype=torch.float32)
    # double-buffered upload on a copy stream: batch i+1 is transferred over PCIe
    # while batch i runs the tower (every step still moves its full batch H2D)
    dimg = [torch.empty_like(host, device=dev) for _ in range(2)]
    copy_stream = torch.cuda.Stream(dev)
    copied = [torch.cuda.Event() for _ in range(2)]
    consumed = [torch.cuda.Event() for _ in range(2)]
    comp = torch.cuda.current_stream(dev)
    counter = {"i": 0}

    def upload(j):
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(consumed[j % 2])
            dimg[j % 2].copy_(host, non_blocking=True)
            copied[j % 2].record(copy_stream)

    for e in consumed:
        e.record(comp)
    upload(0)

    def step():
        i = counter["i"]
        counter["i"] += 1
        upload(i + 1)
        comp.wait_event(copied[i % 2])
        emb = model.encode_image_uint8(dimg[i % 2])
        consumed[i % 2].record(comp)
        comm.all_gather_into(gathered, emb)
        return emb

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ok = bool(torch.isfinite(gathered).all().item())
    steady = None
    if args.seconds > 0:
        # steady-state window: whole steps until >= --seconds of wall clock (BASELINE.md rule)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        n_ss, t_ss0 = 0, time.perf_counter()
        while True:
            for _ in range(5):
                step()
            n_ss += 5
            torch.cuda.synchronize()
            if time.perf_counter() - t_ss0 >= args.seconds:
                break
        el = torch.tensor([time.perf_counter() - t_ss0], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        steady = {"seconds": round(float(el.item()), 2), "steps": n_ss,
                  "images_per_s": round(world * B * n_ss / float(el.item()), 2)}
    e2e = e2e_dev = None
    if args.include_decode:
        e2e = _decode_window(model, B, args.src_size, dev, world, max(3, min(args.steps, 10)), g)
        try:
            e2e_dev = _device_decode_window(model, B, args.src_size, dev, world, max(3, min(args.steps, 10)), g)
        except Exception as exc:       # side metric only: never fail the headline line over it
            e2e_dev = {"error": f"{type(exc).__name__}: {exc}"[:200]}
    # side metric (BASELINE config 2 "image + text embed"): text tower on a batch of B
    # 77-token prompts, timed separately AFTER the headline window (never inside it)
    text_per_s = None
    if text_steps > 0:
        ids = torch.randint(1, cfg.text.vocab_size - 1, (B, cfg.text.context_length), generator=g).to(dev)
        ids[:, -1] = cfg.text.vocab_size - 1          # EOT = max id (argmax pooling)
        for _ in range(2):
            model.encode_text_ids(ids)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(text_steps):
            temb = model.encode_text_ids(ids)
        torch.cuda.synchronize()
        tt = torch.tensor([time.perf_counter() - t1], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        text_per_s = world * B * text_steps / float(tt.item())
        ok = ok and bool(torch.isfinite(temb).all().item())
    if rank == 0:
        ms = dt / args.steps * 1e3
        total = world * B * args.steps / dt
        v = cfg.vision
        S = (v.image_size // v.patch_size) ** 2 + 1
        W = v.width
        gemm_flops = 2 * S * (v.layers * (4 * W * W + 2 * W * int(W * v.mlp_ratio))) + 2 * (S - 1) * W * 3 * v.patch_size ** 2
        attn_flops = v.layers * 4 * S * S * W
        flops_img = gemm_flops + attn_flops
        out = {
            "metric": METRIC,
            "value": round(total, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random uint8 256x256 RGB images, random-init weights)",
            "config": {
                "model": f"CLIP {args.model} image tower",
                "global_batch": world * B,
                "seq_len": S,
                "parallelism": f"dp{world}",
                "image_size": v.image_size,
                "per_gpu_batch": B,
                "includes": "H2D (double-buffered, overlapped) + resize/normalise/patchify + tower + L2 + all-gather",
            },
            "tflops_per_gpu": round(flops_img * total / world / 1e12, 1),
            "texts_per_s": round(text_per_s, 1) if text_per_s else None,
            "text_config": {"context_length": cfg.text.context_length, "batch_per_gpu": B,
                            "timed": "separately, after the image window"} if text_per_s else None,
            "steady_state": steady,
            "e2e_with_jpeg_decode": e2e_dev,
            "e2e_with_pillow_decode": e2e,
            "finite": ok,
        }
        print(json.dumps(out), flush=True)
    destroy()


if __name__ == "__main__":
    main()
