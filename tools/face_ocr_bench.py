"""Face and OCR pipeline throughput on one MI355X (synthetic images, random-init weights).

face: JPEG decode -> letterbox 640 -> SCRFD-10G-shaped detector -> decode/NMS ->
      ArcFace IResNet-100 (antelopev2 geometry) on a fixed number of faces per image
      (random weights detect nothing meaningful, so the recogniser batch is fed a
      fixed F faces/image of 5-point alignments to exercise the full path).
ocr:  JPEG decode -> DBNet (limit 960) -> DB geometry -> SVTR recogniser on a fixed
      number of text crops per image.

usage: python tools/face_ocr_bench.py --what face --batch 32 --iters 10
       torchrun --nproc-per-node N tools/face_ocr_bench.py --what face --gpus N   (face SPMD DP:
       each rank detects + embeds its own batch, one RCCL all-gather of the packed
       bbox / confidence / landmarks / embedding rows per step; weak scaling, whole-job img/s)
       torchrun --nproc-per-node N tools/face_ocr_bench.py --what ocr --gpus N    (OCR SPMD DP:
       the same with the packed box / confidence / code-point rows, services/ocr/spmd.py)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lumen_amd._native import load_hip  # noqa: E402
from lumen_amd.ops import vision  # noqa: E402
from lumen_amd.utils.image import decode_many, encode_jpeg  # noqa: E402


def synth_image(rng, h, w, kind):
    """uint8 [h, w, 3]: 'noise' = uniform random pixels (incompressible: a ~0.8 MB q90 JPEG at 1280x720,
    the worst case for the host entropy decoder); 'photo' = smooth low-frequency colour fields +
    edges + mild sensor noise (~130 KB at 1280x720, like a camera photo)."""
    if kind == "noise":
        return rng.integers(0, 255, (h, w, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.zeros((h, w, 3), np.float32)
    for c in range(3):
        for _ in range(6):
            fy, fx = rng.uniform(0.5, 6, 2) / np.array([h, w])
            ph = rng.uniform(0, 2 * np.pi, 2)
            img[..., c] += rng.uniform(10, 40) * np.sin(2 * np.pi * fy * yy + ph[0]) * np.cos(2 * np.pi * fx * xx + ph[1])
    for _ in range(12):      # flat-coloured rectangles: edges
        y0, x0 = rng.integers(0, h - 40), rng.integers(0, w - 40)
        img[y0:y0 + rng.integers(20, h // 3), x0:x0 + rng.integers(20, w // 3)] += rng.uniform(-60, 60, 3)
    img += 128 + rng.normal(0, 3, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def bench_face(args):
    from lumen_amd.models.face import IRESNET_PRESETS, SCRFD, SCRFD_PRESETS, IResNet
    from lumen_amd.services.face.backend import DetParams, FaceDetection, FaceSpec, MI355XFaceBackend

    runner, world, rank = None, 1, 0
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from lumen_amd.parallel import Communicator, init_distributed
        from lumen_amd.services.face.spmd import SPMDFaceRunner

        local = int(os.environ.get("LOCAL_RANK", "0"))
        st = init_distributed(tp_size=1, device=torch.device("cuda", local))
        world, rank = st.world, st.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    det = SCRFD(SCRFD_PRESETS["10g"])
    det.random_init(torch.Generator().manual_seed(0))
    rec = IResNet(IRESNET_PRESETS[args.rec])
    rec.random_init(torch.Generator().manual_seed(1))
    be = MI355XFaceBackend.__new__(MI355XFaceBackend)
    be.det, be.rec, be.spec, be.device, be.dtype = det.to(dev).eval(), rec.to(dev).eval(), FaceSpec(), dev, torch.bfloat16
    be.template = vision.ARCFACE_DST
    be._pool, be._dp, be.align_mode = None, {}, "standard"
    if world > 1:
        runner = SPMDFaceRunner(be, Communicator(st.dp_group, dev, ipc=False), dev)
    rng = np.random.default_rng(rank)
    jpegs = [encode_jpeg(synth_image(rng, 720, 1280, args.image_kind)) for _ in range(args.batch)]
    lms = np.array([[500, 300], [580, 300], [540, 350], [510, 400], [570, 400]], np.float32)
    minv = np.stack([vision.invert_affine(vision.similarity_transform(lms + 3 * k)) for k in range(args.faces)])

    # the next batch's JPEGs decode on the host threads while this batch runs on the GPU
    # (what the serving path does with two batches in flight per GPU worker)
    from concurrent.futures import ThreadPoolExecutor

    ahead = ThreadPoolExecutor(max_workers=1)
    pre = decode_many(jpegs) if args.predecoded else None
    dec = (lambda: pre) if pre is not None else (lambda: decode_many(jpegs))  # noqa: E731

    def dec_up():    # decode + pinned staging + H2D (own stream) of the NEXT batch, off the main thread
        if pre is None and not args.pillow:
            # JPEG-inclusive: host entropy decode on the pool + one batched GPU reconstruction
            imgs, up = be.decode_device(jpegs)
            ev = torch.cuda.Event()
            ev.record()
            return imgs, (up[0], up[1], ev)
        imgs = dec()
        return imgs, be.upload_async(imgs)

    nxt = [ahead.submit(dec_up)]

    from lumen_amd.runtime.metrics import StageTimer, use_timer

    stages: dict = {}

    params = [DetParams(0.5, 0.4, 20, 2000)] * args.batch
    idx = [i for i in range(args.batch) for _ in range(args.faces)]
    minv_all = np.concatenate([minv] * args.batch)

    def launch_next():     # batch i+1's detector queued on the stream, nothing waited for
        imgs, up = nxt[0].result()
        nxt[0] = ahead.submit(dec_up)
        return imgs, be.detect_launch(imgs, params[:len(imgs)], pre=up)

    cur = [None]

    def step():
        # software pipeline: batch i's detections are read, its recogniser queued, batch i+1's
        # detector queued behind it, and only then is batch i's embedding copy waited for -- the
        # host work between batches (parse, geometry, launches) overlaps GPU work
        if cur[0] is None:
            cur[0] = launch_next()
        imgs, st = cur[0]
        t = StageTimer("face-bench", gpu=args.gpu_timers)
        with use_timer(t):
            be.detect_finish(st)
            h = be.embed_faces_async(imgs, idx[:len(imgs) * args.faces], minv_all[:len(imgs) * args.faces])
            cur[0] = launch_next()
            emb = be.embed_wait(h)
        if runner is not None:   # DP result gather: every rank gets every image's faces
            res = [[(FaceDetection(bbox=(490.0 + 3 * k, 280.0, 590.0, 420.0), confidence=1.0,
                                   landmarks=[tuple(p) for p in lms + 3 * k]), emb[i * args.faces + k])
                    for k in range(args.faces)] for i in range(len(imgs))]
            runner.gather(res, len(imgs) * world)
        for k, v in t.finish().items():
            stages[k] = stages.get(k, 0.0) + v

    found = []
    pend: list = []

    def step_real():
        # --real-dets: the detector's own output drives the recogniser (no fabricated rows); under
        # DP the whole SPMD path (services/face/spmd.py: SPMDFaceRunner.run -- shard, detect +
        # embed the shard, one all-gather of the packed results)
        imgs = [np.asarray(im) for im in dec()] * world        # the global batch: world x batch images
        t = StageTimer("face-bench", gpu=args.gpu_timers)
        with use_timer(t):
            if runner is not None:
                res = runner.run(imgs, [params[0]] * len(imgs), args.faces)
            elif args.pipeline:
                # pipelined, two detector batches in flight: batch i's kept rows are parsed while batch
                # i + 1's detector runs; batch i's warp + recogniser are queued behind it, then batch
                # i + 2's detector, and only then are batch i's embeddings waited for -- the GPU always
                # has the next batch queued while the host parses / builds the alignment geometry
                while len(pend) < 2:
                    pend.append(be.detect_launch(imgs, params[:len(imgs)]))
                st0 = pend.pop(0)
                dets = be.detect_finish(st0)
                h = be.embed_batch_detections_async(st0[0], dets, [args.faces] * len(st0[0]))
                nimgs = [np.asarray(im) for im in dec()]
                pend.append(be.detect_launch(nimgs, params[:len(nimgs)]))
                res = be.embed_batch_detections_wait(h)
            else:
                res = be.detect_and_embed_images(imgs, params[:len(imgs)], args.faces)
        found.append(sum(len(f) for f in res) / max(len(res), 1))
        for k, v in t.finish().items():
            stages[k] = stages.get(k, 0.0) + v

    if args.real_dets:
        # random-init SCRFD scores sit far below any threshold: the class-logit bias is bisected on
        # these images to the lowest value that still yields args.faces detections per image after
        # NMS (a realistic candidate count, not every anchor firing)
        A = det.cfg.anchors
        if pre is None:
            pre = decode_many(jpegs)
            dec = (lambda: pre)  # noqa: E731
        probe = [np.asarray(im) for im in pre[:4]]
        lo, hi = -8.0, 8.0      # bisect the bias: the lowest that still gives >= args.faces per image after NMS
        for _ in range(14):
            mid = 0.5 * (lo + hi)
            be.det.head_out.b.data[:A] = mid
            n = np.mean([len(d) for d in be.detect_images(probe, params[:len(probe)])])
            lo, hi = (lo, mid) if n >= args.faces else (mid, hi)
        be.det.head_out.b.data[:A] = hi
        step = step_real       # noqa: F811
    for _ in range(args.warmup):
        step()
    stages.clear()
    found.clear()
    if runner is not None:
        runner.comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    torch.cuda.synchronize()        # (includes the extra batch's queued detector: conservative)
    dt = (time.perf_counter() - t0) / args.iters
    if runner is not None:
        import torch.distributed as dist

        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return {"metric": "face detect+embed images/s (whole job)", "value": world * args.batch / dt, "unit": "img/s",
            "n_gpus": world, "parallelism": f"dp{world} (SPMD, RCCL all-gather of packed results)" if world > 1
            else "single GPU", "_rank": rank,
            "ms_per_batch": dt * 1000, "batch": args.batch, "faces_per_image": args.faces,
            ("gpu" if args.gpu_timers else "host") + "_stage_ms_per_batch":
                {k: round(v / args.iters, 2) for k, v in stages.items()},
            "faces_per_s": world * args.batch * args.faces / dt, "detector": "SCRFD-10G-shaped 640",
            "recogniser": f"IResNet-{args.rec}", "image": "1280x720 JPEG",
            "jpeg_decode": "excluded (decoded once up front)" if args.predecoded or args.real_dets else
                ("included (Pillow, host pool)" if args.pillow else
                 "included (device JPEG: host entropy decode pool + one batched GPU reconstruction)"),
            "image_kind": args.image_kind, "jpeg_kb": round(sum(len(j) for j in jpegs) / len(jpegs) / 1024, 1),
            "pipeline": ("real detections on the detector's own output, images pre-decoded, " +
                         ("SPMDFaceRunner.run" if runner is not None else
                          "two detector batches in flight: batch i+2's detector queued behind batch i's recogniser (detect_launch / "
                          "detect_finish / embed_batch_detections_async)" if args.pipeline else "detect_and_embed_images")
                         if args.real_dets else
                         "JPEG decode + pinned staging + H2D (own stream) of batch i+1 overlapped with the GPU "
                         "work of batch i; batch i+1's detector queued before batch i's embeddings are read"),
            "faces_found_per_image": round(float(np.mean(found)), 2) if found else None}


def bench_ocr(args):
    from lumen_amd.models.ocr import DBNET_PRESETS, REC_PRESETS, DBNet, SVTRRecognizer
    from lumen_amd.services.ocr.backend import DET_DEFAULTS, REC_DEFAULTS, MI355XOcrBackend, OcrParams

    runner, world, rank = None, 1, 0
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from lumen_amd.parallel import Communicator, init_distributed
        from lumen_amd.services.ocr.spmd import SPMDOcrRunner

        local = int(os.environ.get("LOCAL_RANK", "0"))
        st = init_distributed(tp_size=1, device=torch.device("cuda", local))
        world, rank = st.world, st.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    be = MI355XOcrBackend.__new__(MI355XOcrBackend)
    det = DBNet(DBNET_PRESETS["mobile"])
    det.random_init(torch.Generator().manual_seed(0))
    rec = SVTRRecognizer(REC_PRESETS["mobile"])
    rec.random_init(torch.Generator().manual_seed(1))
    be.det, be.rec, be.device, be.dtype = det.to(dev).eval(), rec.to(dev).eval(), dev, torch.bfloat16
    be.det_config, be.rec_config = dict(DET_DEFAULTS), dict(REC_DEFAULTS)
    be.rec_h, be.rec_batch, be.bucket = 48, 256, 32
    be.character_str = ["blank"] + [chr(0x4E00 + i) for i in range(REC_PRESETS["mobile"].num_classes - 1)]
    if world > 1:
        runner = SPMDOcrRunner(be, Communicator(st.dp_group, dev, ipc=False), dev)
    rng = np.random.default_rng(rank)
    jpegs = [encode_jpeg(synth_image(rng, 720, 960, args.image_kind)) for _ in range(args.batch)]
    boxes = []
    for k in range(args.crops):
        y = 20 + 25 * k
        boxes.append(np.array([[30, y], [30 + 200 + 10 * k, y], [30 + 200 + 10 * k, y + 22], [30, y + 22]], np.int32))

    from concurrent.futures import ThreadPoolExecutor

    ahead = ThreadPoolExecutor(max_workers=1)
    pre = decode_many(jpegs) if args.predecoded else None
    dec = (lambda: pre) if pre is not None else (lambda: decode_many(jpegs))  # noqa: E731
    nxt = [ahead.submit(dec)]

    from lumen_amd.runtime.metrics import StageTimer, use_timer

    stages: dict = {}

    # pipelined (default): batch i + 1's upload + detector go out on their own stream as soon as batch
    # i's connected components are back on the host, so the detector overlaps batch i's host geometry
    # and its recogniser (MI355XOcrBackend.detect_submit / detect_finish)
    det_stream = torch.cuda.Stream(dev) if args.pipeline and runner is None else None
    pending = [None]
    # JPEG-inclusive: the prefetch thread decodes batch i + 1 AND queues its upload + detector, so the
    # decode never waits in the main thread; pre-decoded: batch i + 1 goes out once batch i's connected
    # components are back (its detector then does not compete with batch i's labelling kernels)
    in_thread = det_stream is not None and pre is None

    def dec_submit():
        if not args.pillow:
            # device JPEG: host entropy decode on the pool + one batched GPU reconstruction, queued on
            # the detector's stream; the detector and the recogniser's crop warps read that buffer
            with torch.cuda.stream(det_stream):
                nimgs, pre_dev = be.decode_device(jpegs)
            return be.detect_submit(nimgs, [OcrParams()] * len(nimgs), stream=det_stream, pre=pre_dev)
        nimgs = dec()
        return be.detect_submit(nimgs, [OcrParams()] * len(nimgs), stream=det_stream)

    if in_thread:
        nxt[0] = ahead.submit(dec_submit)

    def step():
        t = StageTimer("ocr-bench", gpu=args.gpu_timers)
        if det_stream is not None:
            with use_timer(t):
                if in_thread:
                    h = nxt[0].result()
                    nxt[0] = ahead.submit(dec_submit)
                    launch_next = None
                else:
                    if pending[0] is None:
                        imgs0 = nxt[0].result()
                        nxt[0] = ahead.submit(dec)
                        pending[0] = be.detect_submit(imgs0, [OcrParams()] * len(imgs0), stream=det_stream)
                    h = pending[0]

                    def launch_next():
                        nimgs = nxt[0].result()
                        nxt[0] = ahead.submit(dec)
                        pending[0] = be.detect_submit(nimgs, [OcrParams()] * len(nimgs), stream=det_stream)

                be.detect_finish(h, on_gpu_done=launch_next)
                imgs = h["images"]
                crops = [(i, b) for i in range(len(imgs)) for b in boxes]
                be.recognize(imgs, crops, upload=h["upload"])
            torch.cuda.current_stream().synchronize()
            for k, v in t.finish().items():
                stages[k] = stages.get(k, 0.0) + v
            return
        imgs = nxt[0].result()
        nxt[0] = ahead.submit(dec)
        with use_timer(t):
            be.detect(imgs, [OcrParams()] * len(imgs))
            crops = [(i, b) for i in range(len(imgs)) for b in boxes]
            texts = be.recognize(imgs, crops)
        if runner is not None:   # DP result gather: every rank gets every image's lines
            from lumen_amd.services.ocr.backend import OcrResult

            lines = [[] for _ in imgs]
            for (i, b), (txt, sc) in zip(crops, texts):
                lines[i].append(OcrResult(box=[(int(x), int(y)) for x, y in b.tolist()], text=txt, confidence=sc))
            runner.gather(lines, len(imgs) * world)
        torch.cuda.synchronize()
        for k, v in t.finish().items():
            stages[k] = stages.get(k, 0.0) + v

    for _ in range(args.warmup):
        step()
    stages.clear()                      # stage times of the timed steps only
    if runner is not None:
        runner.comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    dt = (time.perf_counter() - t0) / args.iters
    if runner is not None:
        import torch.distributed as dist

        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    n_steps = args.iters
    return {"metric": "ocr images/s (whole job)", "value": world * args.batch / dt, "unit": "img/s",
            "n_gpus": world, "parallelism": f"dp{world} (SPMD, RCCL all-gather of packed lines)" if world > 1
            else "single GPU", "_rank": rank, "ms_per_batch": dt * 1000,
            ("gpu" if args.gpu_timers else "host") + "_stage_ms_per_batch":
                {k: round(v / n_steps, 2) for k, v in stages.items()},
            "batch": args.batch, "crops_per_image": args.crops, "crops_per_s": world * args.batch * args.crops / dt,
            "jpeg_decode": "excluded (decoded once up front)" if args.predecoded or args.real_dets else
                ("included (host decode pool)" if args.pillow or not in_thread else
                 "included (device JPEG: host entropy decode pool + one batched GPU reconstruction)"),
            "image_kind": args.image_kind, "jpeg_kb": round(sum(len(j) for j in jpegs) / len(jpegs) / 1024, 1),
            "detector": "DBNet-mobile 960", "recogniser": "SVTR-LCNet mobile", "image": "960x720 JPEG",
            "pipeline": "batch i+1 upload + detector on a second stream, overlapping batch i's DB host geometry and "
                        "recogniser" if det_stream is not None else "one batch at a time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["face", "ocr"], default="face")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--faces", type=int, default=4)
    ap.add_argument("--crops", type=int, default=20)
    ap.add_argument("--rec", default="r100")
    ap.add_argument("--gpus", type=int, default=1, help="SPMD data parallel over N ranks (torchrun)")
    ap.add_argument("--image-kind", choices=["noise", "photo"], default="noise",
                    help="synthetic JPEG content: uniform noise (worst-case host decode) or photo-like")
    ap.add_argument("--gpu-timers", action="store_true",
                    help="OCR stage times from HIP events (device time per stage) instead of host clocks")
    ap.add_argument("--pillow", action="store_true",
                    help="JPEG-inclusive face / OCR: decode on the host pool instead of the device JPEG path")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="ocr / face --real-dets: one batch at a time (no detector / recogniser overlap across "
                         "batches)")
    ap.add_argument("--real-dets", action="store_true",
                    help="face: the recogniser embeds the detector's real output (seeded head bias), SPMD via "
                         "SPMDFaceRunner.run")
    ap.add_argument("--predecoded", action="store_true",
                    help="decode the JPEGs once up front (GPU pipeline throughput without host JPEG decode)")
    a = ap.parse_args()
    load_hip(required=True)
    with torch.no_grad():
        out = bench_face(a) if a.what == "face" else bench_ocr(a)
    out.update({"dtype": "bf16", "data": "synthetic (random-init weights, random JPEGs)"})
    if out.pop("_rank", 0) == 0:
        print(json.dumps(out))
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from lumen_amd.parallel import destroy

        destroy()


if __name__ == "__main__":
    main()
