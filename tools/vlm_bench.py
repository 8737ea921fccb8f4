"""VLM time-to-first-token / decode throughput benchmark (BASELINE metric "VLM p50 TTFT").

TTFT is measured like the reference's generate() up to its first sampled token
(packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:161-214): JPEG decode ->
pad/resize/normalise -> vision tower -> projector -> token embeddings + image splice
-> full prefill -> first token, single request, random-init weights of the named
architecture, synthetic 1024x768 JPEG.  Also reports single-stream decode tokens/s and
batched decode throughput with concurrent requests on the continuous-batching engine.

usage: python tools/vlm_bench.py --preset fastvlm-0.5b --n 20 --max-new 64 --batch 16
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
from lumen_amd.models.vlm import VLM, VLM_PRESETS  # noqa: E402
from lumen_amd.runtime.engine import LLMEngine, SamplingParams  # noqa: E402
from lumen_amd.runtime.kv_cache import PagedKVCache  # noqa: E402
from lumen_amd.utils.image import decode_rgb, encode_jpeg  # noqa: E402
from lumen_amd.models.vlm import ENCODE_AHEAD, PreparedPrefill  # noqa: E402
from lumen_amd.utils.jpeg import decode_image  # noqa: E402
from tools.face_ocr_bench import synth_image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="fastvlm-0.5b")
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--batch-max-new", type=int, default=256,
                    help="tokens per stream in the batched phase (long enough that all streams overlap)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--max-new", type=int, default=64)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--prompt-tokens", type=int, default=48)
    ap.add_argument("--kv-blocks", type=int, default=4096)
    ap.add_argument("--full-decode", action="store_true", help="host decode: the JPEG at full resolution")
    ap.add_argument("--host-decode", action="store_true", help="Pillow on the host instead of the device JPEG path")
    ap.add_argument("--fp8", action="store_true", help="weight-only OCP e4m3 decoder weights (per-channel scales)")
    ap.add_argument("--kv-fp8", action="store_true", help="OCP e4m3 paged KV cache (unit scale)")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="idle time between the TTFT requests (0: back to back, the next request arrives as the "
                         "previous stream ends)")
    ap.add_argument("--image-kind", choices=["noise", "photo"], default="noise",
                    help="synthetic JPEG content: uniform noise (worst-case host decode) or photo-like")
    args = ap.parse_args()
    load_hip(required=True)
    dev = torch.device("cuda")
    cfg = VLM_PRESETS[args.preset]
    t0 = time.time()
    m = VLM(cfg, device=dev)
    m.random_init(0)
    if args.fp8:
        m.quantize_fp8()
    torch.cuda.synchronize()
    load_s = time.time() - t0
    kv = PagedKVCache(cfg.llm.num_layers, m.llm.Hkv, cfg.llm.head_dim, num_blocks=args.kv_blocks, device=dev,
                      dtype=torch.float8_e4m3fn if args.kv_fp8 else torch.bfloat16)

    dec_ms, enc_ms = [], []
    # JPEG decoded with libjpeg DCT scaling down to >= the vision input (as the VLM service does,
    # services/vlm/backend.py:jpeg_draft_size); --full-decode measures the full-resolution decode
    draft = None if args.full_decode else (cfg.vision.image_size, cfg.vision.image_size)

    # as in the VLM service (services/vlm/backend.py _submit): the JPEG is decoded in the caller's
    # thread before the request is queued, so the engine thread never blocks on it; TTFT below is
    # still measured from BEFORE the decode (request arrival -> first token)
    build_ms = []

    def build(a):
        ids, img = a
        t = time.perf_counter()
        x = img.x if isinstance(img, PreparedPrefill) else m.build_prefill(ids, [img])
        build_ms.append((time.perf_counter() - t) * 1000)
        return x

    def decode(jpeg):
        # as the service: baseline JPEGs -> parallel host entropy decode + GPU reconstruction
        # (utils/jpeg.py); --host-decode: Pillow on the host (DCT-scaled unless --full-decode)
        t = time.perf_counter()
        img = torch.from_numpy(decode_rgb(jpeg, draft_to=draft)) if args.host_decode else \
            decode_image(jpeg, dev, draft_to=draft)
        dec_ms.append((time.perf_counter() - t) * 1000)
        return img

    def prepare(ids, img):
        # as the service: the prompt embeddings and the image encoder are queued in the request's
        # thread (models/vlm.py:prepare_prefill) before the engine admits the request
        if not ENCODE_AHEAD:
            return img
        t = time.perf_counter()
        pre = m.prepare_prefill(ids, [img])
        enc_ms.append((time.perf_counter() - t) * 1000)
        return pre if pre is not None else img

    eng = LLMEngine(m.llm, kv, build, max_batch=max(args.batch, 1))
    rng = np.random.default_rng(0)
    jpeg = encode_jpeg(synth_image(rng, 768, 1024, args.image_kind))
    V = cfg.llm.vocab_size
    text = [int(t) for t in rng.integers(1000, min(V, 30000), args.prompt_tokens)]
    ids = text[:8] + [cfg.image_token_id] + text[8:]
    full, _ = m.expand_image_tokens(ids, 1)
    eos_none = SamplingParams(max_new_tokens=args.max_new, stop_token_ids=())

    def one(max_new):
        t_arrive = time.perf_counter()
        r = eng.submit((ids, prepare(ids, decode(jpeg))), len(full), SamplingParams(max_new_tokens=max_new))
        r.t_arrive = t_arrive
        times = []
        for kind, _ in r.stream(timeout=600):
            times.append(time.perf_counter())
        return r, times

    for _ in range(args.warmup):
        one(4)
    ttft, tps, queue_ms, admit_first_ms = [], [], [], []
    dec_ms.clear()
    for _ in range(args.n):
        if args.gap_ms > 0:
            time.sleep(args.gap_ms / 1000)
        r, times = one(args.max_new)
        ttft.append((r.t_first - r.t_arrive) * 1000)
        queue_ms.append((r.t_admit - r.t_submit) * 1000)
        admit_first_ms.append((r.t_first - r.t_admit) * 1000)
        if len(r.tokens) > 1:
            tps.append((len(r.tokens) - 1) / (times[len(r.tokens) - 1] - times[0]))
    # batched decode throughput
    # (16 concurrent clients: each decodes its JPEG in its own thread, then submits)
    from concurrent.futures import ThreadPoolExecutor

    if args.batch <= 0:       # TTFT / single-stream only (profiling runs)
        eng.close()
        print(json.dumps({"metric": "VLM p50 TTFT", "value": float(np.percentile(ttft, 50)), "unit": "ms",
                          "admit_to_first_token": float(np.median(admit_first_ms)),
                          "queue": float(np.median(queue_ms)), "build_host_ms": float(np.median(build_ms[-args.n:])),
                          "encode_ahead_host_ms": float(np.median(enc_ms[-args.n:])) if enc_ms else None,
                          "jpeg_decode": float(np.median(dec_ms[:args.n])),
                          "decode_tok_s_single": float(np.median(tps)) if tps else None, "n": args.n,
                          "gap_ms": args.gap_ms}))
        return
    t1 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=max(args.batch, 1)) as ex:
        rs = list(ex.map(lambda _: eng.submit((ids, prepare(ids, decode(jpeg))), len(full),
                                              SamplingParams(max_new_tokens=args.batch_max_new)), range(args.batch)))
    # steady-state batched decode: per-token arrival times of every stream; the window starts
    # when the LAST request has its first token (all B in the running batch) and ends when the
    # first request finishes (the batch starts shrinking)
    stamps = [[] for _ in rs]

    def drain(i):
        for _ in rs[i].stream(timeout=900):
            stamps[i].append(time.perf_counter())

    with ThreadPoolExecutor(max_workers=len(rs)) as ex:
        list(ex.map(drain, range(len(rs))))
    ntok = sum(len(r.tokens) for r in rs)
    batch_s = time.perf_counter() - t1
    w0 = max(st[0] for st in stamps if st)
    w1 = min(st[-1] for st in stamps if st)
    in_win = sum(sum(1 for t in st if w0 < t <= w1) for st in stamps)
    batch_decode = in_win / (w1 - w0) if w1 > w0 else None
    eng.close()
    out = {"metric": "VLM p50 TTFT", "value": float(np.percentile(ttft, 50)), "unit": "ms",
           "higher_is_better": False, "p90_ttft_ms": float(np.percentile(ttft, 90)),
           "p99_ttft_ms": float(np.percentile(ttft, 99)),
           "min_ttft_ms": float(np.min(ttft)),
           "ttft_breakdown_ms": {"queue": float(np.median(queue_ms)), "jpeg_decode": float(np.median(dec_ms[:args.n])),
                                 "admit_to_first_token": float(np.median(admit_first_ms))},
           "decode_tok_s_single": float(np.median(tps)) if tps else None,
           "batch": args.batch, "batch_tok_s": ntok / batch_s,
           "batch_decode_tok_s": batch_decode, "batch_note": "batch_tok_s = all tokens / wall time incl. the "
           "B prefills; batch_decode_tok_s = steady-state decode while all B streams run",
           "prompt_tokens": len(full),
           "image_tokens": cfg.num_image_tokens, "max_new_tokens": args.max_new, "batch_max_new_tokens": args.batch_max_new, "n": args.n,
           "preset": args.preset, "kv_cache": "fp8-e4m3" if args.kv_fp8 else "bf16", "dtype": "bf16" if not args.fp8 else "fp8-e4m3 decoder (W8A8 prefill, fp8-weight decode), " + ("W8A8 MX vision" if getattr(m.vision, "w8a8", False) else "bf16 vision"), "data": f"synthetic (random-init weights, {args.image_kind} 1024x768 JPEG, {len(jpeg) // 1024} KiB)",
           "load_s": load_s, "kv_cache_tokens": kv.capacity_tokens,
           "jpeg_decode": ("host, full resolution" if args.full_decode else
                           f"host, DCT-scaled to >= {cfg.vision.image_size}px") if args.host_decode else
                          "parallel host entropy decode + GPU reconstruction, full resolution"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
