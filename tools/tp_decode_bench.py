"""Tensor-parallel VLM decode through the serving stack (leader + spawned follower ranks):
single-stream decode tokens/s and the step-descriptor counts.  Under rocprofv3 the kernel
trace gives the all-reduce share of the decode step (tools/rocpd_stats.py --ar-share).

  python tools/tp_decode_bench.py --preset llava-llama3-8b --tp 2 --fp8 [--share-gpu]

``--share-gpu`` runs every rank on GPU 0 with gloo for the host-side step broadcast (the only
way to run TP on a one-GPU box; the decode graphs' all-reduce is the IPC one-shot kernel).
Random-init weights of the named architecture, synthetic image / prompt.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llava-llama3-8b")
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--share-gpu", action="store_true")
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--max-new", type=int, default=64)
    ap.add_argument("--kv-blocks", type=int, default=512)
    a = ap.parse_args()
    os.environ["LUMEN_TP_SIZE"] = str(a.tp)
    os.environ["LUMEN_KV_BLOCKS"] = str(a.kv_blocks)
    if a.fp8:
        os.environ["LUMEN_VLM_FP8"] = "1"
    if a.share_gpu:
        os.environ["LUMEN_DIST_BACKEND"] = "gloo"
        os.environ["HIP_VISIBLE_DEVICES"] = os.environ.get("HIP_VISIBLE_DEVICES", "0").split(",")[0]
    import numpy as np

    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.vlm import GeneralFastVLMService
    from lumen_amd.utils.image import encode_jpeg

    cache = tempfile.mkdtemp(prefix="lumen_tp_")
    os.environ["LUMEN_TP_FOLLOWER_STATS"] = os.path.join(cache, "follower_stats")
    write_vlm_model(os.path.join(cache, "models", "vlm-bench"), "vlm-bench", preset=a.preset, weights=False)
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": cache},
           "deployment": {"mode": "single", "service": "vlm"}, "server": {"port": 50559, "host": "127.0.0.1"},
           "services": {"vlm": {"enabled": True, "package": "lumen_vlm",
                                "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                                                "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                                "backend_settings": {"device": "cuda"},
                                "models": {"general": {"model": "vlm-bench", "runtime": "onnx"}}}}}
    s = GeneralFastVLMService.from_config(config_from_dict(cfg).services["vlm"], cache)
    t0 = time.time()
    s.initialize()
    load_s = time.time() - t0
    img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (768, 1024, 3), dtype=np.uint8))
    meta = {"prompt": "Describe the image in detail.", "max_new_tokens": str(a.max_new)}
    try:
        s.handle("vlm_generate", img, "image/jpeg", dict(meta, max_new_tokens="4"))       # warm-up + captures
        rates, ttft = [], []
        for _ in range(a.n):
            t = time.perf_counter()
            body, _, m = s.handle("vlm_generate", img, "image/jpeg", meta)
            dt = time.perf_counter() - t
            ntok = int(m.get("tokens_generated", a.max_new)) if isinstance(m, dict) else a.max_new
            ft = float(m.get("ttft_ms", 0.0)) if isinstance(m, dict) else 0.0
            ttft.append(ft)
            rates.append((ntok - 1) / max(dt - ft / 1000.0, 1e-9))
        eng = s.backend.engine
        print(json.dumps({"metric": "VLM decode tokens/s (single stream)", "value": float(np.median(rates)),
                          "unit": "tokens/s", "tp": a.tp, "share_gpu": a.share_gpu, "preset": a.preset,
                          "fp8": a.fp8, "p50_ttft_ms": float(np.median(ttft)), "load_s": load_s,
                          "graphs": eng.graphs is not None and len(eng.graphs.graphs) > 0,
                          "sync": dict(eng.sync.stats) if eng.sync is not None else None,
                          "data": "synthetic (random-init weights, random 1024x768 JPEG)"}), flush=True)
    finally:
        s.close()
    fol = {}
    for r in range(1, a.tp):
        p = os.path.join(cache, f"follower_stats.rank{r}")
        if os.path.exists(p):
            fol[r] = json.load(open(p))
    print(json.dumps({"follower_stats": fol, "leader_lookahead_steps": eng.stats.get("lookahead_steps", 0)}), flush=True)


if __name__ == "__main__":
    main()
