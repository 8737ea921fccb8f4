"""Service-level VLM time to first token: the hub's gRPC ``vlm_generate_stream`` task end to end
(JPEG bytes in the request -> first streamed chunk at the client), the way a Lumen client sees it,
next to tools/vlm_bench.py's engine-API TTFT.  Synthetic LLaVA-Llama-3-8B pack (random-init
weights on the device, byte-level tokenizer), fp8 decoder (LUMEN_VLM_FP8=1), one GPU.

    python tools/vlm_service_ttft.py [--n 30] [--warmup 3] [--prompt-chars 40] [--max-new 32] [--frontends 2]

``--frontends K``: the serving topology (hub/server.py serve_frontends): K gRPC front-end processes
feeding one GPU engine process that holds the model; the engine streams each token back over the
shared-memory channel as it is produced (partial records), so the first chunk does not wait for the
last token.  Without it: an in-process hub.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prompt-chars", type=int, default=40)
    ap.add_argument("--max-new", type=int, default=8)
    ap.add_argument("--fp8", type=int, default=1)
    ap.add_argument("--frontends", type=int, default=0)
    ap.add_argument("--preset", default="llava-llama3-8b")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    if a.fp8:
        os.environ["LUMEN_VLM_FP8"] = "1"
    import grpc

    from lumen_amd.hub.router import HubRouter
    from lumen_amd.hub.server import AppService, build_server
    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.proto import ml_service as pb
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.utils.image import encode_jpeg
    from tools.vlm_bench import synth_image

    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        free_port = so.getsockname()[1]
    cache = tempfile.mkdtemp(prefix="lumen-vlm-ttft-")
    write_vlm_model(os.path.join(cache, "models", a.preset), a.preset)
    svc = {"enabled": True, "package": "lumen_vlm",
           "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                           "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
           "backend_settings": {"device": a.device, "batch_size": 8},
           "models": {"general": {"model": a.preset, "runtime": "onnx"}}}
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": cache},
           "deployment": {"mode": "hub", "services": ["vlm"]},
           "server": {"port": free_port, "host": "127.0.0.1"}, "services": {"vlm": svc}}
    t0 = time.time()
    app = server = th = stop = None
    if a.frontends > 0:
        import multiprocessing as mp
        import threading

        import yaml

        from lumen_amd.hub.server import serve_frontends

        cfg_path = os.path.join(cache, "cfg.yaml")
        with open(cfg_path, "w") as f:
            yaml.safe_dump(cfg, f)
        stop = threading.Event()
        ready = mp.get_context("spawn").Queue()
        th = threading.Thread(target=serve_frontends, args=(cfg_path, free_port, a.frontends),
                              kwargs={"stop_event": stop, "ready_q": ready,
                                      "devices": ["cuda:0" if a.device == "cuda" else a.device]})
        th.start()
        for _ in range(a.frontends):
            ready.get(timeout=1200)
        port = free_port
    else:
        app = AppService.from_app_config(config_from_dict(cfg))
        server, port = build_server(HubRouter(app.services), "127.0.0.1", 0)
        server.start()
    load_s = time.time() - t0
    jpeg = encode_jpeg(synth_image(np.random.default_rng(0), 768, 1024, "photo"))
    prompt = ("Describe the picture " * 8)[:a.prompt_chars]
    meta = {"prompt": prompt, "max_new_tokens": str(a.max_new)}
    ttft, total, chunks, gaps, lag, egaps = [], [], [], [], [], []
    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        stub = pb.InferenceStub(ch)
        for i in range(a.warmup + a.n):
            t = time.perf_counter()
            first, n, last, last_te = None, 0, None, None
            for r in stub.Infer(iter([pb.InferRequest(correlation_id=str(i), task="vlm_generate_stream", payload=jpeg,
                                                      payload_mime="image/jpeg", meta=meta)]), timeout=300):
                if r.HasField("error"):
                    raise RuntimeError(r.error.message)
                now = time.perf_counter()
                te = r.meta.get("t_emit")
                if te is not None and i >= a.warmup:
                    tw = time.time()
                    lag.append((tw - float(te)) * 1e3)          # engine emit -> client receive
                    if last_te is not None:
                        egaps.append((float(te) - last_te) * 1e3)
                    last_te = float(te)
                if first is None:
                    first = now
                elif i >= a.warmup:
                    gaps.append((now - last) * 1e3)
                last = now
                n += 1
            if i >= a.warmup:
                ttft.append((first - t) * 1e3)
                total.append((time.perf_counter() - t) * 1e3)
                chunks.append(n)
    eng_stats = None
    if server is not None:
        try:
            svc_obj = app.services["vlm"] if isinstance(app.services, dict) else app.services[0]
            eng = svc_obj.backend.engine
            eng_stats = dict(eng.stats, graphs=sorted(eng.graphs.graphs) if eng.graphs is not None else None)
        except Exception as e:  # noqa: BLE001 - diagnostics only
            eng_stats = repr(e)
        server.stop(0)
        app.close()
    else:
        stop.set()
        th.join(300)
    print(json.dumps({"metric": "VLM p50 TTFT (service: gRPC vlm_generate_stream, first chunk)",
                      "value": round(float(np.percentile(ttft, 50)), 3), "unit": "ms",
                      "p99_ms": round(float(np.percentile(ttft, 99)), 3),
                      "request_ms_p50": round(float(np.percentile(total, 50)), 3),
                      "chunks_per_request": float(np.median(chunks)), "n": a.n,
                      "engine_stats": eng_stats,
                      "inter_chunk_ms_p50": round(float(np.percentile(gaps, 50)), 3) if gaps else None,
                      "engine_inter_emit_ms_p50": round(float(np.percentile(egaps, 50)), 3) if egaps else None,
                      "emit_to_client_ms_p50": round(float(np.percentile(lag, 50)), 3) if lag else None, "load_s": round(load_s, 1),
                      "config": {"model": f"{a.preset} (synthetic pack, random-init weights)", "device": a.device,
                                 "decoder": "fp8" if a.fp8 else "bf16", "image": f"1024x768 JPEG {len(jpeg) // 1024} KiB",
                                 "prompt_chars": a.prompt_chars, "max_new_tokens": a.max_new,
                                 "topology": f"{a.frontends} front ends + 1 GPU engine (token stream over the shm "
                                             f"channel)" if a.frontends else "in-process hub"}}), flush=True)


if __name__ == "__main__":
    main()
