"""VLM decoder / engine / service on the MI355X path vs the fp32 CPU reference."""
import json

import numpy as np
import pytest
import torch

from lumen_amd.models.llm import LLM, LLM_PRESETS, LLMConfig
from lumen_amd.runtime.engine import LLMEngine, SamplingParams
from lumen_amd.runtime.kv_cache import PagedKVCache

pytestmark = pytest.mark.gpu


def _cos(a, b):
    return torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()


@pytest.mark.parametrize("preset", ["qwen2-0.5b", "llama-small"])
def test_decoder_gpu_vs_cpu(preset):
    if preset == "llama-small":
        cfg = LLMConfig(vocab_size=32000, hidden_size=1024, num_layers=4, num_heads=8, num_kv_heads=2, head_dim=128,
                        intermediate_size=2816, rope_theta=500000.0, rms_eps=1e-5, max_position=4096,
                        tie_word_embeddings=False, qkv_bias=False)
    else:
        cfg = LLM_PRESETS[preset]
    ref = LLM(cfg, dtype=torch.float32, device="cpu")
    ref.random_init(1)
    gpu = LLM(cfg, dtype=torch.bfloat16, device="cuda")
    gpu.load_state_dict({k: v.to(torch.bfloat16) if v.dtype == torch.float32 and "qkv_b" not in k else v
                         for k, v in ref.state_dict().items()}, strict=False)
    T = 150
    ids = torch.randint(0, cfg.vocab_size, (T + 3,), generator=torch.Generator().manual_seed(0))
    outs = {}
    for name, m, dev in (("cpu", ref, "cpu"), ("gpu", gpu, "cuda")):
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=16, device=dev,
                          dtype=torch.float32 if dev == "cpu" else torch.bfloat16)
        kv.blocks.reserve(1, T + 3)
        lg = [m.prefill(m.embed_tokens(ids[:T].to(dev)), kv, torch.from_numpy(kv.slots(1, 0, T)).to(dev)).cpu()]
        bt = torch.from_numpy(kv.block_table([1])).to(dev)
        for p in range(T, T + 3):
            lg.append(m.decode(ids[p:p + 1].to(dev), torch.tensor([p], dtype=torch.int32, device=dev),
                               torch.from_numpy(kv.slots(1, p, 1)).to(dev), kv, bt,
                               torch.tensor([p + 1], dtype=torch.int32, device=dev)).cpu())
        outs[name] = lg
    for a, b in zip(outs["gpu"], outs["cpu"]):
        assert _cos(a, b) > 0.995


def test_engine_gpu_batched():
    cfg = LLM_PRESETS["qwen2-0.5b"]
    m = LLM(cfg, device="cuda")
    m.random_init(2)
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=256, device="cuda")
    eng = LLMEngine(m, kv, lambda ids: m.embed_tokens(torch.tensor(ids, device="cuda")), max_batch=16)
    try:
        prompts = [list(np.random.default_rng(i).integers(0, 150000, 30 + 11 * i)) for i in range(6)]
        solo = []
        for p in prompts:
            r = eng.submit(p, len(p), SamplingParams(max_new_tokens=5))
            list(r.stream(timeout=120))
            solo.append(r.tokens)
        rs = [eng.submit(p, len(p), SamplingParams(max_new_tokens=5)) for p in prompts]
        agree = 0
        for r, ref in zip(rs, solo):
            list(r.stream(timeout=120))
            assert len(r.tokens) == 5
            agree += r.tokens[:2] == ref[:2]
        assert agree >= 5          # bf16 batch-vs-solo rounding may flip a near-tie
        s = eng.submit(prompts[0], len(prompts[0]), SamplingParams(max_new_tokens=16, temperature=0.8, top_p=0.9,
                                                                   repetition_penalty=1.2, seed=1))
        list(s.stream(timeout=120))
        assert len(s.tokens) == 16
    finally:
        eng.close()


def test_vlm_service_gpu(tmp_path):
    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.vlm import GeneralFastVLMService
    from lumen_amd.utils.image import encode_jpeg

    write_vlm_model(tmp_path / "models" / "fastvlm-tiny", "fastvlm-tiny")
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(tmp_path)},
           "deployment": {"mode": "single", "service": "vlm"}, "server": {"port": 50557, "host": "127.0.0.1"},
           "services": {"vlm": {"enabled": True, "package": "lumen_vlm",
                                "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                                                "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                                "backend_settings": {"device": "cuda"},
                                "models": {"general": {"model": "fastvlm-tiny", "runtime": "onnx"}}}}}
    s = GeneralFastVLMService.from_config(config_from_dict(cfg).services["vlm"], tmp_path)
    s.initialize()
    try:
        img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (50, 70, 3), dtype=np.uint8))
        body, _, meta = s.handle("vlm_generate", img, "image/jpeg", {"prompt": "Describe.", "max_new_tokens": "10"})
        d = json.loads(body)
        assert d["generated_tokens"] == 10 and float(meta["ttft_ms"]) > 0
        out = list(s.handle("vlm_generate_stream", img, "image/jpeg", {"prompt": "Hi", "max_new_tokens": "7"}))
        assert json.loads(out[-1][0])["generated_tokens"] == 7 and out[-1][3]
    finally:
        s.close()


def test_decode_graphs_match_eager():
    cfg = LLM_PRESETS["qwen2-0.5b"]
    m = LLM(cfg, device="cuda")
    m.random_init(5)
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=64, device="cuda")
    prompts = [list(np.random.default_rng(i).integers(0, 150000, 40 + 9 * i)) for i in range(3)]
    outs = {}
    for graphs in (False, True):
        eng = LLMEngine(m, kv, lambda ids: m.embed_tokens(torch.tensor(ids, device="cuda")), max_batch=4,
                        use_graphs=graphs)
        try:
            # different lengths: requests leave the batch at different steps (look-ahead discards)
            rs = [eng.submit(p, len(p), SamplingParams(max_new_tokens=6 + 5 * i)) for i, p in enumerate(prompts)]
            for r in rs:
                list(r.stream(timeout=120))
            outs[graphs] = [r.tokens for r in rs]
            if graphs:
                assert eng.graphs is not None and eng.graphs.graphs, "decode graphs were not captured"
                assert eng.stats.get("lookahead_steps", 0) > 0, "look-ahead decode never engaged"
        finally:
            eng.close()
    assert outs[True] == outs[False]


def test_chunked_prefill_gpu_matches_single_shot():
    """Chunked prefill on the HIP kernels (prefix K/V gathered from the paged cache, causal
    attention aligned to the last key) reproduces the single-shot prefill's logits and
    K/V cache, and the engine streams with 128-token chunks."""
    cfg = LLM_PRESETS["qwen2-0.5b"]
    m = LLM(cfg, device="cuda")
    m.random_init(4)
    ids = torch.tensor(np.random.default_rng(20).integers(0, 150000, 700), device="cuda")
    res = {}
    for chunk in (700, 128):
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=32, device="cuda")
        assert kv.blocks.reserve(1, 700)
        x = m.embed_tokens(ids)
        tab = torch.from_numpy(np.asarray(kv.blocks.table(1), np.int64)).cuda()
        for s in range(0, 700, chunk):
            e = min(700, s + chunk)
            slots = torch.from_numpy(kv.slots(1, s, e - s)).cuda()
            logits = m.prefill(x[s:e], kv, slots, start_pos=s, prefix_blocks=tab[: -(-e // 64)] if s else None)
        res[chunk] = (logits.float(), kv.k[5][tab].float())
    assert _cos(res[128][0], res[700][0]) > 0.999
    assert _cos(res[128][1], res[700][1]) > 0.999
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=64, device="cuda")
    eng = LLMEngine(m, kv, lambda t: m.embed_tokens(torch.tensor(t, device="cuda")), max_batch=8, prefill_chunk=128)
    try:
        rs = [eng.submit(list(ids.cpu().numpy()[:n]), n, SamplingParams(max_new_tokens=6)) for n in (700, 90, 333)]
        for r in rs:
            list(r.stream(timeout=120))
            assert len(r.tokens) == 6
        assert eng.stats["prefill_chunks"] >= 6 + 1 + 3
    finally:
        eng.close()


def test_engine_fp8_kv_cache_serves():
    """The engine on an OCP e4m3 paged KV cache (eager and hipGraph decode give the same tokens;
    first-step logits close to the bf16-cache run: per-element fp8 rounding of K / V only)."""
    cfg = LLM_PRESETS["qwen2-0.5b"]
    m = LLM(cfg, device="cuda")
    m.random_init(6)
    prompts = [list(np.random.default_rng(10 + i).integers(0, 150000, 70 + 30 * i)) for i in range(2)]
    toks = {}
    for dt, graphs in ((torch.float8_e4m3fn, False), (torch.float8_e4m3fn, True)):
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=32, device="cuda", dtype=dt)
        eng = LLMEngine(m, kv, lambda ids: m.embed_tokens(torch.tensor(ids, device="cuda")), max_batch=4,
                        use_graphs=graphs)
        try:
            rs = [eng.submit(p, len(p), SamplingParams(max_new_tokens=5)) for p in prompts]
            for r in rs:
                list(r.stream(timeout=120))
            toks[graphs] = [r.tokens for r in rs]
        finally:
            eng.close()
    assert toks[True] == toks[False] and all(len(t) == 5 for t in toks[True])
    # one decode step on the two cache dtypes from the same prefill
    logits = []
    p = prompts[1]
    for dt in (torch.bfloat16, torch.float8_e4m3fn):
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=8, device="cuda", dtype=dt)
        T = len(p)
        slots = torch.arange(T + 1, device="cuda", dtype=torch.long)
        m.prefill(m.embed_tokens(torch.tensor(p, device="cuda")), kv, slots[:T])
        bt = torch.arange(8, device="cuda", dtype=torch.int32).view(1, 8)
        lg = m.decode(torch.tensor([5], device="cuda"), torch.tensor([T], device="cuda", dtype=torch.int32),
                      slots[T:T + 1], kv, bt, torch.tensor([T + 1], device="cuda", dtype=torch.int32))
        logits.append(lg.float().cpu())
    assert _cos(logits[0], logits[1]) > 0.99


def test_vlm_backend_fp8_shard_cache(tmp_path, monkeypatch):
    """precision fp8 on the GPU: the first build writes this rank's quantised shard
    (.lumen_shards/tp1_r0_fp8-fp8.safetensors: compute dtype + configured precision), the second
    build loads it (no requantisation) and
    generates the same greedy tokens."""
    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.vlm.backend import ChatMessage, GenerationRequest, create_backend

    write_vlm_model(tmp_path / "models" / "fastvlm-tiny", "fastvlm-tiny")
    res = load_model_resources(tmp_path, ModelConfig(model="fastvlm-tiny", runtime=Runtime.onnx, precision="fp8"))
    settings = type("S", (), {"device": "cuda"})()
    shard = tmp_path / "models" / "fastvlm-tiny" / ".lumen_shards" / "tp1_r0_fp8-fp8.safetensors"
    outs = []
    for i in range(2):
        b = create_backend(settings, res, "onnx")
        b.initialize()
        try:
            assert shard.is_file()
            assert b.model.llm.weight_dtype == "fp8"
            if i == 0:
                mtime = shard.stat().st_mtime_ns
            else:
                assert shard.stat().st_mtime_ns == mtime          # loaded, not rewritten
            from lumen_amd.utils.image import encode_jpeg

            jpg = encode_jpeg(np.random.default_rng(0).integers(0, 255, (40, 60, 3), dtype=np.uint8))
            req = GenerationRequest(messages=[ChatMessage(role="user", content="hello there")], image_bytes=jpg,
                                    max_new_tokens=8, temperature=0.0)
            outs.append(b.generate(req).text)
        finally:
            b.close()
    assert outs[0] == outs[1]


@pytest.mark.parametrize("preset,fp8", [("tiny", False), ("tiny", True), ("tiny-fastvit", False)])
def test_image_encoder_graph_and_encode_ahead(preset, fp8):
    """The image encoder replayed from its hipGraph (models/vlm.py:_graph_encode) equals the eager
    launches, and a prompt built from encode_ahead's EncodedImage equals one built from the raw
    image (the service encodes in the request's thread)."""
    from lumen_amd.models.vlm import VLM, VLM_PRESETS, EncodedImage

    if preset not in VLM_PRESETS:
        pytest.skip(f"no {preset} preset")
    m = VLM(VLM_PRESETS[preset], device="cuda")
    m.random_init(3)
    if fp8:
        m.quantize_fp8()
    imgs = [torch.randint(0, 256, (40 + 7 * i, 52, 3), dtype=torch.uint8, device="cuda") for i in range(2)]
    with torch.no_grad():
        for k in (1, 2):
            eager = m._encode_tower(m.preprocess(imgs[:k]), k)
            g1 = m.encode_images(imgs[:k])
            g2 = m.encode_images(imgs[:k])           # replay
            assert torch.equal(g1, eager) and torch.equal(g2, eager)
        assert m._vgraphs and all(v is not False for v in m._vgraphs.values())
        ids = [5, 6, m.cfg.image_token_id, 7, 8]
        ref = m.build_prefill(ids, [imgs[0]])
        enc = m.encode_ahead([imgs[0]])
        assert isinstance(enc[0], EncodedImage)
        got = m.build_prefill(ids, enc)
        assert torch.equal(got, ref)
        pre = m.prepare_prefill(ids, [imgs[0]])
        assert torch.equal(pre.x, ref)
        m.invalidate_graphs()
        assert not m._vgraphs
