"""VLM stack on the CPU reference path: decoder parity with HF transformers (Qwen2 and
Llama, prefill + paged decode, TP=2 over gloo), engine batching invariance, service."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lumen_amd.models.llm import LLM, LLM_PRESETS, LLMConfig, TPInfo
from lumen_amd.runtime.engine import LLMEngine, SamplingParams
from lumen_amd.runtime.kv_cache import PagedKVCache

transformers = pytest.importorskip("transformers")


def _hf(kind: str, cfg: LLMConfig, seed=0):
    torch.manual_seed(seed)
    if kind == "qwen2":
        hc = transformers.Qwen2Config(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                      num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                                      num_key_value_heads=cfg.num_kv_heads, intermediate_size=cfg.intermediate_size,
                                      rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
                                      max_position_embeddings=cfg.max_position, tie_word_embeddings=True)
        m = transformers.Qwen2ForCausalLM(hc)
    else:
        hc = transformers.LlamaConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                      num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                                      num_key_value_heads=cfg.num_kv_heads, intermediate_size=cfg.intermediate_size,
                                      rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
                                      max_position_embeddings=cfg.max_position, tie_word_embeddings=False,
                                      rope_scaling=cfg.rope_scaling)
        m = transformers.LlamaForCausalLM(hc)
    for n, p in m.named_parameters():
        if "bias" in n:
            p.data.normal_(0, 0.1)
        if "layernorm" in n or n.endswith("norm.weight"):
            p.data.normal_(1.0, 0.1)
    return m.eval()


def _cfgs():
    q = LLM_PRESETS["tiny"]
    l = LLMConfig(vocab_size=512, hidden_size=128, num_layers=2, num_heads=4, num_kv_heads=4, head_dim=32,
                  intermediate_size=256, rope_theta=500000.0, rms_eps=1e-5, max_position=2048,
                  tie_word_embeddings=False, qkv_bias=False,
                  rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                "high_freq_factor": 4.0, "original_max_position_embeddings": 64})
    return {"qwen2": q, "llama": l}


@pytest.mark.parametrize("kind", ["qwen2", "llama"])
def test_decoder_matches_hf(kind):
    cfg = _cfgs()[kind]
    hf = _hf(kind, cfg)
    m = LLM(cfg, dtype=torch.float32, device="cpu")
    m.load_hf_state_dict(hf.state_dict())
    ids = torch.randint(0, cfg.vocab_size, (1, 90), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(ids).logits[0]
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=8, dtype=torch.float32)
    kv.blocks.reserve(5, 90)
    x = m.embed_tokens(ids[0, :70])
    lg = m.prefill(x, kv, torch.from_numpy(kv.slots(5, 0, 70)))
    assert torch.allclose(lg[0], ref[69], atol=1e-4), (lg[0] - ref[69]).abs().max()
    bt = torch.from_numpy(kv.block_table([5]))
    for p in range(70, 90):   # crosses the 64-token block boundary
        lg = m.decode(ids[0, p:p + 1], torch.tensor([p], dtype=torch.int32), torch.from_numpy(kv.slots(5, p, 1)),
                      kv, bt, torch.tensor([p + 1], dtype=torch.int32))
        assert torch.allclose(lg[0], ref[p], atol=1e-4), (p, (lg[0] - ref[p]).abs().max())


def _tp_worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfgs()[kind]
        hf = _hf(kind, cfg)
        m = LLM(cfg, TPInfo(rank, world, None), dtype=torch.float32, device="cpu")
        m.load_hf_state_dict(hf.state_dict())
        ids = torch.randint(0, cfg.vocab_size, (1, 40), generator=torch.Generator().manual_seed(2))
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=4, dtype=torch.float32)
        kv.blocks.reserve(1, 41)
        lg = m.prefill(m.embed_tokens(ids[0]), kv, torch.from_numpy(kv.slots(1, 0, 40)))
        parts = [torch.empty_like(lg) for _ in range(world)]
        dist.all_gather(parts, lg)
        full = torch.cat(parts, 1)
        nxt = int(full.argmax())
        lg2 = m.decode(torch.tensor([nxt]), torch.tensor([40], dtype=torch.int32),
                       torch.from_numpy(kv.slots(1, 40, 1)), kv, torch.from_numpy(kv.block_table([1])),
                       torch.tensor([41], dtype=torch.int32))
        parts2 = [torch.empty_like(lg2) for _ in range(world)]
        dist.all_gather(parts2, lg2)
        if rank == 0:
            with torch.no_grad():
                ref = hf(torch.cat([ids, torch.tensor([[nxt]])], 1)).logits[0]
            e1 = (full[0] - ref[39]).abs().max().item()
            e2 = (torch.cat(parts2, 1)[0] - ref[40]).abs().max().item()
            q.put((e1, e2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["qwen2", "llama"])
def test_tensor_parallel_gloo(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:                 # a free port: a fixed one collides with earlier runs
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    e1, e2 = q.get(timeout=5)
    assert e1 < 1e-4 and e2 < 1e-4, (e1, e2)


def test_engine_batching_invariance():
    cfg = LLM_PRESETS["tiny"]
    m = LLM(cfg, dtype=torch.float32, device="cpu")
    m.random_init(3)
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=64, dtype=torch.float32)
    eng = LLMEngine(m, kv, lambda ids: m.embed_tokens(torch.tensor(ids)), max_batch=8)
    try:
        prompts = [list(np.random.default_rng(i).integers(0, cfg.vocab_size, 20 + 7 * i)) for i in range(5)]
        sp = SamplingParams(max_new_tokens=12)
        solo = []
        for p in prompts:
            r = eng.submit(p, len(p), SamplingParams(max_new_tokens=12))
            list(r.stream(timeout=60))
            solo.append(r.tokens)
        rs = [eng.submit(p, len(p), SamplingParams(max_new_tokens=12)) for p in prompts]
        for r, ref in zip(rs, solo):
            list(r.stream(timeout=60))
            assert r.tokens == ref and r.finish_reason == "length"
        assert eng.stats["decode_steps"] > 0 and kv.blocks.num_seqs() == 0
        # sampling with a seed is reproducible
        a = eng.submit(prompts[0], 20, SamplingParams(max_new_tokens=8, temperature=0.9, top_p=0.8, seed=7))
        list(a.stream(timeout=60))
        b = eng.submit(prompts[0], 20, SamplingParams(max_new_tokens=8, temperature=0.9, top_p=0.8, seed=7,
                                                      repetition_penalty=1.3))
        list(b.stream(timeout=60))
        assert len(a.tokens) == 8 and len(b.tokens) == 8
        # stop token
        stop = solo[1][-1]
        st = eng.submit(prompts[1], 27, SamplingParams(max_new_tokens=12, stop_token_ids=(stop,)))
        list(st.stream(timeout=60))
        assert st.finish_reason == "eos_token" and st.tokens == solo[1][:solo[1].index(stop)]
    finally:
        eng.close()


@pytest.fixture(scope="module")
def vlm_service(tmp_path_factory):
    from lumen_amd.models.vlm import write_vlm_model
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.vlm import GeneralFastVLMService

    d = tmp_path_factory.mktemp("cache")
    write_vlm_model(d / "models" / "fastvlm-tiny", "fastvlm-tiny")
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(d)},
           "deployment": {"mode": "single", "service": "vlm"}, "server": {"port": 50556, "host": "127.0.0.1"},
           "services": {"vlm": {"enabled": True, "package": "lumen_vlm",
                                "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                                                "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                                "backend_settings": {"device": "cpu"},
                                "models": {"general": {"model": "fastvlm-tiny", "runtime": "onnx"}}}}}
    s = GeneralFastVLMService.from_config(config_from_dict(cfg).services["vlm"], d)
    s.initialize()
    yield s
    s.close()


def _img():
    from lumen_amd.utils.image import encode_jpeg

    return encode_jpeg(np.random.default_rng(0).integers(0, 255, (40, 60, 3), dtype=np.uint8))


def test_vlm_service_generate(vlm_service):
    s = vlm_service
    body, mime, meta = s.handle("vlm_generate", _img(), "image/jpeg", {"prompt": "Describe.", "max_new_tokens": "9"})
    d = json.loads(body)
    assert mime == "application/json;schema=text_generation_v1"
    assert d["generated_tokens"] == 9 and d["finish_reason"] == "length" and meta["finish_reason"] == "length"
    assert d["model_id"] == "fastvlm-tiny_onnx" and d["input_tokens"] > 16   # 16 image tokens spliced in
    msgs = json.dumps([{"role": "system", "content": "be brief"}, {"role": "user", "content": "<image>\nwhat?"}])
    body2, _, _ = s.handle("vlm_generate", _img(), "image/jpeg", {"messages": msgs, "max_new_tokens": "4",
                                                                   "temperature": "0.7", "seed": "3"})
    assert json.loads(body2)["generated_tokens"] == 4
    with pytest.raises(ValueError):
        s.handle("vlm_generate", _img(), "image/jpeg", {})
    prompt = s.backend.build_prompt(s.backend._with_image_token(
        [__import__("lumen_amd.services.vlm", fromlist=["ChatMessage"]).ChatMessage("user", "hi")]))
    assert prompt.startswith("<|im_start|>user\n<image>\nhi<|im_end|>") and prompt.endswith("assistant")


def test_vlm_service_stream(vlm_service):
    from lumen_amd.proto import ml_service as pb

    req = pb.InferRequest(correlation_id="s1", task="vlm_generate_stream", payload=_img(), payload_mime="image/jpeg",
                          meta={"prompt": "Hi", "max_new_tokens": "6"})
    out = list(vlm_service.Infer(iter([req]), None))
    assert out[-1].is_final and all(not r.is_final for r in out[:-1])
    d = json.loads(out[-1].result)
    assert d["generated_tokens"] == 6 and out[-1].meta["streaming_chunks"] == str(len(out) - 1)
    assert "processing_time_ms" in out[-1].meta
    for k in ("t_tokenize_ms", "t_decode_ms", "t_prefill_ms", "t_decode_tokens_ms"):
        assert float(out[-1].meta[k]) >= 0.0, (k, dict(out[-1].meta))
    cap = vlm_service.build_capability()
    assert cap.service_name == "vlm-fast" and {t.name for t in cap.tasks} == {"vlm_generate", "vlm_generate_stream"}


def test_chunked_prefill_matches_single_shot():
    """Prompts longer than the prefill chunk (64 tokens here, crossing KV block
    boundaries) are prefilled chunk by chunk, interleaved with other streams' decode
    steps, and generate exactly the tokens of a single-shot prefill."""
    cfg = LLM_PRESETS["tiny"]
    m = LLM(cfg, dtype=torch.float32, device="cpu")
    m.random_init(5)
    prompts = [list(np.random.default_rng(10 + i).integers(0, cfg.vocab_size, n)) for i, n in enumerate((150, 30, 200))]
    outs = {}
    for chunk in (4096, 64):
        kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=64, dtype=torch.float32)
        eng = LLMEngine(m, kv, lambda ids: m.embed_tokens(torch.tensor(ids)), max_batch=8, prefill_chunk=chunk)
        try:
            rs = [eng.submit(p, len(p), SamplingParams(max_new_tokens=10)) for p in prompts]
            for r in rs:
                list(r.stream(timeout=120))
            outs[chunk] = [r.tokens for r in rs]
            if chunk == 64:
                assert eng.stats["prefill_chunks"] >= 3 + 1 + 4
        finally:
            eng.close()
    assert outs[64] == outs[4096]
