"""Tensor-parallel prefill with the row-parallel all-reduces overlapped (models/llm.py
LLM._layers_tp_overlap: two row halves, each half's o / down all-reduce on the communication stream
while the other half computes) at TP = 2 / 4 / 8 over gloo, one process per rank.

Teacher-forced numerics: a 300-token prefill (above the overlap threshold) plus 4 decode steps fed the
same tokens give per-step full-vocab logits (the ranks' vocab shards all-gathered) with cosine >= 0.999
against TP = 1 on the same weights and the same arg-max, and the overlapped prefill matches the plain
TP prefill of the same ranks.  GPU twin (two-stream overlap on one device): tests/test_tp_gpu.py.
SURVEY §5.8; reference prefill /root/reference/packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:161-234."""
import multiprocessing as mp
import os
import socket

import pytest
import torch


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def hf_state_dict(cfg, seed: int = 0) -> dict:
    """A full (unsharded) HF-layout Qwen2 / Llama state dict with deterministic random weights."""
    g = torch.Generator().manual_seed(seed)
    Hd, D, I, L = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.num_layers

    def r(*shape, std=0.05):
        return torch.randn(*shape, generator=g) * std

    sd = {"model.embed_tokens.weight": r(cfg.vocab_size, Hd, std=0.5), "lm_head.weight": r(cfg.vocab_size, Hd),
          "model.norm.weight": 1 + r(Hd, std=0.1)}
    for i in range(L):
        p = f"model.layers.{i}."
        sd[p + "self_attn.q_proj.weight"] = r(cfg.num_heads * D, Hd, std=Hd ** -0.5)
        sd[p + "self_attn.k_proj.weight"] = r(cfg.num_kv_heads * D, Hd, std=Hd ** -0.5)
        sd[p + "self_attn.v_proj.weight"] = r(cfg.num_kv_heads * D, Hd, std=Hd ** -0.5)
        if cfg.qkv_bias:
            sd[p + "self_attn.q_proj.bias"] = r(cfg.num_heads * D, std=0.02)
            sd[p + "self_attn.k_proj.bias"] = r(cfg.num_kv_heads * D, std=0.02)
            sd[p + "self_attn.v_proj.bias"] = r(cfg.num_kv_heads * D, std=0.02)
        sd[p + "self_attn.o_proj.weight"] = r(Hd, cfg.num_heads * D, std=(cfg.num_heads * D) ** -0.5)
        sd[p + "mlp.gate_proj.weight"] = r(I, Hd, std=Hd ** -0.5)
        sd[p + "mlp.up_proj.weight"] = r(I, Hd, std=Hd ** -0.5)
        sd[p + "mlp.down_proj.weight"] = r(Hd, I, std=I ** -0.5)
        sd[p + "input_layernorm.weight"] = 1 + r(Hd, std=0.1)
        sd[p + "post_attention_layernorm.weight"] = 1 + r(Hd, std=0.1)
    return sd


def teacher_forced_logits(m, ids: torch.Tensor, T: int, steps: int, dev, dtype, gather=None) -> list:
    """Prefill ids[:T], then decode ids[T:T+steps] one at a time; per step the full-vocab fp32 logits
    (``gather``: all-gathers the ranks' vocab shards)."""
    from lumen_amd.runtime.kv_cache import PagedKVCache

    cfg = m.cfg
    kv = PagedKVCache(cfg.num_layers, m.Hkv, cfg.head_dim, num_blocks=16, device=dev, dtype=dtype)
    kv.blocks.reserve(1, T + steps)
    out = [m.prefill(m.embed_tokens(ids[:T].to(dev)), kv, torch.from_numpy(kv.slots(1, 0, T)).to(dev))]
    bt = torch.from_numpy(kv.block_table([1])).to(dev)
    for p in range(T, T + steps):
        out.append(m.decode(ids[p:p + 1].to(dev), torch.tensor([p], dtype=torch.int32, device=dev),
                            torch.from_numpy(kv.slots(1, p, 1)).to(dev), kv, bt,
                            torch.tensor([p + 1], dtype=torch.int32, device=dev)))
    out = [o.float() for o in out]
    if gather is not None:
        out = [gather(o) for o in out]
    return [o.cpu() for o in out]


def _rank(rank, world, port, preset, T, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import lumen_amd.models.llm as llm_mod
    from lumen_amd.models.llm import LLM, LLM_PRESETS, TPInfo

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = LLM_PRESETS[preset]
        sd = hf_state_dict(cfg, seed=3)
        m = LLM(cfg, TPInfo(rank, world, None), dtype=torch.float32, device="cpu")
        m.load_hf_state_dict(sd)
        ids = torch.randint(3, cfg.vocab_size, (T + steps,), generator=torch.Generator().manual_seed(7))

        def gather(t):
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t.contiguous())
            return torch.cat(parts, dim=-1)

        calls = {"n": 0}
        orig = m._layers_tp_overlap

        def counted(*a, **k):
            calls["n"] += 1
            return orig(*a, **k)

        m._layers_tp_overlap = counted
        over = teacher_forced_logits(m, ids, T, steps, "cpu", torch.float32, gather)
        llm_mod._TP_OVERLAP_MIN_ROWS = 1 << 30            # the plain TP path, same ranks
        plain = teacher_forced_logits(m, ids, T, steps, "cpu", torch.float32, gather)
        # numpy: tensors would travel as shared-memory handles that die with this process
        q.put({"rank": rank, "over": [t.numpy() for t in over], "plain": [t.numpy() for t in plain],
               "overlap_calls": calls["n"]})
    except BaseException as e:  # noqa: BLE001
        q.put({"rank": rank, "error": repr(e)})
    finally:
        dist.destroy_process_group()


def _cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


@pytest.mark.parametrize("world,preset", [(2, "tiny-h8"), (4, "tiny-gqa8"), (8, "tiny-h8")])
def test_tp_overlapped_prefill_teacher_forced_matches_tp1(world, preset):
    from lumen_amd.models.llm import LLM, LLM_PRESETS

    T, steps = 300, 4
    cfg = LLM_PRESETS[preset]
    ref_m = LLM(cfg, dtype=torch.float32, device="cpu")
    ref_m.load_hf_state_dict(hf_state_dict(cfg, seed=3))
    ids = torch.randint(3, cfg.vocab_size, (T + steps,), generator=torch.Generator().manual_seed(7))
    ref = teacher_forced_logits(ref_m, ids, T, steps, "cpu", torch.float32)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, preset, T, steps, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=600) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(60)
    for r in out:
        assert "error" not in r, r
        r["over"] = [torch.from_numpy(a) for a in r["over"]]
        r["plain"] = [torch.from_numpy(a) for a in r["plain"]]
        assert r["overlap_calls"] == 1                    # the 300-row prefill took the overlapped path
        for k, (a, b, c) in enumerate(zip(r["over"], r["plain"], ref)):
            assert a.shape == c.shape == (1, cfg.vocab_size)
            assert _cos(a, c) >= 0.999, (world, k, _cos(a, c))
            assert int(a.argmax()) == int(c.argmax()), (world, k)
            assert _cos(a, b) >= 0.99999, (world, k)
    for r in out[1:]:
        for a, b in zip(r["over"], out[0]["over"]):
            assert torch.equal(a, b)                      # every rank holds the same gathered logits
