"""Tensor-parallel VLM decode on MI355X: TP=2 (two ranks sharing the box's one GPU, gloo for the
control collectives, the IPC one-shot all-reduce inside the decode graphs) with hipGraph-captured
decode steps generates the same greedy text as TP=1.  Decode steps travel as int32 descriptors
over the host shared-memory step bus; the greedy sampler (vocab-parallel top-k merge through one
in-graph all-reduce) runs inside the graph, so the follower makes ZERO device->host copies per
decode step and the leader runs look-ahead steps under TP.  CPU twin:
test_parallel_cpu.py::test_vlm_tensor_parallel_*."""
import multiprocessing as mp
import os

import pytest

pytestmark = pytest.mark.gpu


def _leader(cache, tp, q, model="fastvlm-tiny"):
    import json as _json

    os.environ["LUMEN_TP_SIZE"] = str(tp)
    os.environ["LUMEN_TP_FOLLOWER_STATS"] = os.path.join(cache, "follower_stats")
    os.environ["LUMEN_DIST_BACKEND"] = "gloo"          # RCCL refuses two ranks on one device
    from lumen_amd.resources.validator import config_from_dict
    from lumen_amd.services.vlm import GeneralFastVLMService
    from lumen_amd.utils.image import encode_jpeg
    import numpy as np

    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": cache},
           "deployment": {"mode": "single", "service": "vlm"}, "server": {"port": 50558, "host": "127.0.0.1"},
           "services": {"vlm": {"enabled": True, "package": "lumen_vlm",
                                "import_info": {"registry_class": "lumen_vlm.fastvlm.GeneralFastVLMService",
                                                "add_to_server": "lumen_vlm.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                                "backend_settings": {"device": "cuda"},
                                "models": {"general": {"model": model, "runtime": "onnx"}}}}}
    s = GeneralFastVLMService.from_config(config_from_dict(cfg).services["vlm"], cache)
    s.initialize()
    try:
        img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (40, 60, 3), dtype=np.uint8))
        outs = []
        for prompt in ("Describe.", "What is this?"):
            body, _, _ = s.handle("vlm_generate", img, "image/jpeg", {"prompt": prompt, "max_new_tokens": "12"})
            outs.append(_json.loads(body)["text"])
        eng = s.backend.engine
        q.put({"texts": outs, "tp": s.backend.tp.world, "graphs": eng.graphs is not None and len(eng.graphs.graphs) > 0,
               "sync": dict(eng.sync.stats, transport=eng.sync.transport) if eng.sync is not None else None,
               "lookahead": eng.stats.get("lookahead_steps", 0)})
    except BaseException as e:  # noqa: BLE001
        q.put({"error": repr(e)})
    finally:
        s.close()


def test_vlm_tp2_graphs_match_tp1(tmp_path):
    from lumen_amd.models.vlm import write_vlm_model

    write_vlm_model(tmp_path / "models" / "fastvlm-tiny", "fastvlm-tiny")
    ctx = mp.get_context("spawn")
    res = {}
    for tp in (1, 2):
        q = ctx.Queue()
        p = ctx.Process(target=_leader, args=(str(tmp_path), tp, q))
        p.start()
        res[tp] = q.get(timeout=110)
        p.join(30)
        assert "error" not in res[tp], res[tp]
        assert p.exitcode == 0
    assert res[2]["tp"] == 2 and res[1]["tp"] == 1
    assert res[1]["graphs"] and res[2]["graphs"]                     # decode replayed from hipGraphs on both
    assert res[2]["sync"]["tensor_steps"] >= 10 and res[2]["sync"]["transport"] == "bus"
    assert res[2]["texts"] == res[1]["texts"]
    assert res[2]["lookahead"] > 0                                  # look-ahead steps under TP
    import json

    fol = json.loads((tmp_path / "follower_stats.rank1").read_text())
    assert fol["transport"] == "bus" and fol["decode_steps"] >= 10
    assert fol["ingraph_steps"] >= 10 and fol["lookahead_steps"] > 0
    # prefill's last chunk still gathers candidates through gloo (one host copy per request);
    # decode steps add none
    assert fol["d2h"] <= fol["prefill_chunks"]


def test_vlm_tp4_gqa_graphs_match_tp1(tmp_path):
    """TP = 4 on one GPU (4 ranks, gloo control + the IPC all-reduce with 3 peers, one- and two-shot):
    8 query heads over 2 KV heads, so every KV head is replicated on 2 ranks (the kv_rep > 1 load
    path); the step bus has 3 readers and the in-graph sampler merges 4 vocab shards.  Same greedy
    text as TP = 1."""
    from lumen_amd.models.vlm import write_vlm_model

    write_vlm_model(tmp_path / "models" / "vlm-gqa8", "vlm-gqa8", preset="tiny-gqa8")
    ctx = mp.get_context("spawn")
    res = {}
    for tp in (1, 4):
        q = ctx.Queue()
        p = ctx.Process(target=_leader, args=(str(tmp_path), tp, q, "vlm-gqa8"))
        p.start()
        res[tp] = q.get(timeout=110)
        p.join(30)
        assert "error" not in res[tp], res[tp]
        assert p.exitcode == 0
    assert res[4]["tp"] == 4 and res[4]["graphs"]
    assert res[4]["sync"]["transport"] == "bus" and res[4]["sync"]["tensor_steps"] >= 10
    # greedy text of a random-init tiny decoder: near-tied bf16 logits may flip a late token under
    # a different reduction order (TP = 4 sums 4 partial o / down products): the texts agree on
    # their first 8 characters and differ in length by at most one token's worth
    for a, b in zip(res[4]["texts"], res[1]["texts"]):
        assert a[:8] == b[:8] and abs(len(a) - len(b)) <= 4, (a, b)
    import json

    for r in (1, 2, 3):
        fol = json.loads((tmp_path / f"follower_stats.rank{r}").read_text())
        assert fol["transport"] == "bus" and fol["ingraph_steps"] >= 10


def _tf_rank(rank, world, port, cfg, T, steps, f8, q):
    """One TP rank on the shared GPU: teacher-forced logits (overlapped prefill + decode steps)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from lumen_amd.models.llm import LLM, TPInfo
    from lumen_amd.parallel.comm import Communicator
    from test_tp_overlap_cpu import hf_state_dict, teacher_forced_logits

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = LLM(cfg, TPInfo(rank, world, None), dtype=torch.bfloat16, device=dev)
        m.load_hf_state_dict(hf_state_dict(cfg, seed=5))
        if f8:
            m.quantize_fp8()
        m.comm = Communicator(None, dev, ipc=True)
        ids = torch.randint(3, cfg.vocab_size, (T + steps,), generator=torch.Generator().manual_seed(9))

        def gather(t):                       # the vocab shards, over gloo (host copies)
            t = t.cpu().contiguous()
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            return torch.cat(parts, dim=-1)

        out = teacher_forced_logits(m, ids, T, steps, dev, torch.bfloat16, gather)
        torch.cuda.synchronize()
        q.put({"rank": rank, "logits": [o.numpy() for o in out], "ipc": m.comm.stats["ipc_calls"],
               "err": m.comm.custom.error()})
        dist.barrier()
        m.comm.close()
    except BaseException as e:  # noqa: BLE001
        q.put({"rank": rank, "error": repr(e)})
    finally:
        dist.destroy_process_group()


F8_CFG = dict(vocab_size=1024, hidden_size=1024, num_layers=2, num_heads=8, num_kv_heads=4, head_dim=128,
              intermediate_size=2048, max_position=2048, tie_word_embeddings=False, qkv_bias=False)


@pytest.mark.parametrize("world,preset,f8", [(4, "tiny-gqa8", False), (2, "tiny-h8", False), (4, "f8", True)])
def test_tp_teacher_forced_logits_match_tp1(world, preset, f8):
    """TP = 2 / 4 ranks sharing the GPU (IPC one- / two-shot all-reduce, the overlapped prefill's
    communication stream): a 300-token prefill + 4 teacher-forced decode steps give per-step
    full-vocab logits with cosine >= 0.999 (bf16; W8A8 fp8 >= 0.995: the row-parallel shards quantise
    their weight rows over fewer columns) against TP = 1 on the same GPU and weights -- a reduction-order
    or shard bug that moves any step's logits fails here, not only one that changes a greedy token."""
    import numpy as np
    import torch

    from lumen_amd.models.llm import LLM, LLM_PRESETS, LLMConfig
    from test_tp_overlap_cpu import _port, hf_state_dict, teacher_forced_logits

    cfg = LLMConfig(**F8_CFG) if preset == "f8" else LLM_PRESETS[preset]
    T, steps = 300, 4
    ref_m = LLM(cfg, dtype=torch.bfloat16, device="cuda")
    ref_m.load_hf_state_dict(hf_state_dict(cfg, seed=5))
    if f8:
        ref_m.quantize_fp8()
    ids = torch.randint(3, cfg.vocab_size, (T + steps,), generator=torch.Generator().manual_seed(9))
    ref = teacher_forced_logits(ref_m, ids, T, steps, "cuda", torch.bfloat16)
    del ref_m
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tf_rank, args=(r, world, port, cfg, T, steps, f8, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=110) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(30)
    bound = 0.995 if f8 else 0.999
    for r in out:
        assert "error" not in r, r
        assert r["ipc"] > 0 and not r["err"]
        for k, (a, b) in enumerate(zip(r["logits"], ref)):
            a = torch.from_numpy(np.asarray(a))
            cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
            assert cos >= bound, (world, preset, k, cos)


def _tp_tower_rank(rank, world, port, fp8, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import lumen_amd.models.vlm as vlm_mod
    from lumen_amd.models.clip import VisionConfig
    from lumen_amd.models.llm import LLM_PRESETS, TPInfo
    from lumen_amd.models.vlm import VLM, VLMConfig
    from lumen_amd.parallel.comm import Communicator

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = VLMConfig(vision=VisionConfig(image_size=224, patch_size=14, width=256, layers=3, heads=4, act="gelu"),
                        llm=LLM_PRESETS["tiny-h8"], image_token_id=259)
        m = VLM(cfg, TPInfo(rank, world, dist.group.WORLD), device=dev)
        m.random_init(0)
        if fp8:
            m.quantize_fp8()
        m.llm.comm = Communicator(None, dev, ipc=True)
        g = torch.Generator().manual_seed(5)
        img = torch.randint(0, 256, (180, 240, 3), generator=g, dtype=torch.uint8).to(dev)
        it = cfg.image_token_id
        ids = [1, 2, it, 5, 6]
        mine = [img] if rank == 0 else []
        vlm_mod.TP_TOWER = False
        ref = m.build_prefill(ids, mine, n_images=1).float()
        vlm_mod.TP_TOWER = True
        got = m.build_prefill(ids, mine, n_images=1).float()
        torch.cuda.synchronize()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
        q.put({"rank": rank, "ok": m.tp_tower_ok(), "cos": cos, "sig": float(got.double().sum())})
        dist.barrier()
        m.llm.comm.close()
    except BaseException as e:  # noqa: BLE001
        q.put({"rank": rank, "error": repr(e)})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fp8", [False, True])
def test_vlm_tp_tower_gpu_matches_rank0_tower(fp8):
    """The tensor-parallel image tower at TP = 2 on the shared GPU (bf16 LN-folded blocks, or the MX
    W8A8 chain on the shards with fp8) equals the rank-0 tower + broadcast, with identical prefill
    inputs on both ranks."""
    from test_tp_overlap_cpu import _port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tp_tower_rank, args=(r, 2, port, fp8, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=110) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(30)
    for r in out:
        assert "error" not in r, r
        assert r["ok"] and r["cos"] > (0.995 if fp8 else 0.9995), r
    assert out[0]["sig"] == out[1]["sig"]
