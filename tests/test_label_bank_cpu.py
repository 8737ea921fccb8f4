"""Sharded label bank (K13, reference bioclip_model.py:286-330 classify path): shard
candidates merged on the host (serving worker pool) and over a gloo process group (SPMD
ranks) give the same top-k indices and scores / softmax probabilities as the unsharded bank;
BioCLIP under LUMEN_DP_SIZE=2 classifies through per-worker bank shards."""
import multiprocessing as mp
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch

from lumen_amd.runtime.label_bank import LabelBank, orient_bank

N, D, B = 103, 32, 5


def _bank(n=N, d=D, seed=0):
    rng = np.random.default_rng(seed)
    e = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((B, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return e, q


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("softmax", [False, True])
def test_merge_host_matches_unsharded(world, softmax):
    e, q = _bank()
    ref_v, ref_i = LabelBank(e, torch.device("cpu")).topk(q, 7, scale=30.0, softmax=softmax)
    parts = [LabelBank(e, torch.device("cpu"), shard=(r, world)).topk_local(q, 7, 30.0, softmax) for r in range(world)]
    assert sum(p[0].shape[1] for p in parts) >= 7
    v, i = LabelBank.merge_host(parts, 7, 30.0, softmax)
    np.testing.assert_array_equal(i, ref_i)
    np.testing.assert_allclose(v, ref_v, rtol=1e-5, atol=1e-6)
    if softmax:
        full = np.exp(30.0 * (q @ (e / np.linalg.norm(e, axis=1, keepdims=True)).T))
        full /= full.sum(1, keepdims=True)
        np.testing.assert_allclose(v, np.take_along_axis(full, ref_i, 1), rtol=1e-4)


def test_shard_slices_memmap_and_empty_shard(tmp_path):
    e, q = _bank(n=5)
    np.save(tmp_path / "b.npy", e)
    mm = np.load(tmp_path / "b.npy", mmap_mode="r")
    world = 4                                  # ceil(5/4)=2 rows per shard -> last shard empty
    shards = [LabelBank(mm, torch.device("cpu"), shard=(r, world)) for r in range(world)]
    assert [s.n_local for s in shards] == [2, 2, 1, 0] and [s.offset for s in shards] == [0, 2, 4, 5]
    parts = [s.topk_local(q, 3, 1.0, True) for s in shards]
    v, i = LabelBank.merge_host(parts, 3, 1.0, True)
    rv, ri = LabelBank(e, torch.device("cpu")).topk(q, 3, softmax=True)
    np.testing.assert_array_equal(i, ri)
    np.testing.assert_allclose(v, rv, rtol=1e-5)
    with pytest.raises(RuntimeError, match="topk_local"):
        shards[0].topk(q, 3)


def test_orient_bank():
    e = np.zeros((8, 20))
    assert orient_bank(e, 20, 8).shape == (20, 8)
    assert orient_bank(e, 8, 20).shape == (8, 20)
    assert orient_bank(e, 20, 16).shape == (8, 20)     # D mismatch -> left alone


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spmd_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e, qs = _bank()
        bank = LabelBank(e, torch.device("cpu"), group=dist.group.WORLD)
        out = {"rank": rank, "n_local": bank.n_local}
        for sm in (False, True):
            v, i = bank.topk(qs, 6, scale=20.0, softmax=sm)
            out[sm] = (v, i)
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_spmd_world2_gloo_matches_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_spmd_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    e, qs = _bank()
    assert [r["n_local"] for r in res] == [52, 51]
    for sm in (False, True):
        rv, ri = LabelBank(e, torch.device("cpu")).topk(qs, 6, scale=20.0, softmax=sm)
        for r in res:
            np.testing.assert_array_equal(r[sm][1], ri)
            np.testing.assert_allclose(r[sm][0], rv, rtol=1e-5, atol=1e-6)


def test_bioclip_dp2_sharded_bank_matches_single(tmp_path, monkeypatch):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.runtime.label_bank import PoolShardedBank
    from lumen_amd.services.clip.backend import create_backend
    from lumen_amd.services.clip.model import BioCLIPModelManager
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    write_clip_model(tmp_path / "models" / "bioclip-tiny", "bioclip-tiny", preset="tiny", dataset="TreeOfLife-10M",
                     n_labels=37)
    res = ResourceLoader.load_model_resources(tmp_path, ModelConfig(model="bioclip-tiny", runtime=Runtime.torch,
                                                                    dataset="TreeOfLife-10M"))
    assert res.label_embeddings is not None
    settings = type("S", (), {"device": "cpu", "batch_size": 4})()
    imgs = [encode_jpeg(np.random.default_rng(i).integers(0, 255, (36, 28 + i, 3), dtype=np.uint8)) for i in range(3)]
    single = BioCLIPModelManager(create_backend(settings, res, "torch"))
    single.initialize()
    try:
        ref = [single.classify_image(b, top_k=5) for b in imgs]
    finally:
        single.backend.close()
    monkeypatch.setenv("LUMEN_DP_SIZE", "2")
    dp = BioCLIPModelManager(create_backend(settings, res, "torch"))
    dp.initialize()
    try:
        assert isinstance(dp.bank, PoolShardedBank) and dp.backend._pool.size == 2
        for b, r in zip(imgs, ref):
            got = dp.classify_image(b, top_k=5)
            assert [g[0] for g in got] == [x[0] for x in r]
            np.testing.assert_allclose([g[1] for g in got], [x[1] for x in r], atol=1e-5)
    finally:
        dp.backend.close()


def _bank_worker(rank, world, port, argv, q):
    import os
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import build_label_bank

    from lumen_amd.parallel import destroy

    sys.argv = ["build_label_bank.py"] + argv
    try:
        q.put((rank, build_label_bank.main()))
    finally:
        destroy()


def test_label_bank_tool_data_parallel_matches_single(tmp_path):
    """tools/build_label_bank.py under 2 gloo ranks (parallel.DataParallelRunner shards the
    labels and all-gathers the rows) writes the same bank as the single-process run."""
    import json
    import socket
    import sys

    import torch.multiprocessing as mp

    from lumen_amd.resources.synthetic import write_clip_model

    write_clip_model(tmp_path / "models" / "clip-tiny", "clip-tiny", preset="tiny")
    labels = [f"label number {i}" for i in range(23)]
    (tmp_path / "labels.json").write_text(json.dumps(labels))
    argv = ["--cache", str(tmp_path), "--model", "clip-tiny", "--dataset", "Bank", "--labels",
            str(tmp_path / "labels.json"), "--device", "cpu", "--batch", "4"]
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import build_label_bank

    old = sys.argv
    sys.argv = ["build_label_bank.py"] + argv
    try:
        assert build_label_bank.main() == 0
    finally:
        sys.argv = old
    emb_path = tmp_path / "models" / "clip-tiny" / "datasets" / "Bank_embeddings.npy"
    single = np.load(emb_path)
    emb_path.unlink()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bank_worker, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in ps:
        p.start()
    rets = [q.get(timeout=240) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    assert sorted(rets) == [(0, 0), (1, 0)]
    dp = np.load(emb_path)
    assert dp.shape == single.shape == (23, single.shape[1])
    np.testing.assert_allclose(dp, single, atol=1e-5)
