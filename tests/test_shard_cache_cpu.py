"""Pre-sharded TP / fp8 weight cache (runtime/shard_cache.py): a rank's tensors round-trip
exactly (fp8 weights + per-row scales included) and a changed source invalidates the file."""
import time

import torch

from lumen_amd.models.llm import TPInfo
from lumen_amd.models.vlm import VLM, VLM_PRESETS
from lumen_amd.runtime import shard_cache


def _model(rank, world, seed=0):
    m = VLM(VLM_PRESETS["tiny"], TPInfo(rank=rank, world=world), dtype=torch.float32, device="cpu")
    m.random_init(seed)
    return m


def test_shard_roundtrip_fp8_tp(tmp_path):
    (tmp_path / "model.safetensors").write_bytes(b"x" * 10)
    fp = shard_cache.source_fingerprint(tmp_path)
    cfg = VLM_PRESETS["tiny"].to_dict()
    for rank in range(2):
        src = _model(rank, 2, seed=3)
        src.llm.quantize_fp8()
        p = shard_cache.shard_path(tmp_path, 2, rank, "fp8")
        assert shard_cache.save(src, p, fp, cfg, {"weight_dtype": src.llm.weight_dtype})
        assert shard_cache.valid(p, fp, cfg)
        dst = _model(rank, 2, seed=9)
        extra = shard_cache.load(dst, p, "cpu")
        assert extra["weight_dtype"] == "fp8"
        a = shard_cache._model_tensors(src)
        b = shard_cache._model_tensors(dst)
        assert a.keys() == b.keys() and any(k.endswith("qkv_s") for k in a)
        for k in a:
            assert a[k].dtype == b[k].dtype and torch.equal(a[k].float(), b[k].float()), k
        assert dst.llm.layers[0].qkv_w.dtype == torch.float8_e4m3fn


def test_shard_invalidated_by_source_change(tmp_path):
    w = tmp_path / "model.safetensors"
    w.write_bytes(b"x" * 10)
    cfg = VLM_PRESETS["tiny"].to_dict()
    fp = shard_cache.source_fingerprint(tmp_path)
    p = shard_cache.shard_path(tmp_path, 2, 1, "bf16")
    assert shard_cache.save(_model(1, 2), p, fp, cfg)
    time.sleep(0.01)
    w.write_bytes(b"y" * 11)
    assert not shard_cache.valid(p, shard_cache.source_fingerprint(tmp_path), cfg)
    other = dict(cfg)
    other["num_image_tokens"] = cfg.get("num_image_tokens", 0) + 1
    assert not shard_cache.valid(p, fp, other)
