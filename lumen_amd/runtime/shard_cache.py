"""Pre-sharded weight cache for tensor-parallel (and fp8) VLM serving.

The reference loads one ONNX decoder per process and has no tensor parallelism
(packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:55-160).  Here every TP rank
would otherwise read the whole checkpoint (16 GB for Llama-3-8B), slice its Megatron shard
and, for ``precision: fp8``, requantise its projections on every start.  After the first
build each rank writes exactly the tensors it holds -- sharded, interleaved (gate|up) and
quantised (fp8 weights + per-row scales) -- to one safetensors file per (tp world, rank,
precision); later starts load only that file straight onto the device (1/TP of the bytes,
no requantisation).

Layout: ``<model_root>/.lumen_shards/tp<W>_r<R>_<precision>.safetensors``.  The file's
metadata records a fingerprint of the source weights (file names, sizes, mtimes), the
model config and a format version; any mismatch ignores the cache and rebuilds it.  The
cache is written before the first forward pass (RMSNorm folding happens later, at first
GPU use, so cached weights are always in checkpoint form).  ``LUMEN_SHARD_CACHE=0``
disables it.
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
from pathlib import Path
from typing import Optional

import torch

log = logging.getLogger("lumen.shard_cache")

FORMAT = 1
_SOURCE_SUFFIXES = (".safetensors", ".onnx", ".onnx_data", ".bin", ".json")


def enabled() -> bool:
    return os.environ.get("LUMEN_SHARD_CACHE", "1") != "0"


def source_fingerprint(model_root: Path) -> str:
    """Names, sizes and mtimes of the weight / config files directly under the model dir
    (and its onnx/ subdir) -- cheap to compute, changes whenever a file is replaced."""
    h = hashlib.sha256()
    root = Path(model_root)
    files = []
    for d in (root, root / "onnx"):
        if d.is_dir():
            files += [p for p in d.iterdir() if p.is_file() and p.suffix in _SOURCE_SUFFIXES]
    for p in sorted(files):
        st = p.stat()
        h.update(f"{p.relative_to(root)}|{st.st_size}|{st.st_mtime_ns}\n".encode())
    return h.hexdigest()


def shard_path(model_root: Path, world: int, rank: int, precision: str) -> Path:
    prec = (precision or "bf16").lower().replace("/", "_")
    return Path(model_root) / ".lumen_shards" / f"tp{world}_r{rank}_{prec}.safetensors"


def _model_tensors(model: torch.nn.Module) -> dict[str, torch.Tensor]:
    """Every parameter and buffer this rank holds (fp8 scales are non-persistent buffers,
    so state_dict() alone would miss them)."""
    out = {}
    for name, p in model.named_parameters():
        out[name] = p.detach()
    for name, b in model.named_buffers():
        if name.endswith("cos_sin") or name.startswith("_"):
            continue                       # derived at construction
        out[name] = b.detach()
    return out


def save(model: torch.nn.Module, path: Path, fingerprint: str, config: dict, extra: Optional[dict] = None) -> bool:
    """Write this rank's tensors (best effort: a failure only logs)."""
    from safetensors.torch import save_file

    try:
        path.parent.mkdir(parents=True, exist_ok=True)
        tensors = {k: v.contiguous().cpu() for k, v in _model_tensors(model).items()}
        meta = {"format": str(FORMAT), "fingerprint": fingerprint, "config": json.dumps(config, sort_keys=True),
                "extra": json.dumps(extra or {}, sort_keys=True)}
        tmp = path.with_suffix(f".tmp{os.getpid()}")
        save_file(tensors, str(tmp), metadata=meta)
        os.replace(tmp, path)                # atomic: concurrent ranks / restarts never see half a file
        log.info("wrote weight shard %s (%.1f MB)", path, path.stat().st_size / 1e6)
        return True
    except Exception as e:  # noqa: BLE001 -- the cache is an optimisation
        log.warning("could not write weight shard %s: %s", path, e)
        return False


def read_meta(path: Path) -> Optional[dict]:
    from safetensors import safe_open

    if not path.is_file():
        return None
    try:
        with safe_open(str(path), "pt") as f:
            return dict(f.metadata() or {})
    except Exception:  # noqa: BLE001
        return None


def valid(path: Path, fingerprint: str, config: dict) -> bool:
    meta = read_meta(path)
    return bool(meta) and meta.get("format") == str(FORMAT) and meta.get("fingerprint") == fingerprint and \
        meta.get("config") == json.dumps(config, sort_keys=True)


def load(model: torch.nn.Module, path: Path, device) -> dict:
    """Load a shard written by :func:`save` into ``model`` (same architecture / TP layout):
    parameters are replaced by the stored tensors (dtype included: fp8 projections come back
    as float8_e4m3fn) and missing buffers (fp8 scales) are registered.  Returns the extra
    metadata."""
    from safetensors.torch import load_file

    sd = load_file(str(path), device=str(device))
    mods = dict(model.named_modules())
    for name, t in sd.items():
        mod_name, _, leaf = name.rpartition(".")
        mod = mods[mod_name] if mod_name else model
        cur = getattr(mod, leaf, None)
        if isinstance(cur, torch.nn.Parameter):
            if cur.dtype == t.dtype and cur.shape == t.shape:
                cur.data.copy_(t)
            else:
                setattr(mod, leaf, torch.nn.Parameter(t, requires_grad=False))
        elif leaf in getattr(mod, "_buffers", {}):
            mod._buffers[leaf] = t
        else:
            mod.register_buffer(leaf, t, persistent=False)
    meta = read_meta(path) or {}
    return json.loads(meta.get("extra", "{}"))
