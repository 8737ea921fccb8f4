"""Synthetic (random-init) model directories.

There is no network in the build/benchmark environment, so every model family
can be materialised as ``<cache_dir>/models/<name>/`` with a valid
``model_info.json``, random-init weights of the real architecture
(safetensors), a small byte-level BPE ``tokenizer.json`` where a tokenizer is
needed, and dataset label banks (labels JSON + L2-normalised ``.npy``
embeddings) laid out exactly like the reference's artefacts.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from .model_info import ModelInfo

SCENE_LABELS = ["animal", "bird", "food", "landscape", "person", "plant", "vehicle", "building"]


def _bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def write_byte_bpe_tokenizer(path: Path, bos: str = "<start_of_text>", eos: str = "<end_of_text>",
                             extra_special: Optional[list[str]] = None, add_bos_eos: bool = True) -> dict:
    """A dependency-free byte-level BPE tokenizer.json (no merges): ids 0..255 = bytes,
    then the special tokens; EOS gets the largest id (CLIP's EOT-argmax pooling)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors

    b2u = _bytes_to_unicode()
    vocab = {b2u[b]: b for b in range(256)}
    specials = (extra_special or []) + [bos, eos]
    for s in specials:
        vocab[s] = len(vocab)
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens(specials)
    if add_bos_eos:
        tok.post_processor = processors.TemplateProcessing(
            single=f"{bos} $A {eos}", special_tokens=[(bos, vocab[bos]), (eos, vocab[eos])])
    tok.save(str(path))
    return {"vocab_size": len(vocab), "bos_id": vocab[bos], "eos_id": vocab[eos]}


def _save_safetensors(sd: dict, path: Path) -> None:
    from safetensors.torch import save_file

    save_file({k: v.contiguous() for k, v in sd.items()}, str(path))


def _write_info(root: Path, info: dict) -> None:
    ModelInfo.model_validate(info)  # fail fast on schema drift
    (root / "model_info.json").write_text(json.dumps(info, indent=2), encoding="utf-8")


def clip_preset_for(name: str) -> str:
    n = name.lower()
    if "tiny" in n:
        return "tiny"
    if "b-32" in n or "b32" in n:
        return "ViT-B-32"
    if "b-16" in n or "b16" in n or "s2" in n:
        return "ViT-B-16"
    if "336" in n:
        return "ViT-L-14-336"
    return "ViT-L-14"


def write_clip_model(root: Path, name: str, preset: Optional[str] = None, dataset: Optional[str] = "ImageNet_1k",
                     n_labels: int = 1000, bio: bool = False, seed: int = 0) -> Path:
    from ..models.clip import CLIPModel, PRESETS, export_openclip_state_dict

    preset = preset or clip_preset_for(name)
    cfg = PRESETS[preset]
    root.mkdir(parents=True, exist_ok=True)
    m = CLIPModel.random(cfg, seed=seed, dtype=torch.float32)
    _save_safetensors({k: v.to(torch.bfloat16) if v.dim() > 0 else v for k, v in export_openclip_state_dict(m).items()},
                      root / "model.safetensors")
    (root / "lumen_clip_config.json").write_text(json.dumps(cfg.to_dict(), indent=2))
    oc = {"embed_dim": cfg.embed_dim,
          "vision_cfg": {"image_size": cfg.vision.image_size, "patch_size": cfg.vision.patch_size,
                         "width": cfg.vision.width, "layers": cfg.vision.layers},
          "text_cfg": {"context_length": cfg.text.context_length, "vocab_size": cfg.text.vocab_size,
                       "width": cfg.text.width, "heads": cfg.text.heads, "layers": cfg.text.layers},
          "preprocess_cfg": {"mean": list(cfg.image_mean), "std": list(cfg.image_std)}}
    (root / "open_clip_config.json").write_text(json.dumps(oc, indent=2))
    write_byte_bpe_tokenizer(root / "tokenizer.json")
    files = ["model.safetensors", "open_clip_config.json", "tokenizer.json"]
    datasets = None
    if dataset:
        rng = np.random.default_rng(seed + 1)
        ddir = root / "datasets"
        ddir.mkdir(exist_ok=True)
        if bio:
            labels = [[["Animalia", "Chordata", "Aves", f"Order{i % 17}", f"Family{i % 53}", f"Genus{i}", f"species{i}"],
                       f"common bird {i}" if i % 3 else ""] for i in range(n_labels)]
        else:
            labels = [f"class {i}" for i in range(n_labels)]
        emb = rng.standard_normal((n_labels, cfg.embed_dim)).astype(np.float32)
        emb /= np.linalg.norm(emb, axis=1, keepdims=True)
        lab_rel, emb_rel = f"datasets/{dataset}_labels.json", f"datasets/{dataset}_embeddings.npy"
        (root / lab_rel).write_text(json.dumps(labels))
        np.save(root / emb_rel, emb)
        datasets = {dataset: {"labels": lab_rel, "embeddings": emb_rel}}
    info = {
        "name": name, "version": "1.0.0",
        "description": f"synthetic random-init {preset} CLIP ({'BioCLIP' if bio else 'general'}) for MI355X tests",
        "model_type": "bioclip" if bio else "clip", "embedding_dim": cfg.embed_dim,
        "source": {"format": "custom", "repo_id": f"synthetic/{name}"},
        "runtimes": {"torch": {"available": True, "files": files, "devices": ["cuda", "cpu"]},
                     "onnx": {"available": True, "files": files, "devices": ["cuda", "cpu"]}},
        "datasets": datasets,
        "extra_metadata": {"synthetic": True, "arch": "clip", "preset": preset, "image_size": cfg.vision.image_size,
                           "context_length": cfg.text.context_length},
    }
    _write_info(root, info)
    return root


def write_synthetic_model(cache_dir: Path, name: str, service: str = "", dataset: Optional[str] = None) -> Path:
    """Dispatch on the service / model name to the right family writer."""
    root = Path(cache_dir) / "models" / name
    kind = (service + " " + name).lower()
    if "face" in kind or "buffalo" in kind or "antelope" in kind:
        from ..models.face import write_face_model

        return write_face_model(root, name)
    if "ocr" in kind:
        from ..models.ocr import write_ocr_model

        return write_ocr_model(root, name)
    if "vlm" in kind or "fastvlm" in kind:
        from ..models.vlm import write_vlm_model

        return write_vlm_model(root, name)
    bio = "bio" in kind
    return write_clip_model(root, name, dataset=dataset or ("TreeOfLife-10M" if bio else None), bio=bio,
                            n_labels=2000 if bio else 1000)
