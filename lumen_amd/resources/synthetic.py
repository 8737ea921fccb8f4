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
                             extra_special: Optional[list[str]] = None, add_bos_eos: bool = True,
                             fill_vocab: int = 0) -> dict:
    """A dependency-free byte-level BPE tokenizer.json (no merges): ids 0..255 = bytes,
    then the special tokens; EOS gets the largest id (CLIP's EOT-argmax pooling).
    ``fill_vocab``: pad the vocabulary with word tokens " w<k>" up to that many ids (after the
    specials), so a random-init decoder over a real-sized vocabulary (128,256 for Llama-3) produces
    readable text instead of ids the tokenizer does not know (service-level streaming benchmarks)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors

    b2u = _bytes_to_unicode()
    vocab = {b2u[b]: b for b in range(256)}
    specials = (extra_special or []) + [bos, eos]
    for s in specials:
        vocab[s] = len(vocab)
    sp = b2u[ord(" ")]
    k = 0
    while len(vocab) < fill_vocab:
        vocab[f"{sp}w{k}"] = len(vocab)
        k += 1
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens(specials)
    if add_bos_eos:
        tok.post_processor = processors.TemplateProcessing(
            single=f"{bos} $A {eos}", special_tokens=[(bos, vocab[bos]), (eos, vocab[eos])])
    tok.save(str(path))
    return {"vocab_size": len(vocab), "bos_id": vocab[bos], "eos_id": vocab[eos]}


def write_wordpiece_tokenizer(path: Path, vocab_size: int) -> dict:
    """A BERT-style WordPiece tokenizer.json for CN-CLIP (RoBERTa-wwm-ext-chinese layout):
    [PAD]=0, [UNK], [CLS], [SEP], [MASK], printable ASCII, then CJK ideographs one per id
    (BertNormalizer splits CJK characters individually, like the real vocab), filled up
    to ``vocab_size`` with ``##``-continuations."""
    from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors

    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + [chr(c) for c in range(33, 127)]
    cjk = 0x4E00
    while len(toks) < vocab_size and cjk <= 0x9FFF:
        toks.append(chr(cjk))
        cjk += 1
    i = 0
    while len(toks) < vocab_size:
        toks.append("##" + toks[5 + i % 94] + ("" if i < 94 else str(i // 94)))
        i += 1
    vocab = {t: j for j, t in enumerate(toks[:vocab_size])}
    tok = Tokenizer(models.WordPiece(vocab=vocab, unk_token="[UNK]"))
    tok.normalizer = normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=True, lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.post_processor = processors.BertProcessing(("[SEP]", vocab["[SEP]"]), ("[CLS]", vocab["[CLS]"]))
    tok.decoder = decoders.WordPiece()
    tok.add_special_tokens(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"])
    tok.save(str(path))
    return {"vocab_size": len(vocab), "cls_id": vocab["[CLS]"], "sep_id": vocab["[SEP]"], "pad_id": 0}


def _save_safetensors(sd: dict, path: Path) -> None:
    from safetensors.torch import save_file

    save_file({k: v.contiguous() for k, v in sd.items()}, str(path))


def _write_info(root: Path, info: dict) -> None:
    ModelInfo.model_validate(info)  # fail fast on schema drift
    (root / "model_info.json").write_text(json.dumps(info, indent=2), encoding="utf-8")


def clip_preset_for(name: str) -> str:
    n = name.lower()
    if "mobileclip" in n:
        return "mobileclip-tiny" if "tiny" in n else ("MobileCLIP2-S4" if "s4" in n else "MobileCLIP2-S2")
    if "cn-clip" in n or "chinese" in n:
        return "cn-tiny" if "tiny" in n else ("CN-ViT-B-16" if "b-16" in n or "b16" in n else "CN-ViT-L-14")
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
    if cfg.text_arch == "bert":
        return _write_cn_clip(root, name, preset, cfg, m, dataset, n_labels, seed)
    _save_safetensors({k: v.to(torch.bfloat16) if v.dim() > 0 else v for k, v in export_openclip_state_dict(m).items()},
                      root / "model.safetensors")
    (root / "lumen_clip_config.json").write_text(json.dumps(cfg.to_dict(), indent=2))
    vcfg = {"image_size": cfg.vision.image_size, "patch_size": cfg.vision.patch_size,
            "width": cfg.vision.width, "layers": cfg.vision.layers}
    if cfg.vision_arch == "fastvit":   # open_clip TimmModel tower
        from ..models.fastvit import FASTVIT_PRESETS

        tname = next((k for k, v in FASTVIT_PRESETS.items() if v == cfg.fastvit), "custom")
        vcfg = {"timm_model_name": f"fastvit_{tname}", "timm_pool": "avg", "timm_proj": None,
                "image_size": cfg.fastvit.image_size}
    oc = {"embed_dim": cfg.embed_dim,
          "vision_cfg": vcfg,
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
        "extra_metadata": {"synthetic": True, "arch": "clip", "preset": preset,
                           "image_size": cfg.fastvit.image_size if cfg.vision_arch == "fastvit" else cfg.vision.image_size,
                           "context_length": cfg.text.context_length},
    }
    _write_info(root, info)
    return root


def _write_cn_clip(root: Path, name: str, preset: str, cfg, m, dataset, n_labels: int, seed: int) -> Path:
    """CN-CLIP in HF ``ChineseCLIPModel`` layout: config.json (model_type chinese_clip),
    model.safetensors with ``vision_model.* / text_model.*`` names, WordPiece tokenizer.json."""
    from ..models.clip import export_chinese_clip_state_dict

    sd = export_chinese_clip_state_dict(m)
    _save_safetensors({k: v.to(torch.bfloat16) for k, v in sd.items()}, root / "model.safetensors")
    v, b = cfg.vision, cfg.bert
    hf = {"model_type": "chinese_clip", "projection_dim": cfg.embed_dim, "logit_scale_init_value": 2.6592,
          "context_length": b.context_length,
          "text_config": {"model_type": "chinese_clip_text_model", "vocab_size": b.vocab_size, "hidden_size": b.width,
                          "num_hidden_layers": b.layers, "num_attention_heads": b.heads,
                          "intermediate_size": b.intermediate, "max_position_embeddings": b.max_position,
                          "type_vocab_size": b.type_vocab, "layer_norm_eps": b.ln_eps, "pad_token_id": b.pad_token_id,
                          "hidden_act": "gelu"},
          "vision_config": {"model_type": "chinese_clip_vision_model", "image_size": v.image_size,
                            "patch_size": v.patch_size, "hidden_size": v.width, "num_hidden_layers": v.layers,
                            "num_attention_heads": v.heads, "intermediate_size": int(v.width * v.mlp_ratio),
                            "hidden_act": v.act, "layer_norm_eps": v.ln_eps},
          "image_mean": list(cfg.image_mean), "image_std": list(cfg.image_std)}
    (root / "config.json").write_text(json.dumps(hf, indent=2))
    write_wordpiece_tokenizer(root / "tokenizer.json", b.vocab_size)
    files = ["model.safetensors", "config.json", "tokenizer.json"]
    datasets = None
    if dataset:
        rng = np.random.default_rng(seed + 1)
        (root / "datasets").mkdir(exist_ok=True)
        emb = rng.standard_normal((n_labels, cfg.embed_dim)).astype(np.float32)
        emb /= np.linalg.norm(emb, axis=1, keepdims=True)
        lab_rel, emb_rel = f"datasets/{dataset}_labels.json", f"datasets/{dataset}_embeddings.npy"
        (root / lab_rel).write_text(json.dumps([f"类别 {i}" for i in range(n_labels)], ensure_ascii=False))
        np.save(root / emb_rel, emb)
        datasets = {dataset: {"labels": lab_rel, "embeddings": emb_rel}}
    info = {
        "name": name, "version": "1.0.0",
        "description": f"synthetic random-init {preset} Chinese-CLIP for MI355X tests",
        "model_type": "clip", "embedding_dim": cfg.embed_dim,
        "source": {"format": "huggingface", "repo_id": f"synthetic/{name}"},
        "runtimes": {"torch": {"available": True, "files": files, "devices": ["cuda", "cpu"]},
                     "onnx": {"available": True, "files": files, "devices": ["cuda", "cpu"]}},
        "datasets": datasets,
        "extra_metadata": {"synthetic": True, "arch": "chinese_clip", "preset": preset, "image_size": v.image_size,
                           "context_length": b.context_length},
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
