"""CLIP resource loader: ``<cache_dir>/models/<model>/`` -> :class:`ModelResources`.

Same contract as packages/lumen-clip/src/lumen_clip/resources/loader.py:36-396:
manifest validation against the requested runtime, runtime directory
(``onnx/``, ``rknn/<device>/``, root for torch), model config
(``open_clip_config.json`` for OpenCLIP, ``config.json`` for HF; plus
``lumen_clip_config.json`` written by synthetic/random-init models), optional
``tokenizer.json``, dataset labels JSON (``np.array(dtype=object)``) and label
embeddings ``.npy`` memory-mapped read-only.
"""
from __future__ import annotations

import json
import logging
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Optional

import numpy as np

from ...models.clip import BertConfig, CLIPConfig, TextConfig, VisionConfig
from ...resources.config import ModelConfig, Runtime
from ...resources.exceptions import (DatasetNotFoundError, ModelInfoError, ResourceNotFoundError,
                                     RuntimeNotSupportedError)
from ...resources.model_info import ModelInfo, load_and_validate_model_info

log = logging.getLogger("lumen.clip.resources")

OPENAI_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_STD = (0.26862954, 0.26130258, 0.27577711)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


@dataclass
class ModelResources:
    model_root_path: Path
    runtime_files_path: Path
    model_name: str
    runtime: str
    model_info: ModelInfo
    config: dict
    tokenizer_path: Optional[Path] = None
    labels: Optional[np.ndarray] = None
    label_embeddings: Optional[np.ndarray] = None
    dataset: Optional[str] = None
    source_format: str = "custom"
    source_repo: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def model_id(self) -> str:
        return f"{self.model_name}_{self.runtime}"

    def has_classification_support(self) -> bool:
        return self.labels is not None and len(self.labels) > 0

    def get_embedding_dim(self) -> int:
        if self.model_info.embedding_dim:
            return int(self.model_info.embedding_dim)
        return int(self.clip_config().embed_dim)

    def get_image_size(self) -> int:
        c = self.config
        if "image_size" in c:
            s = c["image_size"]
            return int(s[0] if isinstance(s, (list, tuple)) else s)
        if "vision_cfg" in c and "image_size" in c["vision_cfg"]:
            s = c["vision_cfg"]["image_size"]
            return int(s[0] if isinstance(s, (list, tuple)) else s)
        if "vision" in c and "image_size" in c["vision"]:
            return int(c["vision"]["image_size"])
        if "vision_config" in c:
            return int(c["vision_config"].get("image_size", 224))
        return 224

    def get_normalization_stats(self) -> tuple[tuple, tuple]:
        c = self.config
        pp = c.get("preprocess_cfg") or {}
        if "mean" in pp and "std" in pp:
            return tuple(pp["mean"]), tuple(pp["std"])
        if "image_mean" in c and "image_std" in c:
            return tuple(c["image_mean"]), tuple(c["image_std"])
        return OPENAI_MEAN, OPENAI_STD

    def clip_config(self) -> CLIPConfig:
        """Architecture of the towers, from whichever config flavour is present."""
        c = self.config
        if "vision" in c and "text" in c:  # lumen_clip_config.json
            return CLIPConfig.from_dict(c)
        mean, std = self.get_normalization_stats()
        if "vision_cfg" in c and str(c["vision_cfg"].get("timm_model_name", "")).startswith("fastvit_"):
            return _mobileclip_config(c, mean, std)
        if "vision_cfg" in c:  # OpenCLIP
            v, t = c["vision_cfg"], c.get("text_cfg", {})
            width = int(v.get("width", 768))
            vc = VisionConfig(image_size=self.get_image_size(), patch_size=int(v.get("patch_size", 16)), width=width,
                              layers=int(v.get("layers", 12)), heads=int(v.get("heads", width // 64)),
                              mlp_ratio=float(v.get("mlp_ratio", 4.0)),
                              act="quick_gelu" if c.get("quick_gelu", False) else "gelu")
            tw = int(t.get("width", 512))
            tc = TextConfig(context_length=int(t.get("context_length", 77)), vocab_size=int(t.get("vocab_size", 49408)),
                            width=tw, layers=int(t.get("layers", 12)), heads=int(t.get("heads", tw // 64)),
                            act=vc.act)
            return CLIPConfig(embed_dim=int(c.get("embed_dim", 512)), vision=vc, text=tc, image_mean=tuple(mean),
                              image_std=tuple(std))
        if "vision_config" in c and (c.get("model_type") == "chinese_clip" or
                                     c.get("text_config", {}).get("model_type") == "chinese_clip_text_model"):
            return _chinese_clip_config(c, mean, std)
        if "vision_config" in c:  # HF CLIPConfig
            v, t = c["vision_config"], c.get("text_config", {})
            act = "quick_gelu" if v.get("hidden_act", "quick_gelu") == "quick_gelu" else "gelu"
            vc = VisionConfig(image_size=int(v.get("image_size", 224)), patch_size=int(v.get("patch_size", 32)),
                              width=int(v.get("hidden_size", 768)), layers=int(v.get("num_hidden_layers", 12)),
                              heads=int(v.get("num_attention_heads", 12)),
                              mlp_ratio=float(v.get("intermediate_size", 3072)) / float(v.get("hidden_size", 768)),
                              act=act, ln_eps=float(v.get("layer_norm_eps", 1e-5)))
            tc = TextConfig(context_length=int(t.get("max_position_embeddings", 77)),
                            vocab_size=int(t.get("vocab_size", 49408)), width=int(t.get("hidden_size", 512)),
                            layers=int(t.get("num_hidden_layers", 12)), heads=int(t.get("num_attention_heads", 8)),
                            mlp_ratio=float(t.get("intermediate_size", 2048)) / float(t.get("hidden_size", 512)),
                            act=act, eot_token_id=t.get("eos_token_id") if t.get("eos_token_id", 2) != 2 else None)
            return CLIPConfig(embed_dim=int(c.get("projection_dim", 512)), vision=vc, text=tc, image_mean=tuple(mean),
                              image_std=tuple(std))
        raise ModelInfoError(f"cannot infer CLIP architecture from config keys {list(c)}")


def _mobileclip_config(c: dict, mean, std) -> CLIPConfig:
    """open_clip MobileCLIP / MobileCLIP2 config: timm ``fastvit_mci*`` trunk + text transformer."""
    import dataclasses

    from ...models.fastvit import FASTVIT_PRESETS

    v, t = c["vision_cfg"], c.get("text_cfg", {})
    name = v["timm_model_name"][len("fastvit_"):]
    if name not in FASTVIT_PRESETS:
        raise ModelInfoError(f"unknown FastViT trunk {v['timm_model_name']}")
    fv = dataclasses.replace(FASTVIT_PRESETS[name], image_size=int(v.get("image_size", 256)))
    tw = int(t.get("width", 512))
    tc = TextConfig(context_length=int(t.get("context_length", 77)), vocab_size=int(t.get("vocab_size", 49408)),
                    width=tw, layers=int(t.get("layers", 12)), heads=int(t.get("heads", tw // 64)), act="gelu")
    return CLIPConfig(embed_dim=int(c.get("embed_dim", 512)), vision=VisionConfig(image_size=fv.image_size),
                      text=tc, image_mean=tuple(mean), image_std=tuple(std), vision_arch="fastvit", fastvit=fv)


def _chinese_clip_config(c: dict, mean, std) -> CLIPConfig:
    """HF ``ChineseCLIPConfig`` (OFA-Sys/chinese-clip-vit-*): ViT vision tower + BERT text tower."""
    v, t = c["vision_config"], c.get("text_config", {})
    vw = int(v.get("hidden_size", 768))
    vc = VisionConfig(image_size=int(v.get("image_size", 224)), patch_size=int(v.get("patch_size", 16)), width=vw,
                      layers=int(v.get("num_hidden_layers", 12)), heads=int(v.get("num_attention_heads", 12)),
                      mlp_ratio=float(v.get("intermediate_size", 4 * vw)) / vw,
                      act="quick_gelu" if v.get("hidden_act", "quick_gelu") == "quick_gelu" else "gelu",
                      ln_eps=float(v.get("layer_norm_eps", 1e-5)))
    bc = BertConfig(vocab_size=int(t.get("vocab_size", 21128)), width=int(t.get("hidden_size", 768)),
                    layers=int(t.get("num_hidden_layers", 12)), heads=int(t.get("num_attention_heads", 12)),
                    intermediate=int(t.get("intermediate_size", 3072)),
                    max_position=int(t.get("max_position_embeddings", 512)),
                    type_vocab=int(t.get("type_vocab_size", 2)), ln_eps=float(t.get("layer_norm_eps", 1e-12)),
                    context_length=int(c.get("context_length", t.get("context_length", 52))),
                    pad_token_id=int(t.get("pad_token_id", 0)))
    return CLIPConfig(embed_dim=int(c.get("projection_dim", 512)), vision=vc, image_mean=tuple(mean),
                      image_std=tuple(std), text_arch="bert", bert=bc)


def _load_json(p: Path) -> dict:
    try:
        return json.loads(p.read_text(encoding="utf-8"))
    except FileNotFoundError as e:
        raise ResourceNotFoundError(f"required file missing: {p}") from e
    except json.JSONDecodeError as e:
        raise ModelInfoError(f"invalid JSON {p}: {e}") from e


class ResourceLoader:
    @staticmethod
    def load_model_resources(cache_dir, model_config: ModelConfig) -> ModelResources:
        root = Path(cache_dir).expanduser().resolve() / "models" / model_config.model
        if not (root / "model_info.json").exists():
            raise ResourceNotFoundError(f"model_info.json not found in {root}")
        info = load_and_validate_model_info(root / "model_info.json")
        rt = model_config.runtime.value
        if rt not in info.runtimes or not info.runtimes[rt].available:
            raise RuntimeNotSupportedError(f"runtime '{rt}' not available for {info.name}")
        if model_config.runtime == Runtime.onnx:
            rdir = root / "onnx"
        elif model_config.runtime == Runtime.rknn:
            rdir = root / "rknn" / (model_config.rknn_device or "")
        else:
            rdir = root
        if not rdir.exists():
            rdir = root
        for name in ("lumen_clip_config.json", "open_clip_config.json", "config.json"):
            if (root / name).exists():
                config = _load_json(root / name)
                break
        else:
            raise ResourceNotFoundError(f"no CLIP config (open_clip_config.json / config.json) in {root}")
        tok = root / "tokenizer.json"
        labels, emb = ResourceLoader._load_dataset(root, info, model_config.dataset)
        return ModelResources(model_root_path=root, runtime_files_path=rdir, model_name=model_config.model,
                              runtime=rt, model_info=info, config=config,
                              tokenizer_path=tok if tok.exists() else None, labels=labels, label_embeddings=emb,
                              dataset=model_config.dataset, source_format=info.source.format.value,
                              source_repo=info.source.repo_id)

    @staticmethod
    def _load_dataset(root: Path, info: ModelInfo, dataset: Optional[str]):
        if not dataset:
            return None, None
        if not info.datasets or dataset not in info.datasets:
            raise DatasetNotFoundError(f"dataset '{dataset}' not declared in model_info.json")
        ds = info.datasets[dataset]
        lp, ep = root / ds.labels, root / ds.embeddings
        if not lp.exists():
            raise DatasetNotFoundError(f"labels file missing: {lp}")
        labels = np.array(json.loads(lp.read_text(encoding="utf-8")), dtype=object)
        emb = None
        if ep.exists():
            emb = np.load(ep, mmap_mode="r", allow_pickle=False)
        return labels, emb


def load_weights(root: Path, precision: Optional[str] = None) -> dict:
    """Model weights with loaders that execute nothing from the file: safetensors / torch
    ``weights_only`` checkpoints, else the reference's ONNX pack (``onnx/vision[.<prec>].onnx``
    + ``onnx/text[.<prec>].onnx``) whose initializers are mapped back to the exported
    model's parameter names (utils/onnx_import.py) -- the graphs themselves never run."""
    import torch

    for name in ("model.safetensors", "open_clip_model.safetensors"):
        if (root / name).exists():
            from safetensors.torch import load_file

            return load_file(str(root / name))
    for name in ("open_clip_pytorch_model.bin", "pytorch_model.bin", "model.pt"):
        if (root / name).exists():
            sd = torch.load(str(root / name), map_location="cpu", weights_only=True)
            return sd.get("state_dict", sd) if isinstance(sd, dict) else sd
    from ...utils import onnx_import

    odir = root / "onnx"
    vis = onnx_import.pick_file(odir, "vision", precision) if odir.is_dir() else None
    if vis is not None:
        txt = onnx_import.pick_file(odir, "text", precision)
        log.info("CLIP weights from ONNX pack: %s + %s", vis.name, txt.name if txt else "-")
        return onnx_import.clip_state_dict(vis, txt)
    raise ResourceNotFoundError(f"no weights (*.safetensors / *.bin / onnx/vision*.onnx) in {root}")
