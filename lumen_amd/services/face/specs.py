"""Static InsightFace pack specifications (reference
packages/lumen-face/src/lumen_face/backends/insightface_specs.py:11-159).

Per pack: detector (SCRFD, 640x640 letterbox, mean 127.5 / std 128, strides 8/16/32,
2 anchors, output index map score 0-2 / bbox 3-5 / kps 6-8, default thresholds) and
recogniser (112x112, mean / std 127.5, RGB, 5-point alignment, 512-d).  The MI355X
detector emits the three strides' heads fused into one NHWC map per stride, so the
output index map documents the ONNX packs' layout only.  Specs are merged with
``model_info.extra_metadata.insightface`` overrides (the model_info wins).
"""
from __future__ import annotations

import copy

_DET = {"type": "scrfd", "input_size": (640, 640), "mean": (127.5, 127.5, 127.5), "std": (128.0, 128.0, 128.0),
        "letterbox": True, "normalized_boxes": False, "strides": [8, 16, 32], "num_anchors": 2,
        "outputs": [{"stride": 8, "score": 0, "bbox": 3, "kps": 6}, {"stride": 16, "score": 1, "bbox": 4, "kps": 7},
                    {"stride": 32, "score": 2, "bbox": 5, "kps": 8}],
        "score_threshold": 0.4, "nms_threshold": 0.4, "min_face": 32, "max_face": 1000}
_REC = {"input_size": (112, 112), "mean": (127.5, 127.5, 127.5), "std": (127.5, 127.5, 127.5), "channels_last": False,
        "color_order": "rgb", "align_landmarks": True, "embedding_dim": 512}

# detector / recogniser architecture presets of lumen_amd.models.face per pack
ARCH = {"antelopev2": ("10g", "r100"), "buffalo_l": ("10g", "r50"), "buffalo_m": ("10g", "r50"),
        "buffalo_s": ("10g", "r18"), "buffalo_sc": ("10g", "r18")}

PACK_SPECS = {name: {"detection": copy.deepcopy(_DET), "recognition": copy.deepcopy(_REC)} for name in ARCH}


def pack_spec(name: str, overrides: dict | None = None) -> dict:
    """Spec for a pack name (unknown names get the buffalo_l spec) merged with overrides."""
    key = next((k for k in PACK_SPECS if k in name.lower()), "buffalo_l")
    spec = copy.deepcopy(PACK_SPECS[key])
    for part in ("detection", "recognition"):
        spec[part].update((overrides or {}).get(part, {}) or {})
    return spec


def arch_for(name: str) -> tuple[str, str]:
    n = name.lower()
    if "tiny" in n:
        return "tiny", "tiny"
    return next((v for k, v in ARCH.items() if k in n), ("10g", "r50"))
