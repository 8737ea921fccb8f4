"""Dotted-path class loader for ``import_info.registry_class`` (reference src/lumen/loader.py:9-45).

Reference configs name the reference packages (``lumen_clip.general_clip.clip_service.
GeneralCLIPService`` ...).  Those dotted paths resolve to the MI355X implementations
through :data:`ALIASES`, so unmodified reference configs run here.
"""
from __future__ import annotations

import importlib

ALIASES = {
    # CLIP family
    "lumen_clip.general_clip.clip_service.GeneralCLIPService": "lumen_amd.services.clip.service.GeneralCLIPService",
    "lumen_clip.general_clip.GeneralCLIPService": "lumen_amd.services.clip.service.GeneralCLIPService",
    "lumen_clip.expert_bioclip.bioclip_service.BioCLIPService": "lumen_amd.services.clip.service.BioCLIPService",
    "lumen_clip.expert_bioclip.BioCLIPService": "lumen_amd.services.clip.service.BioCLIPService",
    "lumen_clip.unified_smartclip.smartclip_service.SmartCLIPService":
        "lumen_amd.services.clip.service.SmartCLIPService",
    "lumen_clip.unified_smartclip.SmartCLIPService": "lumen_amd.services.clip.service.SmartCLIPService",
    # face
    "lumen_face.general_face.face_service.GeneralFaceService": "lumen_amd.services.face.service.GeneralFaceService",
    "lumen_face.general_face.GeneralFaceService": "lumen_amd.services.face.service.GeneralFaceService",
    # OCR
    "lumen_ocr.general_ocr.ocr_service.GeneralOcrService": "lumen_amd.services.ocr.service.GeneralOcrService",
    "lumen_ocr.general_ocr.GeneralOcrService": "lumen_amd.services.ocr.service.GeneralOcrService",
    # VLM
    "lumen_vlm.fastvlm.fastvlm_service.GeneralFastVLMService": "lumen_amd.services.vlm.service.GeneralFastVLMService",
    "lumen_vlm.fastvlm.GeneralFastVLMService": "lumen_amd.services.vlm.service.GeneralFastVLMService",
}

ADD_TO_SERVER = "lumen_amd.proto.ml_service.add_InferenceServicer_to_server"


def resolve_path(dotted: str) -> str:
    if dotted in ALIASES:
        return ALIASES[dotted]
    if dotted.endswith("add_InferenceServicer_to_server"):
        return ADD_TO_SERVER
    return dotted


class ServiceLoader:
    @staticmethod
    def get_class(dotted: str):
        path = resolve_path(dotted)
        mod_name, _, attr = path.rpartition(".")
        if not mod_name:
            raise ImportError(f"invalid dotted path: {dotted}")
        try:
            mod = importlib.import_module(mod_name)
        except ImportError as e:
            raise ImportError(f"cannot import module {mod_name} for {dotted}: {e}") from e
        try:
            return getattr(mod, attr)
        except AttributeError as e:
            raise ImportError(f"{mod_name} has no attribute {attr}") from e
