"""lumen-vlm equivalent: LLaVA-family VLM (ViT -> projector -> Qwen2/Llama) on MI355X."""
from .backend import (ChatMessage, GenerationChunk, GenerationConfig, GenerationRequest, GenerationResult,
                      KVCacheConfig, MI355XVLMBackend, create_backend)
from .service import FastVLMModelManager, GeneralFastVLMService

__all__ = ["ChatMessage", "GenerationChunk", "GenerationConfig", "GenerationRequest", "GenerationResult",
           "KVCacheConfig", "MI355XVLMBackend", "create_backend", "FastVLMModelManager", "GeneralFastVLMService"]
