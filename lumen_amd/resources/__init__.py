"""lumen-resources equivalent: configuration, manifests, result schemas, downloader."""
from .config import AmdRuntimeSettings, BackendSettings, LumenConfig, ModelConfig, Region, Runtime, Services  # noqa
from .downloader import Downloader, DownloadResult  # noqa: F401
from .exceptions import (ConfigError, DownloadError, ModelInfoError, PlatformUnavailableError,  # noqa: F401
                         ResourceError, ValidationError)
from .model_info import Metadata, ModelInfo, Runtimes, Source, load_and_validate_model_info  # noqa: F401
from .schemas import OCRV1, EmbeddingV1, FaceV1, LabelsV1, TextGenerationV1  # noqa: F401
from .validator import load_and_validate_config  # noqa: F401

__all__ = ["LumenConfig", "Runtime", "Region", "load_and_validate_config", "ModelInfo", "Source", "Runtimes",
           "Metadata", "load_and_validate_model_info", "FaceV1", "EmbeddingV1", "LabelsV1", "OCRV1",
           "TextGenerationV1", "Downloader", "DownloadResult", "ResourceError", "ConfigError", "DownloadError",
           "PlatformUnavailableError", "ValidationError", "ModelInfoError"]
