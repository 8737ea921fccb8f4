"""Resource-layer exceptions (same hierarchy as packages/lumen-resources/.../exceptions.py:8-110)."""
from __future__ import annotations


class ResourceError(Exception):
    """Base class for every resource-management error."""


class ConfigError(ResourceError):
    """Configuration file missing / unparsable / invalid."""


class DownloadError(ResourceError):
    """A model could not be fetched or verified."""


class PlatformUnavailableError(ResourceError):
    """The requested model platform SDK (ModelScope / HF hub) is unavailable."""


class ValidationError(ResourceError):
    """Generic validation failure (files, runtimes, datasets)."""


class ModelInfoError(ResourceError):
    """model_info.json missing or invalid."""


# ---- per-package resource-loader errors (CLIP/face/OCR/VLM loaders)
class ResourceNotFoundError(ResourceError):
    pass


class ResourceValidationError(ResourceError):
    pass


class RuntimeNotSupportedError(ResourceError):
    pass


class DatasetNotFoundError(ResourceError):
    pass


class TokenizerError(ResourceError):
    pass
