"""lumen-clip equivalent: general CLIP, BioCLIP and SmartCLIP services on MI355X."""
from .backend import MI355XClipBackend, create_backend  # noqa: F401
from .model import BioCLIPModelManager, CLIPModelManager  # noqa: F401
from .resources import ModelResources, ResourceLoader  # noqa: F401
from .service import BioCLIPService, GeneralCLIPService, SmartCLIPService  # noqa: F401
