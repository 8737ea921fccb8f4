"""lumen-face equivalent: SCRFD detection + ArcFace embedding on MI355X."""
from .backend import FaceDetection, MI355XFaceBackend, create_backend
from .model import FaceModelManager
from .service import GeneralFaceService

__all__ = ["FaceDetection", "MI355XFaceBackend", "create_backend", "FaceModelManager", "GeneralFaceService"]
