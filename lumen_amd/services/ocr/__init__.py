"""lumen-ocr equivalent: DBNet + SVTR CTC OCR on MI355X."""
from .backend import MI355XOcrBackend, OcrResult, create_backend
from .service import GeneralOcrService, OcrModelManager

__all__ = ["MI355XOcrBackend", "OcrResult", "create_backend", "GeneralOcrService", "OcrModelManager"]
