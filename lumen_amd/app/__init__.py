"""lumen-app equivalent: FastAPI control plane for the MI355X Lumen stack."""
from .main import AppState, create_app

__all__ = ["AppState", "create_app"]
