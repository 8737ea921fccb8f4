"""Hub (multi-service router + server) — the `lumen` entry point."""
from .loader import ServiceLoader  # noqa: F401
from .router import HubRouter  # noqa: F401
