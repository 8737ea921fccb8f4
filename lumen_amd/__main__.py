"""``python -m lumen_amd --config hub.yaml`` == the ``lumen`` hub server."""
import sys

from .cli import lumen

sys.exit(lumen())
