"""Console entry points (reference pyproject.toml:17-18 and packages/*/pyproject.toml
``[project.scripts]``): ``lumen`` (hub), ``lumen-clip`` / ``lumen-face`` / ``lumen-ocr`` /
``lumen-vlm`` (single-service servers; flags ``--config --port --log-level --version``),
``lumen-resources`` and ``lumen-app``."""
from __future__ import annotations

import sys

from .hub.server import main as hub_main
from .hub.server import main_single


def lumen(argv=None) -> int:
    return hub_main(argv, mode="hub", prog="lumen")


def _single(prog):
    def run(argv=None) -> int:
        return main_single_named(argv, prog)
    return run


def main_single_named(argv, prog: str) -> int:
    return hub_main(argv, mode="single", prog=prog)


clip = _single("lumen-clip")
face = _single("lumen-face")
ocr = _single("lumen-ocr")
vlm = _single("lumen-vlm")


def resources(argv=None) -> int:
    from .resources.cli import main

    return main(argv)


def app(argv=None) -> int:
    from .app.main import main

    return main(argv)


if __name__ == "__main__":
    sys.exit(lumen())
