"""Console logging setup (reference uses colorlog; plain ANSI colours here, no dependency)."""
from __future__ import annotations

import logging
import os
import sys

_COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m", "ERROR": "\033[31m", "CRITICAL": "\033[35m"}


class _Fmt(logging.Formatter):
    def __init__(self, color: bool):
        super().__init__("%(asctime)s %(levelname)-8s %(name)s: %(message)s", "%H:%M:%S")
        self.color = color

    def format(self, record):
        s = super().format(record)
        if self.color and record.levelname in _COLORS:
            return f"{_COLORS[record.levelname]}{s}\033[0m"
        return s


def setup_logging(level: str = "INFO") -> None:
    root = logging.getLogger()
    root.setLevel(getattr(logging, level.upper(), logging.INFO))
    for h in list(root.handlers):
        root.removeHandler(h)
    h = logging.StreamHandler(sys.stdout)
    h.setFormatter(_Fmt(color=sys.stdout.isatty() and os.environ.get("NO_COLOR") is None))
    root.addHandler(h)
    for noisy in ("grpc", "urllib3", "PIL", "asyncio", "httpx"):
        logging.getLogger(noisy).setLevel(logging.WARNING)


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(name)
