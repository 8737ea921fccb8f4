"""Per-service GPU placement for the hub (SURVEY §2.5 "process topology").

The reference hub builds every service in one process on whatever single device each
backend picks (packages/lumen-*/src/*/backends/*: one ORT session per service).  On an
8 x MI355X node that would pile CLIP, face, OCR and the VLM onto GPU 0.  Here the hub
gives each enabled service a disjoint set of GPUs before constructing it; the service's
backend reads its set through :func:`current` and runs one data-parallel worker per GPU
(CLIP / face / OCR) or uses the first GPU (VLM, whose tensor-parallel ranks are
launched by torchrun instead).

``LUMEN_PLACEMENT`` overrides the automatic plan, e.g. ``clip=0-3;face=4,5;ocr=6;vlm=7``
(unlisted services fall back to the automatic plan over the unused GPUs).  An explicit
``backend_settings.device`` in the config still pins a backend to one device.

Automatic plan: every service gets at least one GPU; the remaining GPUs go one at a time
to the service with the largest ``weight / gpus`` (image-embedding throughput services
weigh most).  With fewer GPUs than services they are shared round-robin.
"""
from __future__ import annotations

import contextlib
import contextvars
import logging
import os
from typing import Iterator, Optional, Sequence

log = logging.getLogger("lumen.placement")

DEFAULT_WEIGHTS = {"clip": 4.0, "smartclip": 4.0, "bioclip": 2.0, "face": 3.0, "ocr": 2.0, "vlm": 1.0}

_CURRENT: contextvars.ContextVar[Optional[tuple[int, ...]]] = contextvars.ContextVar("lumen_placement", default=None)


def _weight(name: str) -> float:
    n = name.lower()
    for k in sorted(DEFAULT_WEIGHTS, key=len, reverse=True):
        if k in n:
            return DEFAULT_WEIGHTS[k]
    return 1.0


def parse_spec(spec: str) -> dict[str, list[int]]:
    """``clip=0-3;face=4,5`` -> {"clip": [0, 1, 2, 3], "face": [4, 5]}."""
    out: dict[str, list[int]] = {}
    for part in filter(None, (p.strip() for p in spec.replace("\n", ";").split(";"))):
        name, _, devs = part.partition("=")
        if not devs:
            raise ValueError(f"placement entry {part!r}: expected name=devices")
        ids: list[int] = []
        for tok in filter(None, (t.strip() for t in devs.split(","))):
            if "-" in tok:
                a, b = (int(x) for x in tok.split("-", 1))
                if b < a:
                    raise ValueError(f"placement range {tok!r}")
                ids.extend(range(a, b + 1))
            else:
                ids.append(int(tok))
        if not ids:
            raise ValueError(f"placement entry {part!r} lists no device")
        out[name.strip()] = ids
    return out


def plan(names: Sequence[str], n_gpus: int, spec: Optional[str] = None) -> dict[str, list[int]]:
    """Device ids per service name (empty lists when there is no GPU)."""
    names = list(names)
    if n_gpus <= 0 or not names:
        return {n: [] for n in names}
    fixed = parse_spec(spec) if spec else {}
    for n, ids in fixed.items():
        bad = [i for i in ids if not 0 <= i < n_gpus]
        if bad:
            raise ValueError(f"placement for {n!r}: device(s) {bad} outside 0..{n_gpus - 1}")
    out = {n: list(fixed[n]) for n in names if n in fixed}
    rest = [n for n in names if n not in out]
    used = {i for ids in out.values() for i in ids}
    free = [i for i in range(n_gpus) if i not in used]
    if not rest:
        return out
    if len(free) < len(rest):                       # share: round-robin over all GPUs
        pool = free or list(range(n_gpus))
        for k, n in enumerate(rest):
            out[n] = [pool[k % len(pool)]]
        return out
    count = {n: 1 for n in rest}
    for _ in range(len(free) - len(rest)):
        best = max(rest, key=lambda n: (_weight(n) / count[n], -rest.index(n)))
        count[best] += 1
    k = 0
    for n in rest:
        out[n] = free[k:k + count[n]]
        k += count[n]
    return out


def plan_from_env(names: Sequence[str]) -> dict[str, list[int]]:
    try:
        import torch

        n = torch.cuda.device_count()       # counts devices without initialising HIP
    except Exception:  # noqa: BLE001
        n = 0
    p = plan(names, n, os.environ.get("LUMEN_PLACEMENT"))
    if n:
        log.info("GPU placement over %d device(s): %s", n, ", ".join(f"{k}={v}" for k, v in p.items()))
    return p


@contextlib.contextmanager
def use(devices: Optional[Sequence[int]]) -> Iterator[None]:
    """Construct / initialise a service under this device set."""
    tok = _CURRENT.set(tuple(devices) if devices else None)
    try:
        yield
    finally:
        _CURRENT.reset(tok)


def current() -> Optional[tuple[int, ...]]:
    return _CURRENT.get()


def dp_size_env() -> Optional[int]:
    v = os.environ.get("LUMEN_DP_SIZE")
    return max(1, int(v)) if v else None


def resolve(device_pref: Optional[str], dp_size_env: Optional[int] = None) -> tuple[Optional[str], list[str]]:
    """(device preference, DP worker devices) of a backend being constructed: an explicit
    ``backend_settings.device`` wins, then the hub's placement, then LUMEN_DP_SIZE over
    the first GPUs.  The worker list is empty for single-process serving."""
    devs = current()
    if device_pref:
        n = dp_size_env or 1
        return device_pref, ([] if n <= 1 else _first_devices(n, device_pref))
    if devs:
        n = dp_size_env or len(devs)
        ids = [devs[i % len(devs)] for i in range(n)]
        return f"cuda:{ids[0]}", ([f"cuda:{i}" for i in ids] if n > 1 else [])
    n = dp_size_env or 1
    return None, (_first_devices(n, None) if n > 1 else [])


def _first_devices(n: int, pref: Optional[str]) -> list[str]:
    if pref and pref.startswith("cpu"):
        return ["cpu"] * n
    from ..parallel.worker_pool import default_devices

    return default_devices(n)
