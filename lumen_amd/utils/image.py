"""Image decoding (K1) and small geometry helpers.

Decoded images are uint8 HWC RGB numpy/torch arrays that feed the fused
resize/normalise kernel (:func:`lumen_amd.ops.image_prep`).  Decoding runs on CPU
threads (Pillow's libjpeg-turbo; this ROCm image ships no rocJPEG).  ``draft``
lets the JPEG decoder produce a DCT-downscaled image (1/2 .. 1/8) when the target
is much smaller than the source — a large decode-throughput win for photos; off
by default because it changes the pixels the resampler sees (the reference
decodes at full resolution, clip onnxrt_backend.py:478).
"""
from __future__ import annotations

import io
from concurrent.futures import ThreadPoolExecutor
from typing import Optional, Sequence

import numpy as np
from PIL import Image, ImageOps

_POOL: Optional[ThreadPoolExecutor] = None


def _pool() -> ThreadPoolExecutor:
    global _POOL
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=8, thread_name_prefix="lumen-decode")
    return _POOL


def decode_rgb(data: bytes, draft_to: Optional[tuple[int, int]] = None, exif_transpose: bool = False) -> np.ndarray:
    """bytes (JPEG/PNG/WebP/BMP/...) -> uint8 [H, W, 3] RGB."""
    if not data:
        raise ValueError("empty image payload")
    try:
        im = Image.open(io.BytesIO(data))
        if draft_to is not None and im.format == "JPEG":
            im.draft("RGB", draft_to)
        if exif_transpose:
            im = ImageOps.exif_transpose(im)
        im = im.convert("RGB")
    except Exception as e:
        raise ValueError(f"cannot decode image: {e}") from e
    return np.array(im, dtype=np.uint8)  # writable copy (torch.from_numpy-safe)


def decode_bgr(data: bytes) -> np.ndarray:
    return decode_rgb(data)[:, :, ::-1].copy()


def decode_many(datas: Sequence[bytes], draft_to: Optional[tuple[int, int]] = None) -> list[np.ndarray]:
    if len(datas) == 1:
        return [decode_rgb(datas[0], draft_to)]
    return list(_pool().map(lambda d: decode_rgb(d, draft_to), datas))


def encode_jpeg(arr: np.ndarray, quality: int = 90) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def encode_png(arr: np.ndarray) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return buf.getvalue()
