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
    """Host decode / staging threads: LUMEN_DECODE_THREADS, else min(16, CPUs) (a GPU box's
    share is 16 CPUs; PIL's libjpeg-turbo and numpy copies release the GIL)."""
    global _POOL
    if _POOL is None:
        import os

        n = int(os.environ.get("LUMEN_DECODE_THREADS", "0")) or min(16, os.cpu_count() or 8)
        _POOL = ThreadPoolExecutor(max_workers=max(1, n), thread_name_prefix="lumen-decode")
    return _POOL


class PinnedUploader:
    """One H2D copy for a batch of decoded images: the images are copied (on the decode
    threads) into a pinned staging buffer and sent with one non-blocking transfer; returns
    the flat uint8 device tensor and each image's element offset.  Two staging buffers
    alternate, each reused only after its previous transfer completed (event), so the
    copy of batch i+1 overlaps the GPU work of batch i.  Replaces torch.cat of pageable
    arrays + a pageable (synchronous) copy per consumer."""

    def __init__(self, device):
        import torch

        self.device = torch.device(device)
        self.bufs = [None, None]
        self.events = [None, None]
        self.k = 0

    def upload(self, images: Sequence[np.ndarray]):
        import torch

        sizes = [int(im.size) for im in images]
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64) if sizes else np.zeros(0, np.int64)
        total = int(sum(sizes))
        k = self.k
        self.k ^= 1
        if self.events[k] is not None:
            self.events[k].synchronize()
        buf = self.bufs[k]
        if buf is None or buf.numel() < total:
            buf = torch.empty(max(total, 1 << 20), dtype=torch.uint8, pin_memory=True)
            self.bufs[k] = buf
        host = buf.numpy()

        def cp(i):
            host[offs[i]:offs[i] + sizes[i]] = np.ascontiguousarray(images[i]).reshape(-1)

        if len(images) > 1:
            list(_pool().map(cp, range(len(images))))
        elif images:
            cp(0)
        stream = self.side_stream if getattr(self, "_side", False) else None
        with torch.cuda.stream(stream) if stream is not None else _null():
            dev = buf[:total].to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self.events[k] = ev
        self.last_event = ev
        return dev, offs

    def upload_async(self, images: Sequence[np.ndarray]):
        """Like :meth:`upload` but the H2D copy runs on this uploader's own stream, so it can be
        issued from a prefetch thread while the compute stream is busy with the previous batch
        without queueing behind (or in the middle of) that batch's kernels.  Returns
        ``(dev, offs, ready)``: the consumer calls :func:`consume` (stream wait + allocator hand-off)
        before its kernels read ``dev``."""
        import torch

        if getattr(self, "side_stream", None) is None:
            self.side_stream = torch.cuda.Stream(self.device)
        self._side = True
        try:
            dev, offs = self.upload(images)
        finally:
            self._side = False
        return dev, offs, self.last_event


def consume(dev, ready) -> None:
    """Make the current stream wait for an :meth:`PinnedUploader.upload_async` copy and tell the
    caching allocator the buffer is used on it."""
    import torch

    cur = torch.cuda.current_stream(dev.device)
    if ready is not None:
        cur.wait_event(ready)
    dev.record_stream(cur)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


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
