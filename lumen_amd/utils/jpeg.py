"""Device-side JPEG decode (K1): parallel host entropy decode + GPU pixel reconstruction.

The reference decodes every image with Pillow on one CPU thread
(packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:661-665,
packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:478,
packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py:716-723).  Here a baseline JPEG is

1. entropy-decoded by ``csrc/host/jpeg_decode.cpp`` over a pool of host threads (speculative
   chunks re-synchronised on block boundaries; restart intervals in parallel when present) into
   int16 coefficient planes, then
2. uploaded (one pinned H2D) and turned into pixels on the GPU by ``csrc/jpeg.hip``
   (dequantise, 8x8 IDCT, libjpeg "fancy" chroma upsampling, libjpeg's YCbCr -> RGB).

:func:`decode_to_device` returns a uint8 [H, W, 3] tensor on the device, ready for
``ops.image_prep``.  Anything else -- PNG / WebP, progressive or arithmetic JPEGs, CMYK --
falls back to Pillow (:func:`lumen_amd.utils.image.decode_rgb`) plus an upload.
:func:`reconstruct_reference` is the NumPy form of step 2 (CPU path and test oracle).
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .._native import load_host

_lock = threading.Lock()
_typed = False


def _lib():
    global _typed
    lib = load_host()
    if lib is None or not hasattr(lib, "lumen_jpeg_decode_coefs"):
        return None
    if not _typed:
        with _lock:
            lib.lumen_jpeg_info.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
            lib.lumen_jpeg_info.restype = ctypes.c_int
            lib.lumen_jpeg_decode_coefs.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p]
            lib.lumen_jpeg_decode_coefs.restype = ctypes.c_int
            if hasattr(lib, "lumen_jpeg_prepare_gpu"):
                lib.lumen_jpeg_prepare_gpu.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p,
                                                       ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                                       ctypes.c_int]
                lib.lumen_jpeg_prepare_gpu.restype = ctypes.c_int
                lib.lumen_jpeg_gpu_emulate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                       ctypes.c_void_p]
                lib.lumen_jpeg_gpu_emulate.restype = ctypes.c_int
                lib.lumen_jpeg_desc_bytes.restype = ctypes.c_int
            _typed = True
    return lib


def default_threads() -> int:
    env = os.environ.get("LUMEN_JPEG_THREADS")
    if env:
        return max(1, int(env))
    return max(1, min(16, os.cpu_count() or 1))


@dataclass
class JpegInfo:
    width: int
    height: int
    ncomp: int
    hmax: int
    vmax: int
    restart: int
    comps: list          # [(h, v, bw, bh, tq)]

    @property
    def coef_count(self) -> int:
        return sum(bw * bh * 64 for _, _, bw, bh, _ in self.comps)

    def meta(self) -> list[int]:
        m = [self.ncomp, self.hmax, self.vmax, self.width, self.height]
        for h, v, bw, bh, _ in self.comps:
            m += [h, v, bw, bh]
        return m


def max_pixels() -> int:
    """Decompression-bomb cap of the device path: Pillow's ``Image.MAX_IMAGE_PIXELS`` (the check
    the Pillow fallback applies), overridable with ``LUMEN_JPEG_MAX_PIXELS``."""
    env = os.environ.get("LUMEN_JPEG_MAX_PIXELS")
    if env:
        return int(env)
    try:
        from PIL import Image

        return int(Image.MAX_IMAGE_PIXELS or (1 << 62))
    except ImportError:     # pragma: no cover
        return 89_478_485


def info(data: bytes) -> Optional[JpegInfo]:
    """Header of a baseline JPEG this decoder handles, else None.  A frame larger than
    :func:`max_pixels` is also None: the caller falls back to Pillow, whose bomb check rejects
    it before any staging buffer is sized from the header."""
    lib = _lib()
    if lib is None or len(data) < 4 or data[:2] != b"\xff\xd8":
        return None
    out = (ctypes.c_int * 32)()
    if lib.lumen_jpeg_info(data, len(data), out) != 0:
        return None
    if out[0] * out[1] > max_pixels():
        return None
    nc = out[2]
    comps = [tuple(out[8 + 5 * c + k] for k in range(5)) for c in range(nc)]
    return JpegInfo(out[0], out[1], nc, out[3], out[4], out[5], comps)


def decode_coefs(data: bytes, threads: Optional[int] = None, jinfo: Optional[JpegInfo] = None,
                 out: Optional[np.ndarray] = None):
    """-> (coefficients int16 [coef_count], quant tables uint16 [ncomp, 64], JpegInfo, stats) or None."""
    lib = _lib()
    ji = jinfo or info(data)
    if lib is None or ji is None:
        return None
    coef = out if out is not None else np.empty(ji.coef_count, np.int16)
    qt = np.empty((ji.ncomp, 64), np.uint16)
    st = np.zeros(4, np.int64)
    r = lib.lumen_jpeg_decode_coefs(data, len(data), int(threads or default_threads()), coef.ctypes.data,
                                    qt.ctypes.data, st.ctypes.data)
    if r != 0:
        return None
    return coef, qt, ji, {"chunks": int(st[0]), "resynced": int(st[1]), "serial_blocks": int(st[2]),
                          "blocks": int(st[3])}


# ------------------------------------------------------------------ GPU entropy decode (csrc/jpeg_huff.hip)
_HEAD = 512                 # blob header: JHuffJob[n] when n <= 32 (else n * 16 rounded up to 256)


def gpu_entropy_enabled() -> bool:
    """``LUMEN_JPEG_GPU_ENTROPY=1``: baseline JPEGs are entropy-decoded on the GPU
    (csrc/jpeg_huff.hip) instead of on the host thread pool.  Off by default: a GPU lane decodes a
    Huffman symbol in ~1 us (a serial dependent chain of ~130 instructions and 3-4 LDS round trips),
    so the lone-image decode (1.3-1.6 ms for a 1024 x 768 photo, bound by the resynchronisation
    chain) loses to the 16-thread host decoder (0.9 ms), and a batch-128 decode (7.8k img/s) holds
    up to 128 CUs for 16 ms that the vision tower would use (profiles/r5_jpeg_gpu_entropy_v1.txt).
    It pays where host cores are the scarce resource."""
    return os.environ.get("LUMEN_JPEG_GPU_ENTROPY", "0") == "1"


def _desc_bytes() -> int:
    return (int(_lib().lumen_jpeg_desc_bytes()) + 255) & ~255


def _cap1(data: bytes, ji: "JpegInfo") -> int:
    """blob bytes one payload may take: descriptor + stream words (+ the restart table, at most one
    4-byte start per 2 payload bytes)"""
    return (_desc_bytes() + (3 if ji.restart else 1) * len(data) + 1024 + 255) & ~255


def _head(n: int) -> int:
    return max(_HEAD, (16 * n + 255) & ~255)


def blob_capacity(datas, infos=None) -> int:
    """Upper bound of the upload blob for these payloads (job header + per image descriptor,
    stream words and restart table)."""
    infos = infos or [info(d) for d in datas]
    return _head(len(datas)) + sum(_cap1(d, ji) for d, ji in zip(datas, infos) if ji is not None)


def single_lanes() -> int:
    """Lanes for a lone image (``LUMEN_JPEG_LANES``, default 1024 = 4 workgroups): more lanes
    shorten each lane's span but add synchronisation rounds (~ resync distance / span), each a
    cross-workgroup barrier (profiles/r5_jpeg_gpu_entropy_*)."""
    return int(os.environ.get("LUMEN_JPEG_LANES", "1024"))


def lanes_for(n_images: int, cus: int = 256) -> int:
    """Decoding lanes per image for a batch of n: 256-lane workgroups, as many per image (<= 16) as
    keep every workgroup of the batch resident at once (the image's workgroups meet at a spin
    barrier), so a lone image spreads over 16 CUs and a batch of >= 256 uses one CU each."""
    return 256 * max(1, min(16, cus // max(1, n_images)))


def prepare_blob(datas, infos, blob: np.ndarray, qt: np.ndarray, pool=None, lanes: Optional[int] = None):
    """Fill ``blob`` (uint8, >= blob_capacity) with each payload's descriptor + stream at a fixed
    offset (prepared on ``pool`` when given: the ctypes calls release the GIL) and a job header
    listing the payloads that prepared; ``qt`` [n, 192] uint16 receives the quantisation tables.
    Coefficients of payload k start at element sum(coef_count of the payloads before it).
    -> (bytes to upload, ok flags); the job count is sum(ok)."""
    lib = _lib()
    n = len(datas)
    lanes = lanes or lanes_for(n)
    offs, coffs, off, coff = [], [], _head(n), 0
    for d, ji in zip(datas, infos):
        offs.append(off)
        coffs.append(coff)
        if ji is not None:
            off += _cap1(d, ji)
            coff += ji.coef_count
    base = blob.ctypes.data

    def one(k):
        if infos[k] is None:
            return False, 0
        need = ctypes.c_int64(0)
        cap = _cap1(datas[k], infos[k])
        r = lib.lumen_jpeg_prepare_gpu(datas[k], len(datas[k]), base + offs[k], cap, qt[k].ctypes.data,
                                       ctypes.byref(need), int(lanes))
        return r == 0, int(need.value)

    res = list(pool.map(one, range(n))) if pool is not None and n > 2 else [one(k) for k in range(n)]
    ok = [r[0] for r in res]
    jobs = np.array([(offs[k], coffs[k]) for k in range(n) if ok[k]], np.int64).reshape(-1, 2)
    blob[:16 * len(jobs)].view(np.int64)[:] = jobs.reshape(-1)
    used = max([_head(n)] + [offs[k] + res[k][1] for k in range(n) if ok[k]])
    return (used + 15) & ~15, ok


def emulate_gpu_decode(data: bytes, lanes: Optional[int] = None, stats: Optional[dict] = None):
    """The GPU decoder's schedule run on the host (csrc/host/jpeg_decode.cpp:lumen_jpeg_gpu_emulate)
    -> (coefficients int16 [coef_count], qt [ncomp, 64], JpegInfo, malformed flag, rounds) or None."""
    ji = info(data)
    if ji is None:
        return None
    blob = np.zeros(blob_capacity([data], [ji]), np.uint8)
    qt = np.zeros((1, 192), np.uint16)
    used, ok = prepare_blob([data], [ji], blob, qt, lanes=lanes)
    if not ok[0]:
        return None
    coef = np.full(ji.coef_count, 12345, np.int16)      # zeroed by the emulation, as by the launcher
    err = np.zeros(2, np.int32)
    st = np.zeros(4, np.int64)
    _lib().lumen_jpeg_gpu_emulate(blob.ctypes.data, 1, coef.ctypes.data, err.ctypes.data, st.ctypes.data)
    if stats is not None:
        stats.update(slides=int(st[0]), blocks=int(st[1]), max_lane_slides=int(st[2]), lanes=int(st[3]))
    return coef, qt[0, :64 * ji.ncomp].reshape(ji.ncomp, 64), ji, int(err[0]), int(err[1])


class _HuffStaging(threading.local):
    blob = None
    qt = None
    ev = None


_hstage = _HuffStaging()


def decode_to_device_gpu(data: bytes, device, ji: Optional["JpegInfo"] = None, lanes: Optional[int] = None):
    """Baseline JPEG -> uint8 [H, W, 3] on ``device`` with the entropy decode on the GPU too:
    the host parses the header and unstuffs the bytes into a pinned blob (one H2D), then
    jpeg_huff_decode + jpeg_reconstruct run on the current stream.  The result carries
    ``jpeg_err`` (device int32 [2]: malformed flag, rounds) for :func:`check_device_error`.
    None when the payload is not a baseline JPEG this path handles."""
    import torch

    from ..ops import hip_ops

    dev = torch.device(device)
    ji = ji or info(data)
    if ji is None:
        return None
    st = _hstage
    if st.ev is not None:
        st.ev.synchronize()              # this thread's previous upload has read the staging blob
    cap = blob_capacity([data], [ji])
    if st.blob is None or st.blob.numel() < cap:
        st.blob = torch.empty(max(cap, 1 << 20), dtype=torch.uint8).pin_memory()
        st.qt = torch.empty((1, 192), dtype=torch.int16).pin_memory()
    bnp = st.blob.numpy()
    used, ok = prepare_blob([data], [ji], bnp, st.qt.numpy().view(np.uint16), lanes=lanes or single_lanes())
    if not ok[0]:
        return None
    hb = st.blob[:used]
    bd = hb.to(dev, non_blocking=True)
    qd = st.qt[0, :64 * ji.ncomp].to(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    st.ev = ev
    n = ji.coef_count
    coef = torch.empty(n, dtype=torch.int16, device=dev)
    err = torch.empty(2, dtype=torch.int32, device=dev)
    ops = hip_ops()
    ops.jpeg_huff_decode(bd, hb, 1, coef, err)
    samp = torch.empty(n, dtype=torch.uint8, device=dev)
    out = torch.empty((ji.height, ji.width, 3), dtype=torch.uint8, device=dev)
    ops.jpeg_reconstruct(coef, qd, ji.meta(), samp, out)
    out.jpeg_err = err
    return out


def check_device_error(img) -> None:
    """Raise ValueError when a GPU-entropy-decoded image's stream was malformed (reads the flag:
    a device sync, so call it where the caller synchronises anyway)."""
    err = getattr(img, "jpeg_err", None)
    if err is not None and int(err[0].item()) != 0:
        raise ValueError("cannot identify image file: malformed JPEG entropy-coded data")


# ------------------------------------------------------------------ NumPy reference of csrc/jpeg.hip
def _idct_matrix() -> np.ndarray:
    k = np.zeros((8, 8), np.float64)
    for u in range(8):
        cu = np.sqrt(0.5) if u == 0 else 1.0
        for x in range(8):
            k[u, x] = cu / 2 * np.cos((2 * x + 1) * u * np.pi / 16)
    return k


def _fancy(pl: np.ndarray, dw: int, dh: int, W: int, H: int, sx: int, sy: int) -> np.ndarray:
    """libjpeg fancy upsampling of a chroma plane (valid region dh x dw) to H x W."""
    p = pl[:dh, :dw].astype(np.int32)
    if sx == 1 and sy == 1:
        return p[:H, :W]
    X = np.arange(W)
    c = X // sx
    if sy == 2:
        Y = np.arange(H)
        r = Y // 2
        rf = np.where(Y & 1, np.minimum(r + 1, dh - 1), np.maximum(r - 1, 0))
        cs = 3 * p[r] + p[rf]                                   # [H, dw]
        left = cs[:, np.maximum(c - 1, 0)]
        right = cs[:, np.minimum(c + 1, dw - 1)]
        mid = cs[:, c]
        return np.where(X & 1, (3 * mid + right + 7) >> 4, (3 * mid + left + 8) >> 4)
    cs = p[:H]
    left, right, mid = cs[:, np.maximum(c - 1, 0)], cs[:, np.minimum(c + 1, dw - 1)], cs[:, c]
    return np.where(X & 1, (3 * mid + right + 2) >> 2, (3 * mid + left + 1) >> 2)


def reconstruct_reference(coef: np.ndarray, qt: np.ndarray, ji: JpegInfo) -> np.ndarray:
    """The GPU kernel's arithmetic in NumPy: coefficient planes -> uint8 [H, W, 3]."""
    K = _idct_matrix()
    planes, off = [], 0
    for c, (h, v, bw, bh, _) in enumerate(ji.comps):
        n = bw * bh * 64
        blk = coef[off:off + n].reshape(bh, bw, 8, 8).astype(np.float64) * qt[c].reshape(8, 8)
        off += n
        pix = np.einsum("vy,ux,abvu->abyx", K, K, blk)           # [bh, bw, y, x]
        pix = np.clip(np.rint(pix + 128.0), 0, 255).astype(np.int32)
        planes.append(pix.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    W, H = ji.width, ji.height
    y = planes[0][:H, :W]
    if ji.ncomp == 1:
        return np.repeat(y[..., None], 3, -1).astype(np.uint8)
    ch = []
    for c in (1, 2):
        h, v = ji.comps[c][0], ji.comps[c][1]
        dw, dh = (W * h + ji.hmax - 1) // ji.hmax, (H * v + ji.vmax - 1) // ji.vmax
        ch.append(_fancy(planes[c], dw, dh, W, H, ji.hmax // h, ji.vmax // v) - 128)
    cb, cr = ch
    r = y + ((91881 * cr + 32768) >> 16)
    g = y + ((-22554 * cb - 46802 * cr + 32768) >> 16)
    b = y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


# ------------------------------------------------------------------ device decode
class _Staging(threading.local):
    buf = None
    ev = None       # the H2D copy that last read buf


_staging = _Staging()


def decode_to_device(data: bytes, device, threads: Optional[int] = None, stats: Optional[dict] = None):
    """JPEG bytes -> uint8 [H, W, 3] tensor on ``device``.  Baseline JPEGs take the parallel
    entropy decoder + GPU reconstruction; everything else (and CPU devices) decodes with
    Pillow.  Raises ValueError on undecodable input, like decode_rgb."""
    import torch

    from .image import decode_rgb

    dev = torch.device(device)
    ji = info(data) if dev.type == "cuda" else None
    if ji is not None and gpu_entropy_enabled() and threads is None and stats is None:
        out = decode_to_device_gpu(data, dev, ji)
        if out is not None:
            return out
    if ji is not None:
        # coefficients straight into a pinned, per-thread staging buffer -> one async H2D
        n = ji.coef_count
        if _staging.ev is not None:
            _staging.ev.synchronize()      # this thread's previous upload has read the buffer
        st = _staging.buf
        if st is None or st.numel() < n:
            st = torch.empty(max(n, 1 << 20), dtype=torch.int16).pin_memory()
            _staging.buf = st
        host = st[:n].numpy()
        res = decode_coefs(data, threads, ji, out=host)
        if res is not None:
            coef, qt, ji, s = res
            if stats is not None:
                stats.update(s)
            from ..ops import hip_ops
            from .h2d import h2d

            cd = st[:n].to(dev, non_blocking=True)
            qd = h2d(qt.view(np.int16), dev)
            samp = torch.empty(n, dtype=torch.uint8, device=dev)
            out = torch.empty((ji.height, ji.width, 3), dtype=torch.uint8, device=dev)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            _staging.ev = ev
            hip_ops().jpeg_reconstruct(cd, qd, ji.meta(), samp, out)
            return out
    return torch.from_numpy(decode_rgb(data)).to(dev)


# ------------------------------------------------------------------ batched device decode (serving engines)
_ENTRY_BYTES = 256            # >= sizeof(JpegBatchEntry) (168 on gfx950 builds)
_pool_lock = threading.Lock()
_decode_pool = None


def _pool():
    global _decode_pool
    with _pool_lock:
        if _decode_pool is None:
            from concurrent.futures import ThreadPoolExecutor

            _decode_pool = ThreadPoolExecutor(max_workers=default_threads(), thread_name_prefix="jpeg-batch")
        return _decode_pool


class _BatchStaging(threading.local):
    """Two pinned staging sets per thread, alternating: a caller that queues batch i + 1 before the
    device has consumed batch i's copies waits only for batch i - 1's."""

    def __init__(self):
        self.slots = [[None, None], [None, None]]    # [bufs (coef, qt, entries, raw, blob), event of their H2D]
        self.k = 0


_bstage = _BatchStaging()


def _pinned(t, n: int, dtype):
    import torch

    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1 << 16), dtype=dtype).pin_memory()
    return t


def decode_batch_to_device(datas, device):
    """Encoded images -> one flat uint8 device tensor holding every image as [H, W, 3] back to
    back, for ``ops.image_prep(src=...)``: returns (flat, offsets, shapes, errors).

    Baseline JPEGs: entropy-decoded on the decode pool (one image per thread, the ctypes call
    releases the GIL) into one pinned coefficient buffer, one H2D copy, then ONE batched IDCT and
    ONE colour launch for the whole batch (csrc/jpeg.hip).  Anything else (PNG, progressive, a
    payload the fast decoder rejects) decodes with Pillow on the same pool and is copied into its
    slot.  ``errors`` maps the index of an undecodable payload to its exception (its slot is a
    1 x 1 black image so the batch stays aligned)."""
    import torch

    from .image import decode_rgb

    dev = torch.device(device)
    n = len(datas)
    infos = [info(d) for d in datas]
    jidx = [i for i, ji in enumerate(infos) if ji is not None]
    cbase, tot = {}, 0
    for i in jidx:
        cbase[i] = tot
        tot += infos[i].coef_count
    st = _bstage
    slot = st.slots[st.k]
    st.k ^= 1
    if slot[1] is not None:
        slot[1].synchronize()        # the batch before last has been copied out of this staging set
    coef_h, qt_h, ent_h, raw_h, blob_h = slot[0] or (None, None, None, None, None)
    qt_h = _pinned(qt_h, max(1, len(jidx)) * 192, torch.int16)
    ent_h = _pinned(ent_h, max(1, len(jidx)) * _ENTRY_BYTES, torch.uint8)
    qt_np = qt_h.numpy()
    gpu_ent = bool(jidx) and gpu_entropy_enabled()
    if gpu_ent:
        # entropy decode on the GPU (csrc/jpeg_huff.hip): the host only parses + unstuffs
        dj, ij = [datas[i] for i in jidx], [infos[i] for i in jidx]
        blob_h = _pinned(blob_h, blob_capacity(dj, ij), torch.uint8)
        used, ok = prepare_blob(dj, ij, blob_h.numpy(), qt_np[:len(jidx) * 192].view(np.uint16).reshape(-1, 192),
                                _pool())
    else:
        coef_h = _pinned(coef_h, tot, torch.int16)
        coef_np = coef_h.numpy()

        def ent(k_i):
            k, i = k_i
            ji = infos[i]
            res = decode_coefs(datas[i], 1, ji, out=coef_np[cbase[i]:cbase[i] + ji.coef_count])
            if res is None:
                return None
            q = res[1]
            qt_np[k * 192:k * 192 + q.size] = q.reshape(-1).view(np.int16)
            return True

        ok = list(_pool().map(ent, list(enumerate(jidx)))) if jidx else []
    good = [i for i, r in zip(jidx, ok) if r]
    good_set = set(good)
    slow = [i for i in range(n) if i not in good_set]

    def pil(i):
        try:
            return decode_rgb(datas[i])
        except Exception as e:    # noqa: BLE001 -- reported per item
            return e

    pix = dict(zip(slow, _pool().map(pil, slow))) if slow else {}
    errors = {i: p for i, p in pix.items() if isinstance(p, BaseException)}
    shapes, offs, off = [], [], 0
    for i in range(n):
        if i in errors:
            h, w = 1, 1
        elif i in pix:
            h, w = pix[i].shape[:2]
        else:
            h, w = infos[i].height, infos[i].width
        shapes.append((h, w))
        offs.append(off)
        off += h * w * 3
    out = torch.zeros(max(off, 1), dtype=torch.uint8, device=dev) if errors else \
        torch.empty(max(off, 1), dtype=torch.uint8, device=dev)
    raw_n = sum(p.size for i, p in pix.items() if i not in errors)
    raw_h = _pinned(raw_h, raw_n, torch.uint8)
    if raw_n:
        rnp, r = raw_h.numpy(), 0
        for i, p in pix.items():
            if i in errors:
                continue
            rnp[r:r + p.size] = np.ascontiguousarray(p).reshape(-1)
            out[offs[i]:offs[i] + p.size].copy_(raw_h[r:r + p.size], non_blocking=True)
            r += p.size
    if good:
        from ..ops import hip_ops

        meta = np.zeros((len(good), 21), np.int64)
        sbase = 0
        for k, i in enumerate(good):
            ji = infos[i]
            row = [cbase[i], sbase, offs[i], ji.ncomp, ji.hmax, ji.vmax, ji.width, ji.height]
            for c in range(3):
                row += list(ji.comps[c][:2]) + list(ji.comps[c][2:4]) if c < ji.ncomp else [0, 0, 0, 0]
            row.append(jidx.index(i))
            meta[k] = row
            sbase += ji.coef_count
        qt_d = qt_h[:len(jidx) * 192].to(dev, non_blocking=True)
        if gpu_ent:
            hb = blob_h[:used]
            coef_d = torch.empty(max(tot, 1), dtype=torch.int16, device=dev)
            err_d = torch.empty(2 * len(good), dtype=torch.int32, device=dev)
            hip_ops().jpeg_huff_decode(hb.to(dev, non_blocking=True), hb, len(good), coef_d, err_d)
            out.jpeg_err = err_d
            out.jpeg_err_items = list(good)
        else:
            coef_d = coef_h[:tot].to(dev, non_blocking=True)
        samp = torch.empty(max(sbase, 1), dtype=torch.uint8, device=dev)
        ent_d = torch.empty(len(good) * _ENTRY_BYTES, dtype=torch.uint8, device=dev)
        hip_ops().jpeg_reconstruct_batch(coef_d, qt_d, torch.from_numpy(meta), samp, out, ent_d, ent_h)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    slot[1] = ev
    slot[0] = (coef_h, qt_h, ent_h, raw_h, blob_h)
    return out, offs, shapes, errors


def device_errors(flat) -> dict:
    """Payloads of a :func:`decode_batch_to_device` batch whose GPU entropy decode found a
    malformed stream -> {index: ValueError} (reads the flags: a device sync, so call it where the
    caller synchronises anyway, e.g. after copying its results to the host)."""
    err = getattr(flat, "jpeg_err", None)
    if err is None:
        return {}
    flags = err.view(-1, 2)[:, 0].cpu().numpy()
    return {i: ValueError("cannot identify image file: malformed JPEG entropy-coded data")
            for i, f in zip(flat.jpeg_err_items, flags) if f}


class DeviceImage:
    """Shape-only stand-in for a decoded image whose pixels live in a device buffer
    (:func:`decode_batch_to_device`): the batched pipelines (face detection / alignment) take
    their geometry from ``shape`` and their pixels from the flat buffer + offset."""

    __slots__ = ("shape",)

    def __init__(self, h: int, w: int):
        self.shape = (int(h), int(w), 3)

    @property
    def size(self) -> int:
        return self.shape[0] * self.shape[1] * 3


def decode_image(data: bytes, device, draft_to: Optional[tuple] = None, stats: Optional[dict] = None):
    """Request image -> uint8 [H, W, 3] torch tensor: on a GPU device a baseline JPEG takes
    :func:`decode_to_device` (full resolution, no DCT-domain shortcut needed: the entropy decode
    runs on every host thread and the pixels on the GPU); anything else decodes with Pillow
    (DCT-scaled to ``draft_to`` when given) and stays on the host."""
    import torch

    from .image import decode_rgb

    if torch.device(device).type == "cuda" and info(data) is not None:
        return decode_to_device(data, device, stats=stats)
    return torch.from_numpy(decode_rgb(data, draft_to=draft_to))
