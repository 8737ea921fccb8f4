"""Parallel baseline-JPEG entropy decoder (csrc/host/jpeg_decode.cpp) and the NumPy form of the
GPU reconstruction (utils/jpeg.py): speculative parallel decode == sequential decode bit for
bit, and the pixels match Pillow's libjpeg-turbo decode (its integer IDCT vs our float IDCT:
|diff| <= 3, p99 <= 1) for 4:2:0 / 4:2:2 / 4:4:4, grayscale, odd sizes and restart intervals;
progressive files are declined (Pillow fallback)."""
import io

import numpy as np
import pytest
from PIL import Image

from lumen_amd.utils import jpeg as J


def _synth(h, w, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    a = np.stack([(x / w * 255) % 256, (y / h * 255) % 256, ((x + y) / (h + w) * 255) % 256], -1)
    for _ in range(5):
        cy, cx, r = rng.integers(0, h), rng.integers(0, w), rng.integers(max(2, h // 16), max(3, h // 4))
        a[(y - cy) ** 2 + (x - cx) ** 2 < r * r] = rng.integers(0, 256, 3)
    return a.astype(np.uint8)


def _enc(a, **kw):
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, "JPEG", **kw)
    return buf.getvalue()


CASES = [("photo420", lambda: _enc(_synth(480, 640, "photo", 0), quality=90)),
         ("noise420", lambda: _enc(_synth(240, 320, "noise", 1), quality=90)),
         ("odd420", lambda: _enc(_synth(333, 517, "photo", 2), quality=80)),
         ("444", lambda: _enc(_synth(200, 300, "photo", 3), quality=85, subsampling=0)),
         ("422", lambda: _enc(_synth(200, 300, "photo", 4), quality=85, subsampling=1)),
         ("gray", lambda: _enc(_synth(200, 300, "photo", 5)[..., 0], quality=85)),
         ("restart", lambda: _enc(_synth(200, 300, "photo", 6), quality=85, restart_marker_blocks=7)),
         ("tiny", lambda: _enc(_synth(9, 13, "noise", 7), quality=95))]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_parallel_decode_matches_sequential_and_pillow(name, make):
    data = make()
    ji = J.info(data)
    assert ji is not None
    seq = J.decode_coefs(data, threads=1)
    par = J.decode_coefs(data, threads=8)
    assert seq is not None and par is not None
    assert np.array_equal(seq[0], par[0]) and np.array_equal(seq[1], par[1])
    assert par[3]["blocks"] > 0
    got = J.reconstruct_reference(par[0], par[1], par[2]).astype(np.int32)
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB")).astype(np.int32)
    assert got.shape == ref.shape
    d = np.abs(got - ref)
    assert d.max() <= 3 and np.percentile(d, 99) <= 1 and d.mean() < 0.1


def test_unsupported_and_garbage_are_declined():
    a = _synth(64, 64, "photo", 9)
    assert J.info(_enc(a, quality=85, progressive=True)) is None
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, "PNG")
    assert J.info(buf.getvalue()) is None
    assert J.info(b"\xff\xd8\xff\xe0garbage") is None
    good = _enc(a, quality=85)
    for th in (1, 4):
        assert J.decode_coefs(good[: len(good) // 2], threads=th) is None   # truncated: declined


def _dht_offset(data: bytes) -> int:
    i = data.find(b"\xff\xc4")
    assert i > 0
    return i


def test_oversubscribed_huffman_table_is_rejected():
    """A DHT whose code counts overflow the code space (3 one-bit codes, 255 one-bit codes) would
    index past the fast lookup tables: parse() must reject it."""
    good = _enc(_synth(64, 64, "photo", 10), quality=85)
    i = _dht_offset(good)
    for n1 in (3, 255):
        bad = bytearray(good)
        bad[i + 5] = n1                    # counts[0] of the first table
        assert J.info(bytes(bad)) is None
        assert J.decode_coefs(bytes(bad), threads=4) is None


def test_missing_restart_interval_is_rejected():
    """A DRI stream with one RSTn marker removed has fewer intervals than the frame needs; the
    decoder must fail instead of leaving blocks unwritten in a reused staging buffer."""
    good = _enc(_synth(200, 300, "photo", 11), quality=85, restart_marker_blocks=7)
    assert J.decode_coefs(good, threads=4) is not None
    sos = good.find(b"\xff\xda")
    k = next(j for j in range(sos + 2, len(good) - 1) if good[j] == 0xFF and 0xD0 <= good[j + 1] <= 0xD7)
    bad = good[:k] + good[k + 2:]
    for th in (1, 4):
        assert J.decode_coefs(bad, threads=th) is None


def test_random_mutations_do_not_crash():
    """Byte mutations of valid JPEGs (headers and entropy data): every call returns a result or
    None, never crashes or hangs."""
    rng = np.random.default_rng(12)
    seeds = [_enc(_synth(48, 64, "photo", 13), quality=80),
             _enc(_synth(48, 64, "photo", 14), quality=80, restart_marker_blocks=3)]
    for base in seeds:
        for _ in range(300):
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 6))):
                pos = int(rng.integers(2, min(len(b), 700) if rng.random() < 0.7 else len(b)))
                b[pos] = int(rng.integers(0, 256))
            data = bytes(b)
            ji = J.info(data)
            if ji is not None and ji.coef_count < (1 << 22):
                J.decode_coefs(data, threads=int(rng.integers(1, 5)), jinfo=ji)


def test_pixel_cap_declines_bomb_headers(monkeypatch):
    """A header declaring a frame beyond the decompression-bomb cap is declined before any
    staging buffer is sized from it (the Pillow fallback then applies its own check)."""
    good = _enc(_synth(64, 96, "photo", 15), quality=85)
    assert J.info(good) is not None
    monkeypatch.setenv("LUMEN_JPEG_MAX_PIXELS", str(64 * 96 - 1))
    assert J.info(good) is None
    monkeypatch.delenv("LUMEN_JPEG_MAX_PIXELS")
    sof = good.find(b"\xff\xc0")
    big = bytearray(good)
    big[sof + 5:sof + 9] = bytes([0xFF, 0xFF, 0xFF, 0xFF])     # 65535 x 65535
    assert J.info(bytes(big)) is None
