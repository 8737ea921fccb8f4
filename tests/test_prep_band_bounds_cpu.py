"""Host bounds of the fused band prep kernel (ops._prep_band_bounds; csrc/image.hip prep_band_kernel).

The kernel clamps the staged canvas rows to ``rcap`` and the taps per window to ``taps`` (LDS safety),
so a bound that is too small would silently drop samples.  Here the kernel's float32 window
arithmetic (image.hip ``window``, PIL filters) is replayed with numpy float32 for many geometries
(resize, centre crop, pad-to-square, letterbox-like destination rects) and every band's real row
span / window length must fit the host bounds."""
import numpy as np
import pytest
import torch

from lumen_amd import ops

f32 = np.float32


def _window(i, in_len, out_len, filt):
    scale = f32(in_len) / f32(out_len)
    ss = max(scale, f32(1.0))
    sup = f32(2.0 if filt == 0 else 1.0) * ss
    center = (f32(i) + f32(0.5)) * scale
    x0 = max(int(center - sup + f32(0.5)), 0)
    x1 = min(int(center + sup + f32(0.5)), in_len)
    return x0, x1


def _real_extents(g, OH, patch, filt):
    taps = rows = 0
    for rx in range(g.dw):
        x0, x1 = _window(rx, g.cw, g.dw, filt)
        taps = max(taps, x1 - x0)
    for band in range(OH // patch):
        live = [oy - g.dy for oy in range(band * patch, band * patch + patch) if 0 <= oy - g.dy < g.dh]
        if not live:
            continue
        y0s = [_window(ry, g.ch, g.dh, filt) for ry in live]
        for a, b in y0s:
            taps = max(taps, b - a)
        rows = max(rows, y0s[-1][1] - y0s[0][0])
    return rows, taps


def _geoms(rng, out):
    gs = []
    for _ in range(12):
        h, w = int(rng.integers(8, 1500)), int(rng.integers(8, 1500))
        kind = rng.integers(0, 3)
        if kind == 0:
            gs.append(ops.ImageGeom.resize(h, w, 0, out, out))
        elif kind == 1:
            gs.append(ops.ImageGeom.center_crop(h, w, 0, out))
        else:
            gs.append(ops.ImageGeom.pad_square(h, w, 0, out))
    return gs


@pytest.mark.parametrize("filt", [0, 1])
@pytest.mark.parametrize("out,patch", [(224, 14), (224, 16), (224, 32), (336, 14), (256, 16)])
def test_band_bounds_cover_every_band(filt, out, patch):
    rng = np.random.default_rng(out * 7 + patch + filt)
    geoms = _geoms(rng, out) + [ops.ImageGeom.resize(256, 256, 0, out, out),
                                ops.ImageGeom.resize(out, out, 0, out, out)]
    for g in geoms:
        b = ops._prep_band_bounds([g], filt, 2, patch, 3 * patch * patch + 8 - (3 * patch * patch) % 8, out,
                                  torch.bfloat16)
        # the LDS cap may reject big geometries; the bounds themselves are checked with it lifted
        old = ops._PREP_BAND_LDS
        ops._PREP_BAND_LDS = 1 << 40
        try:
            bb = ops._prep_band_bounds([g], filt, 2, patch, 3 * patch * patch + 8 - (3 * patch * patch) % 8, out,
                                       torch.bfloat16)
        finally:
            ops._PREP_BAND_LDS = old
        rows, taps = _real_extents(g, out, patch, filt)
        if bb is None:                       # > 16 taps: the two-pass kernels take it
            assert b is None
            continue
        rcap, cwcap, tmax = bb
        assert rows <= rcap, (g.ch, g.dh, rows, rcap)
        assert taps <= tmax <= 16, (g.cw, g.dw, g.ch, g.dh, taps, tmax)
        assert cwcap >= g.cw


def test_band_path_needs_integral_pad_and_pil_patches():
    g = [ops.ImageGeom.resize(256, 256, 0, 224, 224)]
    assert ops._prep_band_bounds(g, 0, 2, 14, 640, 224, torch.bfloat16) is not None
    assert ops._prep_band_bounds(g, 0, 2, 14, 640, 224, torch.bfloat16, pad=122.5) is None
    assert ops._prep_band_bounds(g, 2, 2, 14, 640, 224, torch.bfloat16) is None      # cv2 filter
    assert ops._prep_band_bounds(g, 0, 1, 14, 640, 224, torch.bfloat16) is None      # NHWC layout
    assert ops._prep_band_bounds(g, 0, 2, 14, 640, 224, torch.float32) is None
    assert ops._prep_band_bounds(g, 0, 2, 14, 644, 224, torch.bfloat16) is None      # kpad % 8
