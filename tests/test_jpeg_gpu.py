"""GPU JPEG reconstruction (csrc/jpeg.hip) from the parallel entropy decoder's coefficient planes:
equal to the NumPy reference of the same arithmetic (float32 rounding aside: |diff| <= 2, mean < 0.01) and
within libjpeg-turbo's output (|diff| <= 3) for every sampling layout; the device decode
falls back to Pillow for progressive files."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from lumen_amd.utils import jpeg as J
from tests.test_jpeg_cpu import CASES, _enc, _synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_device_decode_matches_reference(name, make):
    data = make()
    st = {}
    got = J.decode_to_device(data, "cuda", stats=st).cpu().numpy().astype(np.int32)
    assert st.get("blocks", 0) > 0, "the native decode path did not run"
    coef, qt, ji, _ = J.decode_coefs(data, threads=4)
    ref = J.reconstruct_reference(coef, qt, ji).astype(np.int32)
    assert got.shape == ref.shape
    d = np.abs(got - ref)      # float32 vs float64 IDCT: a sample rounding the other way (+-1 in Y and in
    assert d.max() <= 2 and d.mean() < 0.01   # chroma shows as +-2 in R / G / B), very rarely
    pil = np.asarray(Image.open(io.BytesIO(data)).convert("RGB")).astype(np.int32)
    assert np.abs(got - pil).max() <= 3


def test_device_decode_progressive_falls_back():
    a = _synth(48, 64, "photo", 11)
    data = _enc(a, quality=90, progressive=True)
    st = {}
    got = J.decode_to_device(data, "cuda", stats=st).cpu().numpy()
    assert not st
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert np.array_equal(got, ref)


def test_device_decode_repeated_threads_reuse_staging():
    datas = [_enc(_synth(120 + 8 * i, 160, "noise", 20 + i), quality=90) for i in range(6)]
    outs = [J.decode_to_device(d, "cuda") for d in datas]      # one thread: staging buffer reused
    torch.cuda.synchronize()
    for d, o in zip(datas, outs):
        coef, qt, ji, _ = J.decode_coefs(d, threads=1)
        ref = J.reconstruct_reference(coef, qt, ji).astype(np.int32)
        assert np.abs(o.cpu().numpy().astype(np.int32) - ref).max() <= 2
