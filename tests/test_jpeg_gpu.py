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


def test_batch_decode_mixed_payloads():
    """decode_batch_to_device: every sampling layout of CASES plus a progressive JPEG, a PNG and a corrupt
    payload in ONE batch -- one IDCT + one colour launch for the baseline JPEGs, Pillow for the rest,
    each image at its offset; the corrupt one reported, not raised; repeated batches reuse the staging."""
    datas = [make() for _, make in CASES]
    prog = _enc(_synth(40, 56, "photo", 3), quality=85, progressive=True)
    png = io.BytesIO()
    Image.fromarray(_synth(30, 20, "noise", 4)).save(png, format="PNG")
    datas += [prog, png.getvalue(), b"\xff\xd8not a jpeg at all"]
    for _rep in range(2):
        flat, offs, shapes, errs = J.decode_batch_to_device(datas, "cuda")
        torch.cuda.synchronize()
        assert list(errs) == [len(datas) - 1]
        host = flat.cpu().numpy()
        for i, d in enumerate(datas[:-1]):
            h, w = shapes[i]
            got = host[offs[i]:offs[i] + h * w * 3].reshape(h, w, 3).astype(np.int32)
            ref = np.asarray(Image.open(io.BytesIO(d)).convert("RGB")).astype(np.int32)
            assert got.shape == ref.shape
            assert np.abs(got - ref).max() <= 3, i


def test_clip_engine_bytes_path_matches_host_decode():
    """The CLIP engine fn on encoded payloads (device batch decode + image_prep from the flat buffer)
    gives the embeddings of the host-decoded arrays."""
    from lumen_amd.models.clip import CLIPModel

    m = CLIPModel.random("ViT-B-32", seed=0, device="cuda")
    datas = [_enc(_synth(200 + 16 * i, 260, "photo", 30 + i), quality=90) for i in range(5)]
    flat, offs, shapes, errs = J.decode_batch_to_device(datas, "cuda")
    assert not errs
    got = m.encode_image_uint8(shapes, src=flat).float().cpu()
    arrs = [torch.from_numpy(np.asarray(Image.open(io.BytesIO(d)).convert("RGB")).copy()) for d in datas]
    ref = m.encode_image_uint8(arrs).float().cpu()
    assert torch.nn.functional.cosine_similarity(got, ref).min().item() > 0.999
