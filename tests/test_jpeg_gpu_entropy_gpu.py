"""GPU entropy decode (csrc/jpeg_huff.hip) on the device: coefficient planes bit-identical to the
host decoder (csrc/host/jpeg_decode.cpp) on every layout, pixels identical to the host-entropy
device path, batches of mixed payloads in one launch, malformed streams flagged without a fault."""
import numpy as np
import pytest
import torch

from lumen_amd.utils import jpeg as J

from test_jpeg_cpu import CASES, _enc, _synth

pytestmark = pytest.mark.gpu
DEV = "cuda"

MORE = [("big420", lambda: _enc(_synth(768, 1024, "photo", 21), quality=92)),
        ("bignoise", lambda: _enc(_synth(600, 800, "noise", 22), quality=95)),
        ("restart444", lambda: _enc(_synth(120, 200, "noise", 24), quality=90, subsampling=0,
                                    restart_marker_blocks=5))]


def _gpu_coefs(datas):
    from lumen_amd.ops import hip_ops

    infos = [J.info(d) for d in datas]
    blob = torch.zeros(J.blob_capacity(datas, infos), dtype=torch.uint8).pin_memory()
    qt = np.zeros((len(datas), 192), np.uint16)
    used, ok = J.prepare_blob(datas, infos, blob.numpy(), qt)
    assert all(ok)
    tot = sum(ji.coef_count for ji in infos)
    coef = torch.full((tot,), 12345, dtype=torch.int16, device=DEV)
    err = torch.full((2 * len(datas),), -1, dtype=torch.int32, device=DEV)
    hb = blob[:used]
    hip_ops().jpeg_huff_decode(hb.to(DEV), hb, len(datas), coef, err)
    torch.cuda.synchronize()
    return coef.cpu().numpy(), err.cpu().numpy(), infos


@pytest.mark.parametrize("name,make", CASES + MORE, ids=[c[0] for c in CASES + MORE])
def test_gpu_entropy_matches_host_decoder(name, make):
    data = make()
    coef, err, infos = _gpu_coefs([data])
    ref = J.decode_coefs(data, threads=1)
    assert err[0] == 0
    assert np.array_equal(coef, ref[0]), int((coef != ref[0]).sum())
    emu = J.emulate_gpu_decode(data)
    assert err[1] == emu[4]          # same synchronisation rounds as the host emulation


def test_batch_one_launch_and_pixels():
    datas = [m() for _, m in CASES] + [MORE[0][1]()]
    coef, err, infos = _gpu_coefs(datas)
    assert (err[0::2] == 0).all()
    off = 0
    for d, ji in zip(datas, infos):
        ref = J.decode_coefs(d, threads=1)
        assert np.array_equal(coef[off:off + ji.coef_count], ref[0])
        off += ji.coef_count
    # the batched device decode (GPU entropy) == the host-entropy path, pixel for pixel
    import os
    os.environ["LUMEN_JPEG_GPU_ENTROPY"] = "1"
    try:
        flat, offs, shapes, errors = J.decode_batch_to_device(datas, DEV)
    finally:
        os.environ.pop("LUMEN_JPEG_GPU_ENTROPY")
    assert getattr(flat, "jpeg_err", None) is not None
    assert not errors and not J.device_errors(flat)
    ref_flat, roffs, rshapes, rerrors = J.decode_batch_to_device(datas, DEV)
    assert shapes == rshapes and offs == roffs and not rerrors
    assert torch.equal(flat, ref_flat)


def test_single_image_path_and_error_flag():
    data = _enc(_synth(480, 640, "photo", 41), quality=90)
    img = J.decode_to_device_gpu(data, DEV)
    assert img is not None and tuple(img.shape) == (480, 640, 3)
    J.check_device_error(img)
    host_path = J.decode_to_device(data, DEV)          # default: host entropy decode
    assert getattr(host_path, "jpeg_err", None) is None
    assert torch.equal(img, host_path)
    # corrupted middle of the segment: flagged (or, if it happens to parse, equal to the host decode)
    b = bytearray(data)
    at = len(b) // 2
    b[at:at + 64] = bytes(np.random.default_rng(3).integers(0, 255, 64, dtype=np.uint8))
    bad = bytes(b)
    img = J.decode_to_device_gpu(bad, DEV)
    torch.cuda.synchronize()
    if img is not None and int(img.jpeg_err[0]) == 0:
        c, q, ji, _ = J.decode_coefs(bad, threads=1)
        assert np.abs(img.cpu().numpy().astype(int) - J.reconstruct_reference(c, q, ji).astype(int)).max() <= 1
    elif img is not None:
        with pytest.raises(ValueError):
            J.check_device_error(img)
    # truncated stream: too few blocks -> flagged
    eoi = data.rindex(b"\xff\xd9")
    cut = data[:eoi // 2] + b"\xff\xd9"
    img = J.decode_to_device_gpu(cut, DEV)
    if img is not None:
        with pytest.raises(ValueError):
            J.check_device_error(img)
