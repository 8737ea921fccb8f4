"""The GPU entropy decoder's schedule (csrc/jpeg_huff.hip, per-lane code csrc/jpeg_huff_core.h) run
on the host by lumen_jpeg_gpu_emulate: lane entry states iterated to the fixed point, prefix sums
of block counts and DC differences, placement -- must reproduce the host decoder's coefficient
planes bit for bit on every layout (4:2:0 / 4:2:2 / 4:4:4, grayscale, odd sizes, restart
intervals, noise that needs many synchronisation rounds) and flag truncated / corrupted streams.
The kernel itself runs the same functions on the GPU (tests/test_jpeg_gpu_entropy_gpu.py)."""
import numpy as np
import pytest

from lumen_amd.utils import jpeg as J

from test_jpeg_cpu import CASES, _enc, _synth

MORE = [("big420", lambda: _enc(_synth(768, 1024, "photo", 21), quality=92)),
        ("bignoise", lambda: _enc(_synth(600, 800, "noise", 22), quality=95)),
        ("q20", lambda: _enc(_synth(300, 400, "photo", 23), quality=20)),
        ("restart444", lambda: _enc(_synth(120, 200, "noise", 24), quality=90, subsampling=0,
                                    restart_marker_blocks=5)),
        ("gray_odd", lambda: _enc(_synth(77, 131, "noise", 25)[..., 1], quality=70))]


@pytest.mark.parametrize("name,make", CASES + MORE, ids=[c[0] for c in CASES + MORE])
def test_emulated_gpu_schedule_matches_host_decoder(name, make):
    data = make()
    ref = J.decode_coefs(data, threads=1)
    got = J.emulate_gpu_decode(data)
    assert ref is not None and got is not None
    coef, qt, ji, bad, rounds = got
    assert bad == 0
    assert np.array_equal(qt, ref[1])
    assert np.array_equal(coef, ref[0]), int((coef != ref[0]).sum())
    if ji.restart == 0:
        assert 1 <= rounds <= 128, rounds      # converges in rounds ~ resync distance / span, not one per lane


def test_truncated_and_corrupted_streams_are_flagged():
    data = _enc(_synth(240, 320, "photo", 31), quality=90)
    ji = J.info(data)
    eoi = data.rindex(b"\xff\xd9")
    # truncated entropy-coded segment: too few blocks
    cut = data[:eoi // 2] + b"\xff\xd9"
    r = J.emulate_gpu_decode(cut)
    assert r is None or r[3] == 1
    # a run of 0xFF-free garbage in the middle of the segment: an invalid code or a wrong block count
    rng = np.random.default_rng(0)
    flagged = 0
    for t in range(6):
        b = bytearray(data)
        at = len(data) // 2 + 97 * t
        b[at:at + 64] = bytes(rng.integers(0, 255, 64, dtype=np.uint8))   # 0xFF excluded
        r = J.emulate_gpu_decode(bytes(b))
        if r is None:
            continue
        ref = J.decode_coefs(bytes(b), threads=1)
        if r[3] == 0:
            # not flagged: then it must decode like the host decoder (garbage that happens to parse)
            assert ref is not None and np.array_equal(r[0], ref[0])
        else:
            flagged += 1
    assert ji is not None and flagged >= 1


def test_blob_layout_for_a_batch():
    """Several images in one blob: jobs point at 256-aligned descriptors and consecutive
    coefficient ranges; the emulation decodes each into its own range."""
    datas = [m() for _, m in CASES[:4]]
    infos = [J.info(d) for d in datas]
    blob = np.zeros(J.blob_capacity(datas), np.uint8)
    qt = np.zeros((len(datas), 192), np.uint16)
    used, ok = J.prepare_blob(datas, infos, blob, qt)
    assert all(ok) and used <= blob.size
    jobs = blob[:16 * len(datas)].view(np.int64).reshape(-1, 2)
    assert (jobs[:, 0] % 256 == 0).all()
    assert list(jobs[:, 1]) == list(np.cumsum([0] + [ji.coef_count for ji in infos])[:-1])
    total = sum(ji.coef_count for ji in infos)
    coef = np.zeros(total, np.int16)
    err = np.zeros(2 * len(datas), np.int32)
    J._lib().lumen_jpeg_gpu_emulate(blob.ctypes.data, len(datas), coef.ctypes.data, err.ctypes.data, None)
    assert (err[0::2] == 0).all()
    for k, d in enumerate(datas):
        ref = J.decode_coefs(d, threads=1)
        assert np.array_equal(coef[jobs[k, 1]:jobs[k, 1] + infos[k].coef_count], ref[0])
