"""F-4 on the GPU: the HIP det_decode kernel's prior-box and decoded-box modes against the CPU
decode (same candidate rows), and the synthetic RetinaFace packs served on cuda vs cpu."""
import numpy as np
import pytest
import torch

from test_face_retinaface_cpu import S, _backend, _faces

pytestmark = pytest.mark.gpu


def _rows(cand, cnt):
    out = []
    for n in range(cand.shape[0]):
        k = min(int(cnt[n]), cand.shape[1])
        r = cand[n, :k].cpu().numpy()
        out.append(r[np.lexsort(np.round(r[:, :5][:, ::-1], 3).T)])
    return out


@pytest.mark.parametrize("mode", ["priors", "decoded", "normalised"])
def test_det_decode_modes_gpu_match_cpu(mode):
    from lumen_amd.ops import vision

    g = torch.Generator().manual_seed(0)
    N, P = 3, 700
    sc = torch.rand(N, P, generator=g)
    kp = torch.rand(N, P, 10, generator=g)
    pr = vision.retinaface_priors((S, S))[:P] if mode == "priors" else None
    if mode == "priors":
        P = pr.shape[0]
        sc, kp = sc[:, :P], kp[:, :P]
        bb = torch.randn(N, P, 4, generator=g) * 0.5
    else:
        xy = torch.rand(N, P, 2, generator=g)
        bb = torch.cat([xy, xy + torch.rand(N, P, 2, generator=g) * 0.5], -1)
        if mode == "decoded":
            bb = bb * S
    img_scale = torch.tensor([1.0, 0.5, 0.25])
    img_hw = torch.tensor([[64.0, 64.0], [128.0, 100.0], [256.0, 200.0]])
    res = {}
    for dev in ("cpu", "cuda"):
        cand = torch.zeros(N, 1024, 16, device=dev)
        cnt = torch.zeros(N, dtype=torch.int32, device=dev)
        args = (sc.to(dev), bb.to(dev), kp.to(dev))
        if mode == "priors":
            vision.det_decode_priors(*args, pr.to(dev), 0.6, img_scale.to(dev), img_hw.to(dev), cand, cnt, (S, S),
                                     min_size=2.0)
        else:
            vision.det_decode_boxes(*args, 0.6, img_scale.to(dev), img_hw.to(dev), cand, cnt,
                                    (1.0, 1.0) if mode == "decoded" else (-1.0, -1.0), min_size=2.0)
        res[dev] = _rows(cand, cnt)
    for a, b in zip(res["cpu"], res["cuda"]):
        assert a.shape == b.shape and len(a) > 0
        np.testing.assert_allclose(b[:, :15], a[:, :15], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("encoding", ["priors", "decoded"])
def test_retinaface_pack_gpu_matches_cpu(tmp_path, encoding):
    from lumen_amd.services.face.backend import MI355XFaceBackend

    be_cpu, _ = _backend(tmp_path, encoding)
    img = np.random.default_rng(11).integers(0, 255, (2 * S, 2 * S, 3), dtype=np.uint8)
    out = {}
    for dev, be in (("cpu", be_cpu), ("cuda", MI355XFaceBackend(be_cpu.resources, device="cuda"))):
        be.initialize()
        try:
            out[dev] = _faces(be, img, 0.6)
        finally:
            be.close()
    fc, fg = out["cpu"], out["cuda"]
    assert len(fc) > 0
    # bf16 detector input on the GPU: counts within a few, matched boxes close
    assert abs(len(fg) - len(fc)) <= max(2, len(fc) // 10)
    bc = np.array(sorted(f.bbox for f in fc))
    bg = np.array(sorted(f.bbox for f in fg))
    n = min(len(bc), len(bg))
    assert np.median(np.abs(bc[:n] - bg[:n])) < 2.0
