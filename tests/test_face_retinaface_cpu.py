"""F-4: RetinaFace-family / generic detector packs (reference
packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py:810-880, ``detector_type`` other than
"scrfd").  Synthetic RetinaFace-shaped ONNX packs (lumen_amd/resources/synthetic_retinaface.py) are
served by the face backend; the candidate boxes are pinned against an independent NumPy decode of
the same graph outputs:

* prior-box exports (loc / conf / landms against the (step, min_size) prior grid, variances
  0.1 / 0.2) -> ``vision.det_decode_priors``;
* already-decoded exports (the reference contract: corner boxes in input pixels) ->
  ``vision.det_decode_boxes``, including boxes normalised to the original image
  (reference ``normalized_boxes``).

Un-letterboxing is exercised with a 2x image (letterbox scale 0.5)."""
import numpy as np
import pytest
import torch

from lumen_amd.resources.synthetic_retinaface import MIN_SIZES, STEPS, write_retinaface_pack
from lumen_amd.runtime.onnx_graph import OnnxGraph

S = 64
MEAN_BGR = np.array([104.0, 117.0, 123.0], np.float32)


def numpy_priors(size):
    out = []
    for step, sizes in zip(STEPS, MIN_SIZES):
        f = int(np.ceil(size / step))
        for i in range(f):
            for j in range(f):
                for ms in sizes:
                    out.append([(j + 0.5) * step / size, (i + 0.5) * step / size, ms / size, ms / size])
    return np.array(out, np.float32)


def graph_input(img):
    """The detector input: an S x S image as is (BGR, mean-subtracted); a larger one through the
    CPU letterbox resize (cv2 INTER_LINEAR, pinned by tests/test_face_compat_cpu.py)."""
    if img.shape[0] == S:
        x = (img.astype(np.float32)[..., ::-1] - MEAN_BGR).transpose(2, 0, 1)[None]
        return torch.from_numpy(np.ascontiguousarray(x))
    from lumen_amd import ops
    from lumen_amd.services.face.backend import letterbox_geom

    g, _ = letterbox_geom(img.shape[0], img.shape[1], 0, S)
    return ops.image_prep([torch.from_numpy(img)], (S, S), mean=tuple(MEAN_BGR), std=(1.0,) * 3, scale=1.0,
                          filter="cv2_linear", layout="nchw", pad=0.0, geoms=[g], swap_rb=True)


def decode_priors_np(loc, conf, land, scale, thresh):
    pr = numpy_priors(S)
    sc = conf[:, 1]
    keep = sc >= thresh
    cx = pr[:, 0] + loc[:, 0] * 0.1 * pr[:, 2]
    cy = pr[:, 1] + loc[:, 1] * 0.1 * pr[:, 3]
    w = pr[:, 2] * np.exp(loc[:, 2] * 0.2)
    h = pr[:, 3] * np.exp(loc[:, 3] * 0.2)
    b = np.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1) * S / scale
    lm = np.stack([(pr[:, k % 2] + land[:, k] * 0.1 * pr[:, 2 + k % 2]) for k in range(10)], 1) * S / scale
    return b[keep], sc[keep], lm[keep]


def _backend(tmp_path, encoding):
    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.common import load_model_resources
    from lumen_amd.services.face.backend import MI355XFaceBackend

    write_retinaface_pack(tmp_path / "models" / f"retinaface_{encoding}", encoding=encoding, size=S)
    res = load_model_resources(tmp_path, ModelConfig(model=f"retinaface_{encoding}", runtime=Runtime.onnx))
    return MI355XFaceBackend(res, device="cpu"), tmp_path / "models" / f"retinaface_{encoding}"


def _faces(be, img, thresh):
    from lumen_amd.services.face.backend import DetParams

    return be.detect_images([img], [DetParams(conf=thresh, nms=1.0, size_min=0.0, size_max=1e9)])[0]


@pytest.mark.parametrize("side", [S, 2 * S])
def test_retinaface_prior_pack_matches_numpy_decode(tmp_path, side):
    from lumen_amd.services.face.onnx_pack import OnnxBoxDetector

    be, root = _backend(tmp_path, "priors")
    be.initialize()
    try:
        assert isinstance(be.det, OnnxBoxDetector) and be.det.kind == "priors" and be.spec.det_bgr
        img = np.random.default_rng(side).integers(0, 255, (side, side, 3), dtype=np.uint8)
        thresh = 0.55
        faces = _faces(be, img, thresh)
        loc, conf, land = [o[0].numpy() for o in OnnxGraph(root / "onnx" / "detection.fp32.onnx")
                           .run({"x": graph_input(img)})]
        assert loc.shape[0] == len(numpy_priors(S))
        rb, rs, rl = decode_priors_np(loc, conf, land, S / side, thresh)
        assert len(rs) > 0 and len(faces) == len(rs)
        ref = np.concatenate([np.clip(rb, 0, side), rs[:, None], rl], 1)
        got = np.array([list(f.bbox) + [f.confidence] + list(np.ravel(f.landmarks)) for f in faces])
        ref = ref[np.lexsort(np.round(ref[:, ::-1], 2).T)]
        got = got[np.lexsort(np.round(got[:, ::-1], 2).T)]
        np.testing.assert_allclose(got[:, 4], ref[:, 4], atol=1e-4)
        np.testing.assert_allclose(got[:, :4], ref[:, :4], atol=0.05 * side / S)
        np.testing.assert_allclose(got[:, 5:], ref[:, 5:], atol=0.05 * side / S)
    finally:
        be.close()


def test_decoded_pack_matches_graph_boxes(tmp_path):
    from lumen_amd.services.face.onnx_pack import OnnxBoxDetector

    be, root = _backend(tmp_path, "decoded")
    be.initialize()
    try:
        assert isinstance(be.det, OnnxBoxDetector) and be.det.kind == "decoded"
        img = np.random.default_rng(7).integers(0, 255, (2 * S, 2 * S, 3), dtype=np.uint8)
        thresh = 0.55
        faces = _faces(be, img, thresh)
        boxes, scores, lms = [o[0].numpy() for o in OnnxGraph(root / "onnx" / "detection.fp32.onnx")
                              .run({"x": graph_input(img)})]
        keep = scores >= thresh
        assert keep.sum() > 0 and len(faces) == keep.sum()
        ref = np.clip(boxes[keep] * 2.0, 0, 2 * S)
        got = np.array(sorted([f.bbox for f in faces]))
        np.testing.assert_allclose(got, np.array(sorted(ref.tolist())), atol=0.1)
        e = be.face_to_embedding(cropped_face_array=np.zeros((112, 112, 3), np.uint8))
        assert e.shape == (512,) and abs(float(np.linalg.norm(e)) - 1) < 1e-4
    finally:
        be.close()


def test_det_decode_boxes_normalised_to_original():
    """Reference ``normalized_boxes``: boxes in [0, 1] of the ORIGINAL image, whatever the
    letterbox scale; landmarks likewise."""
    from lumen_amd.ops import vision

    sc = torch.tensor([[0.9, 0.2, 0.7]])
    bb = torch.tensor([[[0.1, 0.2, 0.5, 0.6], [0.0, 0.0, 1.0, 1.0], [0.5, 0.5, 0.9, 0.8]]])
    kp = torch.rand(1, 3, 10)
    cand = torch.zeros(1, 16, 16)
    cnt = torch.zeros(1, dtype=torch.int32)
    vision.det_decode_boxes(sc, bb, kp, 0.5, torch.tensor([0.25]), torch.tensor([[300.0, 400.0]]), cand, cnt,
                            (-1.0, -1.0))
    assert int(cnt[0]) == 2
    rows = cand[0, :2].numpy()
    np.testing.assert_allclose(rows[0, :4], [40, 60, 200, 180], atol=1e-3)
    np.testing.assert_allclose(rows[1, :4], [200, 150, 360, 240], atol=1e-3)
    np.testing.assert_allclose(rows[0, 5:15:2], kp[0, 0, 0::2].numpy() * 400, atol=1e-3)
    np.testing.assert_allclose(rows[0, 6:16:2], kp[0, 0, 1::2].numpy() * 300, atol=1e-3)


def test_retinaface_priors_layout():
    from lumen_amd.ops.vision import retinaface_priors

    got = retinaface_priors((S, S)).numpy()
    np.testing.assert_allclose(got, numpy_priors(S), atol=1e-6)
    assert got.shape == (2 * sum((S // s) ** 2 for s in STEPS), 4)
