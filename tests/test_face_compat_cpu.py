"""Reference-compatible face alignment (``LUMEN_FACE_ALIGN=reference``), pinned against a
NumPy re-derivation of the reference pipeline:

  face_model.crop_face_from_image  (face_model.py:429-470): int bbox, clipped, img[y1:y2, x1:x2]
  _align_face_5points              (onnxrt_backend.py:1382-1417): similarity from the ORIGINAL-
                                   image landmarks onto the 96-wide template, warpAffine of the
                                   CROP, INTER_LINEAR, BORDER_CONSTANT 0, 112x112
  _preprocess_recognition          (onnxrt_backend.py:1351-1380): (x/255 - 0.5)/0.5, RGB->BGR

cv2 is not importable here, so the reference's warpAffine / resize are re-derived in NumPy
(float64); estimateAffinePartial2D on five consistent points is the least-squares similarity
(solved below with lstsq), see SURVEY §A.6 Q8/Q9."""
import numpy as np
import pytest

from lumen_amd.ops import vision
from lumen_amd.services.face.backend import MI355XFaceBackend

TEMPLATE96 = np.array([[30.2946, 51.6963], [65.5318, 51.5014], [48.0252, 71.7366], [33.5493, 92.3655],
                       [62.7299, 92.2041]], np.float64)


def _lsq_similarity(src, dst):
    # [x -y 1 0; y x 0 1] [a b tx ty]^T = dst
    A, rhs = [], []
    for (x, y), (u, v) in zip(src, dst):
        A += [[x, -y, 1, 0], [y, x, 0, 1]]
        rhs += [u, v]
    a, b, tx, ty = np.linalg.lstsq(np.asarray(A), np.asarray(rhs), rcond=None)[0]
    return np.array([[a, -b, tx], [b, a, ty]])


def _bilinear(img, sx, sy, border):
    h, w = img.shape[:2]
    x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
    fx, fy = sx - x0, sy - y0
    out = np.zeros(sx.shape + (3,))
    for dy, wy in ((0, 1 - fy), (1, fy)):
        for dx, wx in ((0, 1 - fx), (1, fx)):
            xx, yy = x0 + dx, y0 + dy
            if border == "replicate":
                v = img[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)]
            else:
                ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
                v = np.where(ok[..., None], img[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], 0.0)
            out += (wx * wy)[..., None] * v
    return out


def reference_input(img, bbox, landmarks):
    h, w = img.shape[:2]
    x1, y1, x2, y2 = map(int, bbox)
    x1, x2 = max(0, min(x1, w)), max(0, min(x2, w))
    y1, y2 = max(0, min(y1, h)), max(0, min(y2, h))
    crop = img[y1:y2, x1:x2].astype(np.float64)
    ys, xs = np.mgrid[0:112, 0:112].astype(np.float64)
    if landmarks is not None:
        M = np.vstack([_lsq_similarity(np.asarray(landmarks, np.float64), TEMPLATE96), [0, 0, 1]])
        Mi = np.linalg.inv(M)                   # warpAffine: dst pixel -> src = M^-1 (x, y, 1)
        aligned = _bilinear(crop, Mi[0, 0] * xs + Mi[0, 1] * ys + Mi[0, 2], Mi[1, 0] * xs + Mi[1, 1] * ys + Mi[1, 2],
                            "constant")
    else:                                       # cv2.resize INTER_LINEAR, half-pixel centres
        ch, cw = crop.shape[:2]
        aligned = _bilinear(crop, (xs + 0.5) * cw / 112 - 0.5, (ys + 0.5) * ch / 112 - 0.5, "replicate")
    aligned = np.clip(np.rint(aligned), 0, 255)   # cv2 writes the warped / resized image as uint8
    x = (aligned / 255.0 - 0.5) / 0.5
    return x[..., ::-1]                         # RGB -> BGR


class _Res:
    extra = {"face_align": "reference"}


def _backend(bgr=True):
    b = MI355XFaceBackend(_Res(), device="cpu")
    b.spec.rec_color = "bgr" if bgr else "rgb"
    b.device = __import__("torch").device("cpu")
    return b


def _ours(b, img, bbox, lm):
    src, minv, rep = b._reference_crop(img, lm, bbox)
    x = b.warp_faces([src], [0], minv[None], [rep])
    return x[0, :, :, :3].float().numpy()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_reference_alignment_geometry(seed):
    rng = np.random.default_rng(seed)
    H, W = 220, 260
    yy, xx = np.mgrid[0:H, 0:W]
    img = np.stack([(xx * 1.3 + yy * 0.4) % 256, (yy * 1.1) % 256, rng.integers(0, 256, (H, W))], -1).astype(np.uint8)
    bbox = (35.7 + rng.uniform(0, 10), 28.2 + rng.uniform(0, 10), 171.9 - rng.uniform(0, 10), 199.6)
    # landmarks in ORIGINAL-image coordinates (inside the bbox), as the detector reports them
    base = np.array([[80, 90], [125, 88], [102, 118], [85, 150], [122, 148]], np.float64)
    lm = [tuple(p) for p in base + rng.normal(0, 2.0, base.shape)]
    b = _backend()
    ref = reference_input(img, bbox, lm)
    ours = _ours(b, img, bbox, lm)
    # bf16 recogniser input: a uint8 rounding flip (2/255) + bf16 rounding at worst, ~exact on average
    d = np.abs(ours - ref)
    assert d.max() < 3 / 255 and d.mean() < 1e-3, (d.max(), d.mean())
    # the standard mode (landmarks in the full image, 112 template) is a different image
    std = _backend()
    std.align_mode, std.template = "standard", vision.ARCFACE_DST
    minv = std._minv_for(img, lm, bbox)
    xs = std.warp_faces([img], [0], minv[None])[0, :, :, :3].float().numpy()
    assert np.abs(xs - ref).max() > 0.1


def test_reference_resize_without_landmarks():
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (90, 120, 3)).astype(np.uint8)
    b = _backend()
    for bbox in [(10.9, 5.2, 100.1, 85.7), (30, 20, 70, 60)]:        # down- and up-scaling crops
        ref = reference_input(img, bbox, None)
        ours = _ours(b, img, bbox, None)
        d = np.abs(ours - ref)
        assert d.max() < 3 / 255 and d.mean() < 1e-3, (d.max(), d.mean())


def test_empty_crop_gives_zero_vector():
    b = _backend()
    assert b._reference_crop(np.zeros((50, 50, 3), np.uint8), None, (60, 10, 80, 30)) is None
