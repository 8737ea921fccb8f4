"""Split DB post-processing (GPU labelling path, csrc/db_post.hip + host candidates/finalize)
reproduces the one-shot host path (lumen_db_boxes) when the labelling is emulated on the CPU
(scipy 8-connected components, root = first pixel in raster order, boundary = any 4-neighbour
outside).  GPU twin: tests/test_postproc_gpu.py::test_db_boxes_gpu_matches_host."""
import ctypes

import numpy as np
import pytest
from scipy import ndimage

from lumen_amd._native import load_host
from lumen_amd.ops import vision


def _blob_map(seed, H=96, W=160):
    rng = np.random.default_rng(seed)
    m = np.zeros((H, W), np.float32)
    for _ in range(7):
        x0, y0 = rng.integers(0, W - 30), rng.integers(0, H - 12)
        w, h = rng.integers(8, 30), rng.integers(4, 12)
        m[y0:y0 + h, x0:x0 + w] = rng.uniform(0.5, 0.95)
    return m + rng.uniform(0, 0.2, (H, W)).astype(np.float32)


def _emulated_points(prob, thresh):
    H, W = prob.shape
    fg = prob > thresh
    lab, n = ndimage.label(fg, structure=np.ones((3, 3)))
    idx = np.arange(H * W).reshape(H, W)
    root = np.zeros(n + 1, np.int64)
    for c in range(1, n + 1):
        root[c] = idx[lab == c].min()
    pad = np.pad(fg, 1)
    interior = fg & pad[:-2, 1:-1] & pad[2:, 1:-1] & pad[1:-1, :-2] & pad[1:-1, 2:]
    interior[0, :] = interior[-1, :] = interior[:, 0] = interior[:, -1] = False
    ys, xs = np.nonzero(fg & ~interior)
    pts = np.stack([root[lab[ys, xs]], xs, ys], 1).astype(np.int32)
    return pts[np.argsort(pts[:, 0], kind="stable")]


def _in_quad_mean(prob, q):
    H, W = prob.shape
    xs, ys = q[0::2], q[1::2]
    x0, x1 = max(0, int(np.floor(xs.min()))), min(W - 1, int(np.ceil(xs.max())))
    y0, y1 = max(0, int(np.floor(ys.min()))), min(H - 1, int(np.ceil(ys.max())))
    s = c = 0.0
    for yy in range(y0, y1 + 1):
        for xx in range(x0, x1 + 1):
            cr = [(xs[(k + 1) % 4] - xs[k]) * (yy - ys[k]) - (ys[(k + 1) % 4] - ys[k]) * (xx - xs[k]) for k in range(4)]
            if not (any(v > 0 for v in cr) and any(v < 0 for v in cr)):
                s += prob[yy, xx]
                c += 1
    return s / c if c else 0.0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_split_host_path_matches_one_shot(seed):
    lib = load_host()
    if lib is None:
        pytest.skip("host library not built")
    prob = _blob_map(seed)
    H, W = prob.shape
    ref_b, ref_s = vision.db_boxes(prob, thresh=0.3, box_thresh=0.5, unclip_ratio=1.5, scale_xy=(2.0, 2.0),
                                   src_wh=(2 * W, 2 * H))
    pts = np.ascontiguousarray(_emulated_points(prob, 0.3))
    ip, fp = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)
    q = np.zeros((1000, 8), np.float32)
    r = np.zeros((1000, 5), np.float32)
    roots = np.zeros(1000, np.int32)
    m = lib.lumen_db_candidates(pts.ctypes.data_as(ip), len(pts), 1000, 3, q.ctypes.data_as(fp), r.ctypes.data_as(fp),
                                roots.ctypes.data_as(ip), 1000)
    scores = np.array([_in_quad_mean(prob, q[i]) for i in range(m)], np.float32)
    boxes = np.zeros((1000, 8), np.float32)
    bs = np.zeros(1000, np.float32)
    k = lib.lumen_db_finalize(r.ctypes.data_as(fp), scores.ctypes.data_as(fp), m, ctypes.c_float(0.5),
                              ctypes.c_float(1.5), 3, ctypes.c_float(2.0), ctypes.c_float(2.0), 2 * W, 2 * H,
                              boxes.ctypes.data_as(fp), bs.ctypes.data_as(fp), 1000)
    assert k == len(ref_b) > 0
    np.testing.assert_array_equal(boxes[:k].reshape(k, 4, 2).astype(np.int32), ref_b)
    np.testing.assert_allclose(bs[:k], ref_s, rtol=1e-5)


@pytest.mark.parametrize("K,maxroot", [(1, 5), (2, 1), (1000, 4095), (5000, 4096), (20000, 1 << 23), (3000, (1 << 24) + 7)])
def test_host_point_sort_is_stable_by_root(K, maxroot):
    """csrc/host/geometry.cpp lumen_sort_points_by_root (the LSD radix sort that replaced a device
    torch.sort of the DB points): rows grouped by root in ascending order, atomic append order kept
    within a root (np.argsort kind="stable" is the reference), every digit-pass count covered."""
    rng = np.random.default_rng(K)
    roots = rng.integers(0, maxroot + 1, K).astype(np.int32)
    roots[rng.integers(0, K)] = maxroot
    P = np.stack([roots, rng.integers(0, 4096, K), np.arange(K)], 1).astype(np.int32)   # y = append order
    ref = P[np.argsort(P[:, 0], kind="stable")]
    got = np.ascontiguousarray(P.copy())
    load_host().lumen_sort_points_by_root(got.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.c_int(K))
    np.testing.assert_array_equal(got, ref)
