"""Detection / recognition post-processing ops.

GPU: the HIP kernels of csrc/postproc.hip (anchor/prior decode + threshold + rescale +
size filter, NMS, batched warp into recogniser batches, CTC greedy decode).
CPU: numpy references with the reference's semantics.  Host C++ (csrc/host/geometry.cpp)
serves the DB-net contour geometry and the 5-point similarity transform on both paths.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch

from .._native import hip_ops, load_host
from ..runtime.metrics import stage
from ..utils.h2d import h2d

# ArcFace 5-point template for 112x112 crops (insightface canonical coordinates)
ARCFACE_DST = np.array([[38.2946, 51.6963], [73.5318, 51.5014], [56.0252, 71.7366], [41.5493, 92.3655],
                        [70.7299, 92.2041]], dtype=np.float32)


# --------------------------------------------------------------------------- decode + NMS
def det_decode_head(head: torch.Tensor, A: int, stride: int, thresh: float, img_scale: torch.Tensor,
                    img_hw: torch.Tensor, cand: torch.Tensor, count: torch.Tensor, min_size: float = 0.0,
                    max_size: float = 1e9, with_kps: bool = True) -> None:
    """SCRFD head of one stride, fused NHWC conv output [N, H, W, Ch] (fp32) with channels
    [0:A] class logits, [A:5A] bbox distances, [5A:15A] keypoint distances.  Survivors
    (sigmoid(score) >= thresh, size-filtered, un-letterboxed) are appended to
    ``cand`` [N, max_cand, 16] / ``count`` [N] int32."""
    N, H, W, Ch = head.shape
    P = H * W * A
    if head.is_cuda:
        h = head.float().contiguous()
        hip_ops().det_decode(h, h[..., A:], h[..., 5 * A:] if with_kps else None, None, int(H), int(W), int(A),
                             int(stride), float(thresh), img_scale.float().contiguous(), img_hw.float().contiguous(),
                             float(min_size), float(max_size), 0.1, 0.2, 0.0, 0.0, cand, count, int(P),
                             int(H * W * Ch), int(Ch), True)
        return
    hf = head.float().reshape(N, H * W, Ch)
    scores = torch.sigmoid(hf[..., :A]).reshape(N, P)
    bbox = hf[..., A:5 * A].reshape(N, P, 4)
    kps = hf[..., 5 * A:15 * A].reshape(N, P, 10) if with_kps else None
    _decode_ref(scores, bbox, kps, H, W, A, stride, thresh, img_scale, img_hw, cand, count, min_size, max_size)


def det_decode_priors(scores, bbox, kps, priors, thresh, img_scale, img_hw, cand, count, in_wh, var=(0.1, 0.2),
                      min_size=0.0, max_size=1e9):
    """RetinaFace-style outputs: scores [N, P] (probabilities), bbox deltas [N, P, 4],
    landmark deltas [N, P, 10] against priors [P, 4] (cx, cy, w, h, normalised)."""
    N, P = scores.shape
    if scores.is_cuda:
        hip_ops().det_decode(scores.float().contiguous(), bbox.float().contiguous(),
                             kps.float().contiguous() if kps is not None else None, priors.float().contiguous(),
                             0, 0, 1, 0, float(thresh), img_scale.float().contiguous(), img_hw.float().contiguous(),
                             float(min_size), float(max_size), float(var[0]), float(var[1]), float(in_wh[0]),
                             float(in_wh[1]), cand, count, int(P), 0, 0, False)
        return
    _decode_ref(scores.float(), bbox.float(), kps.float() if kps is not None else None, 0, 0, 1, 0, thresh,
                img_scale, img_hw, cand, count, min_size, max_size, priors=priors, var=var, in_wh=in_wh)


def det_decode_boxes(scores, bbox, kps, thresh, img_scale, img_hw, cand, count, in_wh=(1.0, 1.0),
                     min_size=0.0, max_size=1e9):
    """Already-decoded detector outputs (generic / RetinaFace exports with the decode in the graph;
    reference onnxrt_backend.py:810-880): scores [N, P] (probabilities), boxes [N, P, 4]
    (x1, y1, x2, y2) and landmarks [N, P, 10] in network-input pixels times ``in_wh`` -- (1, 1)
    for pixel outputs, (S, S) for outputs normalised to the input -- or, with ``in_wh`` = (-1, -1),
    normalised to the ORIGINAL image (reference ``normalized_boxes``).  Same candidate rows,
    un-letterbox, clip and size filter as the anchor / prior decodes."""
    N, P = scores.shape
    if scores.is_cuda:
        hip_ops().det_decode(scores.float().contiguous(), bbox.float().contiguous(),
                             kps.float().contiguous() if kps is not None else None, None,
                             0, 0, 1, -1, float(thresh), img_scale.float().contiguous(), img_hw.float().contiguous(),
                             float(min_size), float(max_size), 0.0, 0.0, float(in_wh[0]), float(in_wh[1]),
                             cand, count, int(P), 0, 0, False)
        return
    _decode_ref(scores.float(), bbox.float(), kps.float() if kps is not None else None, 0, 0, 1, -1, thresh,
                img_scale, img_hw, cand, count, min_size, max_size, in_wh=in_wh)


def retinaface_priors(in_hw, steps=(8, 16, 32), min_sizes=((16, 32), (64, 128), (256, 512)),
                      clip: bool = False) -> torch.Tensor:
    """RetinaFace prior boxes [P, 4] (cx, cy, w, h) normalised to the network input: per level
    (step, sizes) a ceil(H / step) x ceil(W / step) grid, every cell emitting one square prior per
    size, in (row, column, size) order -- the layout RetinaFace heads are flattened in."""
    H, W = int(in_hw[0]), int(in_hw[1])
    out = []
    for step, sizes in zip(steps, min_sizes):
        fh, fw = -(-H // step), -(-W // step)
        ys, xs = torch.meshgrid(torch.arange(fh, dtype=torch.float32), torch.arange(fw, dtype=torch.float32),
                                indexing="ij")
        cx = ((xs + 0.5) * step / W).reshape(-1, 1)
        cy = ((ys + 0.5) * step / H).reshape(-1, 1)
        for_sizes = []
        for ms in sizes:
            wh = torch.tensor([ms / W, ms / H], dtype=torch.float32).expand(cx.shape[0], 2)
            for_sizes.append(torch.cat([cx, cy, wh], 1))
        out.append(torch.stack(for_sizes, 1).reshape(-1, 4))
    pr = torch.cat(out)
    return pr.clamp(0, 1) if clip else pr


def _decode_ref(sc, bb, kp, H, W, A, stride, thresh, img_scale, img_hw, cand, count, min_size, max_size,
                priors=None, var=(0.1, 0.2), in_wh=(0.0, 0.0)):
    N, P = sc.shape
    decoded = priors is None and stride < 0
    for n in range(N):
        s_img = float(img_scale[n])
        ih, iw = float(img_hw[n, 0]), float(img_hw[n, 1])
        fx = (iw * s_img if in_wh[0] < 0 else in_wh[0]) if decoded else 0.0
        fy = (ih * s_img if in_wh[1] < 0 else in_wh[1]) if decoded else 0.0
        for i in torch.nonzero(sc[n] >= thresh).flatten().tolist():
            d = bb[n, i]
            if decoded:
                cx = cy = 0.0
                x1, y1, x2, y2 = d[0] * fx, d[1] * fy, d[2] * fx, d[3] * fy
            elif priors is None:
                loc = i // A
                cx, cy = float((loc % W) * stride), float((loc // W) * stride)
                x1, y1, x2, y2 = cx - d[0] * stride, cy - d[1] * stride, cx + d[2] * stride, cy + d[3] * stride
            else:
                pr = priors[i].float()
                cx = pr[0] + d[0] * var[0] * pr[2]
                cy = pr[1] + d[1] * var[0] * pr[3]
                pw, ph = pr[2] * torch.exp(d[2] * var[1]), pr[3] * torch.exp(d[3] * var[1])
                x1, y1 = (cx - pw / 2) * in_wh[0], (cy - ph / 2) * in_wh[1]
                x2, y2 = (cx + pw / 2) * in_wh[0], (cy + ph / 2) * in_wh[1]
            x1 = min(max(float(x1) / s_img, 0.0), iw); x2 = min(max(float(x2) / s_img, 0.0), iw)
            y1 = min(max(float(y1) / s_img, 0.0), ih); y2 = min(max(float(y2) / s_img, 0.0), ih)
            fw, fh = x2 - x1, y2 - y1
            if min(fw, fh) < min_size or max(fw, fh) > max_size:
                continue
            slot = int(count[n])
            count[n] += 1
            if slot >= cand.shape[1]:
                continue
            row = [x1, y1, x2, y2, float(sc[n, i])]
            if kp is not None:
                for k in range(5):
                    if decoded:
                        kx, ky = kp[n, i, 2 * k] * fx, kp[n, i, 2 * k + 1] * fy
                    elif priors is None:
                        kx, ky = cx + kp[n, i, 2 * k] * stride, cy + kp[n, i, 2 * k + 1] * stride
                    else:
                        pr = priors[i].float()
                        kx = (pr[0] + kp[n, i, 2 * k] * var[0] * pr[2]) * in_wh[0]
                        ky = (pr[1] + kp[n, i, 2 * k + 1] * var[0] * pr[3]) * in_wh[1]
                    row += [float(kx) / s_img, float(ky) / s_img]
            else:
                row += [-1.0] * 10
            row.append(0.0)
            cand[n, slot] = torch.tensor(row)


def nms_ref(boxes: np.ndarray, scores: np.ndarray, thr: float) -> np.ndarray:
    if len(boxes) == 0:
        return np.zeros((0,), np.int32)
    x1, y1, x2, y2 = boxes.T
    areas = (x2 - x1) * (y2 - y1)
    order = scores.argsort()[::-1]
    keep = []
    while order.size > 0:
        i = int(order[0])
        keep.append(i)
        xx1 = np.maximum(x1[i], x1[order[1:]]); yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]]); yy2 = np.minimum(y2[i], y2[order[1:]])
        inter = np.maximum(0.0, xx2 - xx1) * np.maximum(0.0, yy2 - yy1)
        iou = inter / (areas[i] + areas[order[1:]] - inter + 1e-8)
        order = order[np.where(iou <= thr)[0] + 1]
    return np.array(keep, dtype=np.int32)


NMS_ASYNC_ROWS = 64     # kept rows per image gathered + copied before the host looks at the counts


def nms_async(cand: torch.Tensor, count: torch.Tensor, iou_thr: float, max_out: int = 1024):
    """Queue per-image NMS on the stream without waiting: the kernel, a device gather of each
    image's first NMS_ASYNC_ROWS kept rows and ONE non-blocking D2H of (counts, rows) into pinned
    memory.  :func:`nms_wait` returns what :func:`nms` does; only an image that kept more rows
    than the gathered window costs a second (synchronous) copy.  A pipelined caller queues batch
    i + 1's detector behind this and parses batch i on the host while it runs."""
    N, MC, C = cand.shape
    keep = torch.empty((N, max_out), dtype=torch.int32, device=cand.device)
    keep_n = torch.empty((N,), dtype=torch.int32, device=cand.device)
    hip_ops().nms(cand, count, float(iou_thr), keep, keep_n)
    w = min(NMS_ASYNC_ROWS, max_out)
    # slots past an image's count hold stale indices: clamp them into range, the host drops them
    idx = keep[:, :w].long().clamp_(0, MC - 1)
    rows = torch.gather(cand, 1, idx.unsqueeze(-1).expand(N, w, C))
    host_rows = torch.empty((N, w, C), dtype=cand.dtype, pin_memory=True)
    host_n = torch.empty((N,), dtype=torch.int32, pin_memory=True)
    host_rows.copy_(rows, non_blocking=True)
    host_n.copy_(keep_n, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return cand, keep, host_rows, host_n, ev


def nms_wait(h):
    """Host half of :func:`nms_async`: waits for the copy, per image kept rows [k, 16]."""
    cand, keep, host_rows, host_n, ev = h
    ev.synchronize()
    counts = host_n.tolist()
    w = host_rows.shape[1]
    out = [host_rows[n, :min(c, w)] for n, c in enumerate(counts)]
    big = [n for n, c in enumerate(counts) if c > w]
    for n in big:       # rare: an image kept more rows than the window -- fetch the rest
        rest = cand[n, keep[n, w:counts[n]].long()].cpu()
        out[n] = torch.cat([out[n], rest])
    return out


def nms(cand: torch.Tensor, count: torch.Tensor, iou_thr: float, max_out: int = 1024):
    """Per-image NMS -> list (per image) of kept candidate rows [k, 16] (score-descending)."""
    N, MC, _ = cand.shape
    if cand.is_cuda:
        # kept rows gathered on the device, then ONE small copy: the whole candidate block
        # (N x MC x 64 B, MBs for a batch) never crosses to the host
        return nms_wait(nms_async(cand, count, iou_thr, max_out))
    out = []
    for n in range(N):
        c = min(int(count[n]), MC)
        rows = cand[n, :c].numpy()
        k = nms_ref(rows[:, :4], rows[:, 4], iou_thr)[:max_out]
        out.append(torch.from_numpy(rows[k]))
    return out


# --------------------------------------------------------------------------- warps
def similarity_transform(src: np.ndarray, dst: np.ndarray = ARCFACE_DST) -> np.ndarray:
    """2x3 similarity (rotation + uniform scale + translation) least-squares src -> dst."""
    lib = load_host()
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 2)
    dst = np.ascontiguousarray(dst, np.float32).reshape(-1, 2)
    M = np.zeros((2, 3), np.float32)
    if lib is not None:
        fp = ctypes.POINTER(ctypes.c_float)
        lib.lumen_similarity_transform(src.ctypes.data_as(fp), dst.ctypes.data_as(fp), ctypes.c_int(len(src)),
                                       M.ctypes.data_as(fp))
        return M
    mx, my = src.mean(0)
    ux, uy = dst.mean(0)
    a_ = src - [mx, my]
    b_ = dst - [ux, uy]
    sxx = (b_[:, 0] * a_[:, 0]).sum(); sxy = (b_[:, 0] * a_[:, 1]).sum()
    syx = (b_[:, 1] * a_[:, 0]).sum(); syy = (b_[:, 1] * a_[:, 1]).sum()
    var = (a_ ** 2).sum()
    a, b = sxx + syy, syx - sxy
    nrm = np.hypot(a, b)
    sc = nrm / var if var > 0 else 1.0
    c, s = (a / nrm, b / nrm) if nrm > 0 else (1.0, 0.0)
    M[0] = [sc * c, -sc * s, 0]
    M[1] = [sc * s, sc * c, 0]
    M[0, 2] = ux - (M[0, 0] * mx + M[0, 1] * my)
    M[1, 2] = uy - (M[1, 0] * mx + M[1, 1] * my)
    return M


def invert_affine(M: np.ndarray) -> np.ndarray:
    A = np.vstack([M.astype(np.float64), [0, 0, 1]])
    return np.linalg.inv(A).astype(np.float32)


def warp_batch(images: Sequence[np.ndarray], img_index: Sequence[int], minv: np.ndarray, out_hw: tuple,
               out_w: Optional[Sequence[int]] = None, cpad: int = 8, scale: float = 1 / 127.5, mean: float = 1.0,
               std: float = 1.0, swap_rb: bool = True, cubic: bool = False, device=None,
               replicate: bool = False, src=None) -> torch.Tensor:
    """Warp F crops (inverse 3x3 maps ``minv`` [F, 3, 3], dst->src) from uint8 RGB images into
    bf16 NHWC [F, OH, OW, cpad]: value = (px * scale - mean) / std, channels reversed if swap_rb.
    Default = ArcFace preprocessing (x/127.5 - 1 == (x/255 - 0.5)/0.5, BGR).  ``replicate``
    selects cv2 BORDER_REPLICATE instead of the constant-0 border."""
    F = len(img_index)
    OH, OW = out_hw
    ow = list(out_w) if out_w is not None else [OW] * F
    device = torch.device(device) if device is not None else torch.device("cpu")
    if device.type == "cuda":
        if src is not None:             # (flat device uint8 tensor, offsets) of an earlier upload
            src, offs = src
        else:
            offs, flat = [], []
            off = 0
            for im in images:
                offs.append(off)
                flat.append(torch.from_numpy(np.ascontiguousarray(im)).reshape(-1))
                off += im.size
            src = h2d(torch.cat(flat), device)
        meta = h2d([[offs[i], images[i].shape[0], images[i].shape[1], ow[f]] for f, i in enumerate(img_index)],
                   device, torch.long)
        mv = h2d(np.ascontiguousarray(minv, np.float32).reshape(F, 9), device)
        out = torch.empty((F, OH, OW, cpad), device=device, dtype=torch.bfloat16)
        hip_ops().warp_batch(src, meta, mv, out, float(scale), float(mean), float(std), bool(swap_rb), bool(cubic),
                             bool(replicate))
        return out
    out = torch.zeros((F, OH, OW, cpad), dtype=torch.float32)
    ys, xs = np.mgrid[0:OH, 0:OW].astype(np.float32)
    for f, i in enumerate(img_index):
        im = images[i].astype(np.float32)
        h, w = im.shape[:2]
        M = np.asarray(minv[f], np.float64).reshape(3, 3)
        X = M[0, 0] * xs + M[0, 1] * ys + M[0, 2]
        Y = M[1, 0] * xs + M[1, 1] * ys + M[1, 2]
        Z = M[2, 0] * xs + M[2, 1] * ys + M[2, 2]
        sx, sy = X / Z, Y / Z
        acc = np.zeros((OH, OW, 3), np.float64)
        x0, y0 = np.floor(sx).astype(np.int64), np.floor(sy).astype(np.int64)
        fx, fy = sx - x0, sy - y0
        taps = range(-1, 3) if cubic else range(0, 2)
        for dy in taps:
            for dx in taps:
                xx, yy = x0 + dx, y0 + dy
                ok = (xx >= 0) & (yy >= 0) & (xx < w) & (yy < h)
                if replicate:
                    ok = np.ones_like(ok)
                if cubic:
                    wt = _cub(dx - fx) * _cub(dy - fy)
                else:
                    wt = (fx if dx else 1 - fx) * (fy if dy else 1 - fy)
                px = im[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)]
                acc += np.where(ok[..., None], wt[..., None] * px, 0.0)
        px = np.clip(np.rint(acc), 0, 255)
        if swap_rb:
            px = px[..., ::-1]
        v = (px * scale - mean) / std
        v[:, ow[f]:] = 0
        out[f, :, :, :3] = torch.from_numpy(v.astype(np.float32))
    return out.to(torch.bfloat16)


def _cub(x):
    a = -0.75
    x = np.abs(x)
    return np.where(x < 1, ((a + 2) * x - (a + 3)) * x * x + 1, np.where(x < 2, (((x - 5) * x + 8) * x - 4) * a, 0.0))


# --------------------------------------------------------------------------- CTC
def ctc_greedy(probs: torch.Tensor, blank: int = 0, from_logits: bool = False,
               tlen: Optional[Sequence[int]] = None):
    """probs [B, T, C] (softmax output, or raw logits with ``from_logits``) -> (ids list per
    sequence, mean confidence per sequence).  ``tlen`` limits each sequence to its valid
    time steps (width-padded recogniser batches)."""
    B, T, C = probs.shape
    if probs.is_cuda:
        ids = torch.empty((B, T), dtype=torch.int32, device=probs.device)
        ln = torch.empty((B,), dtype=torch.int32, device=probs.device)
        cf = torch.empty((B,), dtype=torch.float32, device=probs.device)
        tl = torch.tensor(list(tlen), dtype=torch.int32).to(probs.device) if tlen is not None else None
        hip_ops().ctc_greedy(probs.float().contiguous(), int(blank), ids, ln, cf, bool(from_logits), tl)
        ids, ln, cf = ids.cpu(), ln.cpu(), cf.cpu()
        return [ids[b, : int(ln[b])].tolist() for b in range(B)], cf.tolist()
    p = torch.softmax(probs.float(), -1) if from_logits else probs.float()
    conf, idx = p.max(dim=-1)
    seqs, confs = [], []
    for b in range(B):
        out, cs, prev = [], [], -1
        for t in range(T if tlen is None else min(int(tlen[b]), T)):
            c = int(idx[b, t])
            if c != blank and c != prev:
                out.append(c)
                cs.append(float(conf[b, t]))
            prev = c
        seqs.append(out)
        confs.append(float(np.mean(cs)) if cs else 0.0)
    return seqs, confs


def cls_ctc_greedy(h: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], num_classes: int, B: int, T: int,
                   blank: int = 0, tlen: Optional[Sequence[int]] = None):
    """Classifier + greedy CTC with the logits never stored (GPU): h [B*T, K] bf16 features,
    w [N, K] bf16 classifier, bias f32 [N]; classes >= num_classes are ignored.  Same result as
    ``ctc_greedy(h @ w.T + bias, from_logits=True)``."""
    dev = h.device
    M = B * T
    i1 = torch.empty(M, dtype=torch.int32, device=dev)
    c1 = torch.empty(M, dtype=torch.float32, device=dev)
    ids = torch.empty((B, T), dtype=torch.int32, device=dev)
    ln = torch.empty((B,), dtype=torch.int32, device=dev)
    cf = torch.empty((B,), dtype=torch.float32, device=dev)
    tl = h2d(list(tlen), dev, torch.int32) if tlen is not None else None
    b = bias.float().contiguous() if bias is not None else None
    hip_ops().cls_ctc(h.contiguous(), w.contiguous(), b, int(num_classes), int(B), int(T), int(blank), tl, i1, c1,
                      ids, ln, cf)
    ids, ln, cf = ids.cpu(), ln.cpu(), cf.cpu()
    return [ids[k, : int(ln[k])].tolist() for k in range(B)], cf.tolist()


# --------------------------------------------------------------------------- DB post-processing (GPU + host)
def db_boxes_gpu(prob: torch.Tensor, params: Sequence, hw: Sequence, rh: int, rw: int, max_candidates: int = 1000,
                 min_size: int = 3, max_boxes: int = 1000, cap: Optional[int] = None, on_gpu_done=None) -> list:
    """Batched DB post-processing of a device probability batch [n, rh, rw]: GPU threshold +
    connected components + boundary extraction (db_post.hip), host hull / min-area rect on
    the boundary pixels, GPU box score, host unclip / order / rescale.  ``params[j]`` has
    ``det_thresh`` / ``box_thresh`` / ``unclip_ratio``; ``hw[j]`` is the source (h, w).
    Returns per image (boxes [k, 4, 2] int32, scores [k]) -- the same boxes as :func:`db_boxes`.
    Components too small on both axes to pass ``min_size`` are dropped on the GPU, before the
    ``max_candidates`` cut (the host path counts them; only maps with > max_candidates
    components -- noise -- can differ)."""
    lib = load_host()
    if lib is None:
        raise RuntimeError("lumen host library (_lumen_host.so) not built")
    n = prob.shape[0]
    prob = prob.contiguous()
    if prob.dtype not in (torch.bfloat16, torch.float32):
        prob = prob.float()
    dev = prob.device
    thr = h2d([float(p.det_thresh) for p in params], dev, torch.float32)
    cap = cap or max(1 << 16, n * rh * rw // 4)
    lab = torch.empty(5 * n * rh * rw, dtype=torch.int32, device=dev)     # labels + per-root bbox
    pts = torch.empty((cap, 3), dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    with stage("db_gpu"):
        hip_ops().db_components(prob, thr, lab, pts, cnt, int(min_size))
        K = int(cnt.item())
    if K > cap:                                      # pathological maps: retry with room for every pixel
        return db_boxes_gpu(prob, params, hw, rh, rw, max_candidates, min_size, max_boxes, cap=n * rh * rw,
                            on_gpu_done=on_gpu_done)
    if on_gpu_done is not None:                      # the device-heavy part is done: e.g. queue the next batch
        on_gpu_done()
    with stage("db_points"):
        P = np.ascontiguousarray(pts[:K].cpu().numpy())
        if K > 1:                                    # group by component: host radix sort (csrc/host/geometry.cpp)
            lib.lumen_sort_points_by_root(P.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.c_int(K))
    HW = rh * rw
    ip = ctypes.POINTER(ctypes.c_int)
    fp = ctypes.POINTER(ctypes.c_float)
    per_img = []
    all_q, all_r, all_i = [], [], []
    starts = np.searchsorted(P[:, 0], np.arange(n + 1) * HW) if K else np.zeros(n + 1, np.int64)
    def cand(j):
        seg = np.ascontiguousarray(P[starts[j]:starts[j + 1]])
        mx = max_candidates
        q = np.zeros((mx, 8), np.float32)
        r = np.zeros((mx, 5), np.float32)
        roots = np.zeros((mx,), np.int32)
        m = lib.lumen_db_candidates(seg.ctypes.data_as(ip), ctypes.c_int(len(seg)), ctypes.c_int(max_candidates),
                                    ctypes.c_int(min_size), q.ctypes.data_as(fp), r.ctypes.data_as(fp),
                                    roots.ctypes.data_as(ip), ctypes.c_int(mx)) if len(seg) else 0
        return q[:m], r[:m], m

    with stage("db_cand"):   # per-image hulls / min-area rects: the C++ calls release the GIL
        res = list(_host_pool().map(cand, range(n))) if n > 1 else [cand(0)]
    for j, (q, r, m) in enumerate(res):
        all_q.append(q)
        all_r.append(r)
        all_i.append(np.full(m, j, np.int32))
        per_img.append(m)
    Q = np.concatenate(all_q) if all_q else np.zeros((0, 8), np.float32)
    scores = np.zeros((len(Q),), np.float32)
    if len(Q):
        with stage("db_score"):
            sc = torch.empty(3 * len(Q), dtype=torch.float32, device=dev)
            hip_ops().db_quad_score(prob, h2d(Q, dev), h2d(np.concatenate(all_i), dev),
                                    sc)
            scores = sc[:len(Q)].cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(per_img)]).astype(np.int64)

    def fin(j):
        m = per_img[j]
        h, w = hw[j]
        boxes = np.zeros((max_boxes, 8), np.float32)
        bs = np.zeros((max_boxes,), np.float32)
        R = np.ascontiguousarray(all_r[j])
        S = np.ascontiguousarray(scores[offs[j]:offs[j] + m])
        k = lib.lumen_db_finalize(R.ctypes.data_as(fp), S.ctypes.data_as(fp), ctypes.c_int(m),
                                  ctypes.c_float(params[j].box_thresh), ctypes.c_float(params[j].unclip_ratio),
                                  ctypes.c_int(min_size), ctypes.c_float(w / rw), ctypes.c_float(h / rh),
                                  ctypes.c_int(w), ctypes.c_int(h), boxes.ctypes.data_as(fp), bs.ctypes.data_as(fp),
                                  ctypes.c_int(max_boxes)) if m else 0
        return boxes[:k].reshape(k, 4, 2).astype(np.int32), bs[:k]

    return list(_host_pool().map(fin, range(n))) if n > 1 else [fin(0)]


_HOST_POOL = None


def _host_pool():
    """Threads for the per-image DB host geometry (hull, min-area rect, unclip: C++ calls that
    release the GIL).  Its own pool: a caller may itself be running on the image decode pool."""
    global _HOST_POOL
    if _HOST_POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _HOST_POOL = ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4), thread_name_prefix="lumen-db")
    return _HOST_POOL


# --------------------------------------------------------------------------- DB post-processing (host C++)
def db_boxes(prob: np.ndarray, thresh: float = 0.3, box_thresh: float = 0.6, unclip_ratio: float = 1.5,
             max_candidates: int = 1000, min_size: int = 3, scale_xy=(1.0, 1.0), src_wh=(0, 0),
             max_boxes: int = 1000):
    """Probability map [H, W] -> (boxes [n, 4, 2] int, scores [n])."""
    lib = load_host()
    if lib is None:
        raise RuntimeError("lumen host library (_lumen_host.so) not built")
    prob = np.ascontiguousarray(prob, np.float32)
    H, W = prob.shape
    boxes = np.zeros((max_boxes, 8), np.float32)
    scores = np.zeros((max_boxes,), np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    n = lib.lumen_db_boxes(prob.ctypes.data_as(fp), ctypes.c_int(H), ctypes.c_int(W), ctypes.c_float(thresh),
                           ctypes.c_float(box_thresh), ctypes.c_float(unclip_ratio), ctypes.c_int(max_candidates),
                           ctypes.c_int(min_size), ctypes.c_float(scale_xy[0]), ctypes.c_float(scale_xy[1]),
                           ctypes.c_int(src_wh[0] or W), ctypes.c_int(src_wh[1] or H), boxes.ctypes.data_as(fp),
                           scores.ctypes.data_as(fp), ctypes.c_int(max_boxes))
    return boxes[:n].reshape(n, 4, 2).astype(np.int32), scores[:n]
