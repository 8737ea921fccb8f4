"""MI355X OCR backend (L2): DBNet detection -> geometry -> batched crops -> SVTR CTC.

Behaviour of the reference ``OnnxOcrBackend``
(packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py:43-632):

* configs from ``model_info.extra_metadata.{det_config, rec_config}`` with the same
  defaults (det ImageNet mean/std on BGR, scale 1/255, ``limit_side_len`` 960,
  ``thresh`` 0.3, ``box_thresh`` 0.6, ``unclip_ratio`` 1.5; rec mean/std 0.5,
  ``image_shape`` [3, 48, 320]) — :242-268;
* vocabulary file + optional space, blank inserted at index 0 — :103-114;
* det: resize so the long side <= limit, each side rounded to x32 (cv2 linear),
  normalise, DBNet, threshold bitmap -> components -> min-area rect -> box score ->
  unclip -> min-area rect -> rescale/clip (host C++ ``lumen_db_boxes``) — :318-476;
* reading-order sort — :478-494;
* crop: perspective warp of each quad (cubic, border replicate), rotate 90 deg if
  h/w >= 1.5, resize to height 48 keeping aspect — :496-594;
* greedy CTC, mean max-prob confidence, ``score >= rec_threshold`` kept — :596-632.

MI355X design: detection images of equal resized shape share one forward; the prob
map is the only D2H copy on the det side; every text crop of every image in the
batch is produced by ONE perspective-warp kernel that fuses the crop, the optional
rotation and the height-48 resize into a single 3x3 inverse map (one cubic
resampling instead of the reference's warp + resize pair) and writes bf16 NHWC8
directly into width-bucketed recogniser batches; the recogniser runs per bucket
with padded time steps masked in attention (kv_len) and in the CTC collapse (tlen);
softmax is fused into the CTC arg-max kernel.
"""
from __future__ import annotations

import contextlib

import json
import os
import logging
import math
import time
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ... import ops
from ...models.ocr import DBNet, DBNetConfig, RecConfig, SVTRRecognizer
from ...ops import vision
from ...resources.exceptions import ResourceNotFoundError
from ...runtime.batcher import DynamicBatcher
from ...runtime.metrics import stage
from ...utils.image import decode_rgb
from ..common import BackendInfo, GenericResources, load_safetensors, pick_device, runtime_name

log = logging.getLogger("lumen.ocr.backend")


class BackendError(Exception):
    pass


class BackendNotInitializedError(BackendError):
    pass


class InvalidInputError(BackendError):
    pass


class ModelLoadingError(BackendError):
    pass


@dataclass
class OcrResult:
    box: list            # [(x, y)] * 4, clockwise from top-left, source-image pixels
    text: str
    confidence: float


@dataclass
class OcrParams:
    det_thresh: float = 0.3
    rec_thresh: float = 0.5
    box_thresh: float = 0.6
    unclip_ratio: float = 1.5
    use_angle_cls: bool = False


DET_DEFAULTS = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225], "scale": 1.0 / 255.0,
                "limit_side_len": 960, "thresh": 0.3, "box_thresh": 0.6, "unclip_ratio": 1.5}
REC_DEFAULTS = {"mean": [0.5, 0.5, 0.5], "std": [0.5, 0.5, 0.5], "scale": 1.0 / 255.0, "image_shape": [3, 48, 320]}


def det_resize_shape(h: int, w: int, limit: int) -> tuple[int, int]:
    """Reference _det_preprocess (onnxrt_backend.py:338-360)."""
    ratio = 1.0
    if max(h, w) > limit:
        ratio = float(limit) / h if h > w else float(limit) / w
    rh, rw = int(h * ratio), int(w * ratio)
    rh = max(int(round(rh / 32) * 32), 32)
    rw = max(int(round(rw / 32) * 32), 32)
    return rh, rw


def sorted_boxes(boxes: Sequence[np.ndarray]) -> list[np.ndarray]:
    """Reference _sorted_boxes (:478-494): by (y, x) of the first point, then a bubble pass
    swapping neighbours on the same line (|dy| < 10) into left-to-right order."""
    b = sorted(boxes, key=lambda x: (x[0][1], x[0][0]))
    for i in range(len(b) - 1):
        for j in range(i, -1, -1):
            if abs(b[j + 1][0][1] - b[j][0][1]) < 10 and b[j + 1][0][0] < b[j][0][0]:
                b[j], b[j + 1] = b[j + 1], b[j]
            else:
                break
    return b


def _perspective(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """3x3 homography mapping 4 src points to 4 dst points (cv2.getPerspectiveTransform)."""
    A, bvec = [], []
    for (x, y), (u, v) in zip(src.astype(np.float64), dst.astype(np.float64)):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y]); bvec.append(u)
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y]); bvec.append(v)
    try:
        h = np.linalg.solve(np.array(A), np.array(bvec))
    except np.linalg.LinAlgError:
        h = np.linalg.lstsq(np.array(A), np.array(bvec), rcond=None)[0]
    return np.append(h, 1.0).reshape(3, 3)


def crop_maps(boxes: Sequence[np.ndarray], rec_h: int) -> tuple[np.ndarray, np.ndarray]:
    """:func:`crop_map` of many boxes at once (batched homography solves and inverses: per-crop
    Python cost was ~15 ms per 320-crop batch) -> (minv [n, 3, 3] f32, resize_w [n] int)."""
    n = len(boxes)
    if n == 0:
        return np.zeros((0, 3, 3), np.float32), np.zeros((0,), np.int64)
    pts = np.stack([np.asarray(b, np.float32) for b in boxes])                       # [n, 4, 2]
    cw = np.maximum(np.linalg.norm(pts[:, 0] - pts[:, 1], axis=1), np.linalg.norm(pts[:, 2] - pts[:, 3], axis=1))
    ch = np.maximum(np.linalg.norm(pts[:, 0] - pts[:, 3], axis=1), np.linalg.norm(pts[:, 1] - pts[:, 2], axis=1))
    cw = np.maximum(cw.astype(np.int64), 1)
    ch = np.maximum(ch.astype(np.int64), 1)
    dst = np.zeros((n, 4, 2), np.float32)
    dst[:, 1, 0] = cw
    dst[:, 2, 0] = cw
    dst[:, 2, 1] = ch
    dst[:, 3, 1] = ch
    src64, dst64 = pts.astype(np.float64), dst.astype(np.float64)
    x, y, u, v = src64[..., 0], src64[..., 1], dst64[..., 0], dst64[..., 1]
    A = np.zeros((n, 8, 8), np.float64)
    A[:, 0::2, 0], A[:, 0::2, 1], A[:, 0::2, 2] = x, y, 1
    A[:, 0::2, 6], A[:, 0::2, 7] = -u * x, -u * y
    A[:, 1::2, 3], A[:, 1::2, 4], A[:, 1::2, 5] = x, y, 1
    A[:, 1::2, 6], A[:, 1::2, 7] = -v * x, -v * y
    bvec = np.zeros((n, 8), np.float64)
    bvec[:, 0::2], bvec[:, 1::2] = u, v
    try:
        h = np.linalg.solve(A, bvec[..., None])[..., 0]
        Hm = np.concatenate([h, np.ones((n, 1))], 1).reshape(n, 3, 3)
        Minv = np.linalg.inv(Hm)
    except np.linalg.LinAlgError:     # a degenerate box in the batch: the per-box path (lstsq fallback)
        out = [crop_map(b, rec_h) for b in boxes]
        return np.stack([o[0] for o in out]), np.array([o[1] for o in out], np.int64)
    rot = ch * 1.0 / cw >= 1.5
    R = np.tile(np.eye(3), (n, 1, 1))
    R[rot] = 0.0
    R[rot, 0, 1], R[rot, 0, 2], R[rot, 1, 0], R[rot, 2, 2] = -1.0, cw[rot] - 1, 1.0, 1.0
    wr, hr = np.where(rot, ch, cw), np.where(rot, cw, ch)
    resize_w = np.maximum(1, np.ceil(wr * rec_h / hr).astype(np.int64))
    sx, sy = wr / resize_w, hr / rec_h
    S = np.zeros((n, 3, 3), np.float64)
    S[:, 0, 0], S[:, 0, 2] = sx, 0.5 * sx - 0.5
    S[:, 1, 1], S[:, 1, 2] = sy, 0.5 * sy - 0.5
    S[:, 2, 2] = 1.0
    return (Minv @ R @ S).astype(np.float32), resize_w


def crop_map(box: np.ndarray, rec_h: int) -> tuple[np.ndarray, int]:
    """Inverse map (rec-input pixel -> source pixel) fusing the reference's perspective crop,
    rot90 for tall crops and the height-``rec_h`` resize; returns (minv 3x3, resize_w)."""
    pts = box.astype(np.float32)
    cw = int(max(np.linalg.norm(pts[0] - pts[1]), np.linalg.norm(pts[2] - pts[3])))
    ch = int(max(np.linalg.norm(pts[0] - pts[3]), np.linalg.norm(pts[1] - pts[2])))
    cw, ch = max(cw, 1), max(ch, 1)
    dst = np.array([[0, 0], [cw, 0], [cw, ch], [0, ch]], np.float32)
    Minv = np.linalg.inv(_perspective(pts, dst))            # crop pixel -> source pixel
    rot = ch * 1.0 / cw >= 1.5
    if rot:   # np.rot90 (CCW): rotated (x, y) = crop (cw - 1 - y, x); rotated is ch wide, cw high
        R = np.array([[0, -1, cw - 1], [1, 0, 0], [0, 0, 1]], np.float64)
        wr, hr = ch, cw
    else:
        R = np.eye(3)
        wr, hr = cw, ch
    resize_w = max(1, math.ceil(wr * rec_h / hr))
    sx, sy = wr / resize_w, hr / rec_h                       # cv2 linear resize, half-pixel centres
    S = np.array([[sx, 0, 0.5 * sx - 0.5], [0, sy, 0.5 * sy - 0.5], [0, 0, 1]], np.float64)
    return (Minv @ R @ S).astype(np.float32), resize_w


class MI355XOcrBackend:
    def __init__(self, resources: GenericResources, device: Optional[str] = None, max_batch: int = 16,
                 max_wait_ms: float = 2.0, rec_batch: int = 256, bucket: int = 32,
                 dp_devices: Optional[Sequence[str]] = None):
        self.resources = resources
        self.dp_devices = list(dp_devices or [])
        self._pool = None
        self.device_pref = device
        self.max_batch = max_batch
        self.max_wait_ms = max_wait_ms
        self.rec_batch = rec_batch
        self.bucket = bucket
        self.is_initialized = False
        self.load_time = 0.0
        self.det: Optional[DBNet] = None
        self.rec: Optional[SVTRRecognizer] = None
        self._batcher: Optional[DynamicBatcher] = None
        self.character_str: list[str] = []

    # ------------------------------------------------------------------ lifecycle
    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        r = self.resources
        extra = r.extra
        self.det_config = {**DET_DEFAULTS, **(extra.get("det_config") or {})}
        self.rec_config = {**REC_DEFAULTS, **(extra.get("rec_config") or {})}
        try:
            vocab_path = r.get_model_file(self.rec_config.get("character_dict_path", "ppocr_keys_v1.txt"))
            lines = vocab_path.read_bytes().decode("utf-8").split("\n")
            if lines and lines[-1] == "":
                lines = lines[:-1]
            chars = [ln.strip("\r") for ln in lines]
        except Exception as e:
            raise ModelLoadingError(f"Failed to load vocab file: {e}") from e
        if self.rec_config.get("use_space_char", True):
            chars.append(" ")
        self.character_str = ["blank"] + chars
        cfgp = r.model_root_path / "lumen_ocr_config.json"
        from ...parallel.engine import current_remote

        remote = current_remote()
        if remote is not None:
            # serving front end (parallel/engine.py): DBNet + SVTR live in the GPU engine processes;
            # request batches (JPEG bytes + parameters) are shipped there whole
            self.device = torch.device("cpu")
            self.dtype = torch.float32
            self._pool = remote

            def rfn(items):
                with stage("dp_forward"):
                    return remote.submit("ocr", list(items)).result()

            self._batcher = DynamicBatcher(rfn, self.max_batch, self.max_wait_ms, "ocr-remote", 2 * remote.size)
            self.load_time = time.time() - t0
            self.is_initialized = True
            log.info("OCR %s served by %d GPU engine(s)", r.model_name, remote.size)
            return
        self.device = pick_device(self.device_pref)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        if len(self.dp_devices) > 1:
            # one DBNet + SVTR per GPU worker (dp_worker); batches go whole to the least-loaded
            # worker, 2 in flight per GPU, JPEG decode on the workers
            from ...parallel.worker_pool import GPUWorkerPool

            self._pool = GPUWorkerPool("lumen_amd.services.ocr.backend:dp_worker", self.dp_devices,
                                       kwargs={"resources": r, "max_batch": self.max_batch})
            pool = self._pool

            def fn(items):
                with stage("dp_forward"):
                    return pool.submit("ocr", list(items)).result()

            self._batcher = DynamicBatcher(fn, self.max_batch, self.max_wait_ms, "ocr-dp", 2 * pool.size)
            self.load_time = time.time() - t0
            self.is_initialized = True
            log.info("OCR %s ready on %d DP workers %s in %.2fs", r.model_name, pool.size, self.dp_devices,
                     self.load_time)
            return
        if cfgp.exists():
            meta = json.loads(cfgp.read_text())
            dcfg = DBNetConfig(**{k: _tup(v) for k, v in meta["det"].items()})
            rcfg = RecConfig(**{k: _tup(v) for k, v in meta["rec"].items()})
            det, rec = DBNet(dcfg), SVTRRecognizer(rcfg)
            try:
                det.load_state_dict(load_safetensors(r.get_model_file("detection.safetensors")))
                rec.load_state_dict(load_safetensors(r.get_model_file("recognition.safetensors")))
            except Exception as e:
                raise ModelLoadingError(f"Initialization failed: {e}") from e
        else:
            # the reference's PP-OCR ONNX pack, run by the MI355X graph executor
            from .onnx_pack import OnnxCTCRecognizer, OnnxDBNet, find_onnx_pair

            dpath, rpath = find_onnx_pair(r.model_root_path)
            if dpath is None or rpath is None:
                raise ResourceNotFoundError(f"{r.model_name}: neither lumen_ocr_config.json (+ safetensors) nor a "
                                            f"detection/recognition ONNX pair found in {r.model_root_path}")
            det, rec = OnnxDBNet(dpath, self.device), OnnxCTCRecognizer(rpath, self.device)
        self.det, self.rec = det.to(self.device).eval(), rec.to(self.device).eval()
        self.rec_h = int(self.rec_config["image_shape"][1])
        self._batcher = DynamicBatcher(self._predict_batch, self.max_batch, self.max_wait_ms, "ocr")
        self.load_time = time.time() - t0
        self.is_initialized = True
        log.info("OCR %s ready on %s in %.2fs (%d classes)", r.model_name, self.device, self.load_time,
                 len(self.character_str))

    def close(self) -> None:
        if self._batcher is not None:
            self._batcher.close()
        if self._pool is not None:
            self._pool.close()
            self._pool = None

    # ------------------------------------------------------------------ detection
    @torch.no_grad()
    def detect(self, images: Sequence[np.ndarray], params: Sequence[OcrParams]) -> list[list[np.ndarray]]:
        """decoded RGB images -> per image list of int boxes [4, 2] in reading order."""
        return self.detect_finish(self.detect_submit(images, params))

    @torch.no_grad()
    def decode_device(self, datas: Sequence[bytes]):
        """A batch of encoded images -> (images, pre): baseline JPEGs entropy-decoded on the host
        pool and reconstructed on the GPU in one batched launch (utils/jpeg.py), other formats through
        Pillow, every image in one flat device buffer -- the pixels never come back to the host.
        ``images[k]`` is a shape-only :class:`~lumen_amd.utils.jpeg.DeviceImage` (or the
        InvalidInputError of an undecodable payload); ``pre`` feeds :meth:`detect_submit`, whose
        upload the recogniser's crop warps then read as well."""
        from ...utils.jpeg import DeviceImage, decode_batch_to_device

        with stage("decode"):
            flat, offs, shapes, errors = decode_batch_to_device(list(datas), self.device)
        images = [InvalidInputError(f"Failed to decode image bytes: {errors[k]}") if k in errors
                  else DeviceImage(*shapes[k]) for k in range(len(datas))]
        return images, (flat, [int(o) for o in offs])

    def detect_submit(self, images: Sequence[np.ndarray], params: Sequence[OcrParams], stream=None,
                      pre=None) -> dict:
        """The device half of :meth:`detect`, queued without waiting: one pinned upload of the batch,
        the resize / normalise and the detector forward per shape group, on ``stream`` (default: the
        current one).  :meth:`detect_finish` runs the DB post-processing.  Submitting batch i + 1 on its
        own stream while batch i is post-processed and recognised overlaps the detector with the host
        geometry and the recogniser (tools/face_ocr_bench.py --what ocr).  ``pre``: the (flat device
        buffer, offsets) of :meth:`decode_device` (queued on the same stream) instead of an upload."""
        dc = self.det_config
        limit = int(dc["limit_side_len"])
        shapes = [det_resize_shape(im.shape[0], im.shape[1], limit) for im in images]
        groups: dict = {}
        for i, s in enumerate(shapes):
            groups.setdefault(s, []).append(i)
        h = {"images": list(images), "params": list(params), "groups": [], "upload": None, "event": None}
        cuda = self.device.type == "cuda"
        ctx = torch.cuda.stream(stream) if (cuda and stream is not None) else contextlib.nullcontext()
        with ctx:
            src, offs = None, None
            if cuda:
                # one pinned H2D for the whole batch; every shape group's resize and the
                # recogniser's crop warps (recognize) read the images from this upload
                if pre is not None:
                    src, offs = pre
                else:
                    if getattr(self, "_uploader", None) is None:
                        from ...utils.image import PinnedUploader

                        self._uploader = PinnedUploader(self.device)
                    with stage("upload"):
                        src, offs = self._uploader.upload(images)
                # (strong refs to the images: recognize matches them by identity)
                h["upload"] = (list(images), src, [int(o) for o in offs])
                self._last_upload = h["upload"]
            for (rh, rw), idx in groups.items():
                geoms, off, tens = [], 0, []
                for i in idx:
                    hh, ww = images[i].shape[:2]
                    geoms.append(ops.ImageGeom.resize(hh, ww, int(offs[i]) if src is not None else off, rh, rw))
                    off += images[i].size
                    tens.append(torch.empty(images[i].shape, dtype=torch.uint8, device="meta") if pre is not None
                                else torch.from_numpy(np.ascontiguousarray(images[i])))
                with stage("det_preprocess"):
                    x = ops.image_prep(tens, (rh, rw), mean=dc["mean"], std=dc["std"], scale=float(dc["scale"]),
                                       filter="cv2_linear", layout="nhwc8", swap_rb=True, geoms=geoms,
                                       out_dtype=self.dtype, device=self.device, src=src)
                with stage("det_forward"):
                    prob = self.det(x)
                h["groups"].append((rh, rw, idx, prob))
            if cuda:
                h["event"] = torch.cuda.Event()
                h["event"].record()
        return h

    @torch.no_grad()
    def detect_finish(self, h: dict, on_gpu_done=None) -> list[list[np.ndarray]]:
        """DB post-processing of a :meth:`detect_submit` handle on the current stream -> per image list
        of int boxes.  ``on_gpu_done()`` is called once the first group's connected components are
        back on the host (the GPU is then free for the next batch's detector)."""
        images, params = h["images"], h["params"]
        out: list = [None] * len(images)
        if h["event"] is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(h["event"])
            for _, _, _, prob in h["groups"]:
                prob.record_stream(cur)
            if h["upload"] is not None:
                h["upload"][1].record_stream(cur)
        for gi, (rh, rw, idx, prob) in enumerate(h["groups"]):
            with stage("db_post"):
                out_g = self._db_post(prob, [images[i].shape[:2] for i in idx], [params[i] for i in idx], rh, rw,
                                      on_gpu_done=on_gpu_done if gi == 0 else None)
            for i, bx in zip(idx, out_g):
                out[i] = bx
        if on_gpu_done is not None and not h["groups"]:
            on_gpu_done()
        return out

    def _db_post(self, prob: torch.Tensor, hw, params, rh: int, rw: int, on_gpu_done=None) -> list:
        """DB post-processing of a [n, rh, rw] probability batch -> boxes in reading order.
        On the GPU: threshold + connected components + boundary extraction + box scores run on
        the device (ops.vision.db_boxes_gpu), only boundary pixels and scores come back."""
        if prob.is_cuda:
            return [sorted_boxes(list(b)) for b, _ in vision.db_boxes_gpu(prob, params, hw, rh, rw,
                                                                          on_gpu_done=on_gpu_done)]
        if on_gpu_done is not None:
            on_gpu_done()
        pm = prob.float().cpu().numpy()
        res = []
        for j, ((h, w), p) in enumerate(zip(hw, params)):
            boxes, _ = vision.db_boxes(pm[j], thresh=p.det_thresh, box_thresh=p.box_thresh,
                                       unclip_ratio=p.unclip_ratio, scale_xy=(w / rw, h / rh), src_wh=(w, h))
            res.append(sorted_boxes(list(boxes)))
        return res

    # ------------------------------------------------------------------ recognition
    @torch.no_grad()
    def recognize(self, images: Sequence[np.ndarray], crops: Sequence[tuple[int, np.ndarray]],
                  upload: Optional[tuple] = None) -> list[tuple[str, float]]:
        """crops: (image index, box [4, 2]) -> (text, confidence) per crop.  ``upload``: the
        :meth:`detect_submit` handle's upload of these images (default: the last one)."""
        if not crops:
            return []
        rc = self.rec_config
        H = self.rec_h
        minvs, rws = crop_maps([b for _, b in crops], H)
        maps = [(minvs[k], int(rws[k])) for k in range(len(crops))]
        order = sorted(range(len(crops)), key=lambda k: maps[k][1])
        res: list = [None] * len(crops)
        mean = float(np.mean(rc["mean"]))
        std = float(np.mean(rc["std"]))
        scale = float(rc["scale"])
        src = None
        last = upload if upload is not None else getattr(self, "_last_upload", None)
        if last is not None and len(last[0]) == len(images) and all(a is b for a, b in zip(last[0], images)):
            src = (last[1], last[2])        # the detector's upload of these same images
        for s in range(0, len(order), self.rec_batch):
            chunk = order[s:s + self.rec_batch]
            widths = [maps[k][1] for k in chunk]
            Wb = max(self.bucket, -(-max(widths) // self.bucket) * self.bucket)
            minv = np.stack([maps[k][0] for k in chunk])
            with stage("crop_warp"):
                x = vision.warp_batch(images, [crops[k][0] for k in chunk], minv, (H, Wb), out_w=widths, cpad=8,
                                      scale=scale / std, mean=mean / std, std=1.0, swap_rb=True, cubic=True,
                                      replicate=True, device=self.device, src=src)
                if x.dtype != self.dtype:
                    x = x.to(self.dtype)
            if hasattr(self.rec, "ctc_from_features"):
                with stage("rec_forward"):
                    hn, nb, nt = self.rec.features(x, valid_w=widths)
                with stage("ctc"):          # classifier + greedy CTC fused on the GPU (no logits stored)
                    ids, conf = self.rec.ctc_from_features(hn, nb, nt, widths, blank=0)
            else:                           # ONNX-pack recogniser: logits graph output
                with stage("rec_forward"):
                    logits = self.rec(x, valid_w=widths)
                ts = self.rec.time_stride
                with stage("ctc"):
                    ids, conf = vision.ctc_greedy(logits, blank=0, from_logits=True,
                                                  tlen=[-(-w // ts) for w in widths])
            for k, seq, c in zip(chunk, ids, conf):
                res[k] = ("".join(self.character_str[i] for i in seq if 0 < i < len(self.character_str)), float(c))
        return res

    # ------------------------------------------------------------------ end to end
    def _predict_batch(self, items, pre=None):
        """(image, OcrParams) items -> per image list of OcrResult; ``pre``: the images' device buffer
        from :meth:`decode_device` (the images are then its shape-only stand-ins)."""
        imgs = [it[0] for it in items]
        params = [it[1] for it in items]
        h = self.detect_submit(imgs, params, pre=pre)
        boxes = self.detect_finish(h)
        crops = [(i, b) for i, bs in enumerate(boxes) for b in bs]
        texts = self.recognize(imgs, crops, upload=h["upload"])
        outs: list = [[] for _ in items]
        for (i, b), (text, score) in zip(crops, texts):
            if score >= params[i].rec_thresh:
                outs[i].append(OcrResult(box=[(int(x), int(y)) for x, y in b.tolist()], text=text,
                                         confidence=min(max(score, 0.0), 1.0)))
        return outs

    def _ensure(self):
        if not self.is_initialized:
            raise BackendNotInitializedError("Backend not initialized")

    def predict(self, image_bytes: bytes, det_threshold: float = 0.3, rec_threshold: float = 0.5,
                use_angle_cls: bool = False, **kwargs) -> list[OcrResult]:
        self._ensure()
        if not image_bytes:
            raise InvalidInputError("Failed to decode image bytes")
        img = None
        if self._pool is None:
            try:
                with stage("decode"):
                    img = decode_rgb(image_bytes)
            except ValueError as e:
                raise InvalidInputError(f"Failed to decode image bytes: {e}") from e
        p = OcrParams(det_thresh=float(det_threshold), rec_thresh=float(rec_threshold),
                      box_thresh=float(kwargs.get("box_thresh", self.det_config["box_thresh"])),
                      unclip_ratio=float(kwargs.get("unclip_ratio", self.det_config["unclip_ratio"])),
                      use_angle_cls=bool(use_angle_cls))
        return self._batcher((img if img is not None else bytes(image_bytes), p))

    def get_info(self) -> BackendInfo:
        r = self.resources
        dev = getattr(self, "device", None)
        cuda = dev is not None and dev.type == "cuda"
        return BackendInfo(runtime=runtime_name(dev) if dev is not None else "mi355x-hip",
                           device=str(dev or self.device_pref), model_id=r.model_id, model_name=r.model_name,
                           version=r.model_info.version, precisions=("bf16",) if cuda or dev is None else ("fp32",),
                           extra={"det_model_id": f"{r.model_info.name}_det", "rec_model_id": f"{r.model_info.name}_rec",
                                  "num_classes": str(len(self.character_str)),
                                  "limit_side_len": str(getattr(self, "det_config", DET_DEFAULTS)["limit_side_len"])})


def _tup(v):
    if isinstance(v, list):
        return tuple(_tup(x) for x in v)
    return v


def create_backend(settings, resources: GenericResources, runtime: Optional[str] = None) -> MI355XOcrBackend:
    """Factory (reference backends/factory.py:75-146: only onnx registered; torch accepted here)."""
    rt = runtime or resources.runtime
    if rt not in ("onnx", "torch", "rknn"):
        raise ValueError(f"unsupported runtime '{rt}'")
    if rt == "rknn":
        raise BackendError("RKNN runtime is not available on MI355X builds")
    from ...resources.config import AmdRuntimeSettings

    from ...runtime import placement

    amd = AmdRuntimeSettings.from_env()
    dev = getattr(settings, "device", None) if settings is not None else None
    dev, dp_devs = placement.resolve(dev, placement.dp_size_env())
    return MI355XOcrBackend(resources, device=dev, max_batch=min(amd.max_batch, 16), max_wait_ms=amd.max_wait_ms,
                            dp_devices=dp_devs)


def engine_spec(resources: GenericResources, max_batch: int = 16) -> tuple:
    """(factory path, kwargs) of the GPU engine side (parallel/engine.py): :func:`dp_worker`."""
    return "lumen_amd.services.ocr.backend:dp_worker", {"resources": resources, "max_batch": max_batch}


def dp_worker(device: str, resources: GenericResources, max_batch: int = 16):
    """GPUWorkerPool factory: DBNet + SVTR on ``device``; fn("ocr", [(jpeg bytes, OcrParams)])
    -> per image list of OcrResult (decode failures -> InvalidInputError for that image)."""
    b = MI355XOcrBackend(resources, device=device, max_batch=max_batch)
    b.initialize()

    def fn(kind, items):
        if kind != "ocr":
            raise ValueError(f"unknown OCR task kind {kind!r}")
        out: list = [None] * len(items)
        if b.device.type == "cuda" and items and all(not isinstance(p, np.ndarray) for p, _ in items):
            # a merged batch of encoded images: one device JPEG decode (host entropy decode + one GPU
            # reconstruction), the detector and the crop warps read the pixels where they landed
            imgs, (flat, offs) = b.decode_device([bytes(p) for p, _ in items])
            ok = [k for k, im in enumerate(imgs) if not isinstance(im, Exception)]
            for k, im in enumerate(imgs):
                if isinstance(im, Exception):
                    out[k] = im
            if ok:
                res = b._predict_batch([(imgs[k], items[k][1]) for k in ok], pre=(flat, [offs[k] for k in ok]))
                for k, r in zip(ok, res):
                    out[k] = r
            return out
        ok = []
        for k, (payload, _) in enumerate(items):
            if isinstance(payload, np.ndarray):
                out[k] = payload
                ok.append(k)
                continue
            try:
                out[k] = decode_rgb(payload)
                ok.append(k)
            except ValueError as e:
                out[k] = InvalidInputError(f"Failed to decode image bytes: {e}")
        if ok:
            res = b._predict_batch([(out[k], items[k][1]) for k in ok])
            for k, r in zip(ok, res):
                out[k] = r
        return out

    return fn
