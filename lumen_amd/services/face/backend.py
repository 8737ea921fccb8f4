"""MI355X face backend (L2): SCRFD detection + ArcFace IResNet embedding.

Contract of the reference ``FaceRecognitionBackend``
(packages/lumen-face/src/lumen_face/backends/base.py:107-308) and behaviour of its
ONNX backend (backends/onnxrt_backend.py:701-1417):

detection  decode -> letterbox (aspect kept, top-left, pad 0, cv2 linear) to the
           detector size -> (x - 127.5) / 128 -> SCRFD -> anchor-centre
           distance2bbox / distance2kps -> score >= threshold -> un-letterbox, clip ->
           size filter (min <= w, h <= max) -> greedy NMS (IoU <= thr kept).
embedding  optional 5-point similarity alignment onto the ArcFace 112x112 template,
           else a plain resize of the (cropped) face -> (x/255 - 0.5) / 0.5 ->
           IResNet -> L2-normalised fp32 vector.

MI355X design: ONE fused letterbox+normalise kernel for the whole image batch into
NHWC8 bf16, the detector's convs as implicit-GEMM MFMA kernels with BN/ReLU/residual
in the epilogue, all three strides' heads decoded+thresholded+size-filtered by one
kernel each and NMS'd on device; every face of every image in a batch is aligned by
ONE batched warp kernel straight from the decoded original (no PIL re-decode per face
— reference face_model.py:429-470) and embedded as ONE recogniser batch.  Concurrent
requests from all gRPC streams are merged by :class:`DynamicBatcher` (one device-owning
thread per model).

Deliberate fixes of reference quirks: alignment uses the landmarks in
the coordinate frame of the image they were detected in (the reference applies
original-image landmarks to the bbox crop, face_model.py:429-470 + onnxrt_backend.py:
1327-1332), and the canonical insightface 112x112 ArcFace template (the reference's
template is the 96-wide one without the +8 px x offset, onnxrt_backend.py:1388-1397).

Embedding compatibility (``LUMEN_FACE_ALIGN=reference``, or ``extra.face_align:
reference`` in model_info): reproduces the reference geometry exactly so vectors match
embeddings a reference deployment already stored — the face is cut out at its integer,
image-clipped bbox, the similarity transform is estimated from the ORIGINAL-image
landmarks onto the 96-wide template and applied to the CROP (border 0 at the crop's
edge), or the crop is resized to 112 when there are no landmarks; an empty crop yields a
zero vector.  ``LUMEN_FACE_REFERENCE_TEMPLATE=1`` switches the template only.

Data parallelism (BASELINE config 3; reference hot loop face_service.py:516-574 is
sequential per face): with more than one device (the hub's placement or
``LUMEN_DP_SIZE``) the backend owns a :class:`GPUWorkerPool`, one worker process per
GPU, each with its own detector + recogniser (:func:`dp_worker`).  Requests are batched
here and every batch goes whole to the least-loaded worker (two batches in flight per
GPU); the worker decodes the JPEGs on its own CPU threads and runs decode -> detect ->
align -> embed for the whole batch, so nothing but compressed bytes and (bbox,
landmarks, embedding) rows cross the process boundary.
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ... import ops
from ...models.face import IRESNET_PRESETS, SCRFD_PRESETS, IResNet, IResNetConfig, SCRFD, SCRFDConfig
from ...ops import vision
from ...resources.exceptions import ResourceNotFoundError
from ...runtime.batcher import DynamicBatcher
from ...runtime.metrics import stage
from ...utils.h2d import h2d
from ...utils.image import decode_rgb
from ..common import BackendInfo, GenericResources, load_safetensors, pick_device, runtime_name

log = logging.getLogger("lumen.face.backend")

MAX_CAND = 1024
REFERENCE_TEMPLATE = vision.ARCFACE_DST - np.array([8.0, 0.0], np.float32)


class BackendError(Exception):
    pass


class BackendNotInitializedError(BackendError):
    pass


class InvalidInputError(BackendError):
    pass


class InferenceError(BackendError):
    pass


class DeviceUnavailableError(BackendError):
    pass


@dataclass
class FaceDetection:
    """bbox (x1, y1, x2, y2) in original-image pixels, optional 5 landmarks, confidence."""

    bbox: tuple
    confidence: float
    landmarks: Optional[list] = None


@dataclass
class DetParams:
    conf: float = 0.7
    nms: float = 0.4
    size_min: float = 50.0
    size_max: float = 1000.0

    def key(self):
        return (self.conf, self.nms, self.size_min, self.size_max)


@dataclass
class FaceSpec:
    det_size: int = 640
    det_mean: float = 127.5
    det_std: float = 128.0
    rec_size: int = 112
    rec_mean: float = 127.5
    rec_std: float = 127.5
    rec_color: str = "rgb"
    align_landmarks: bool = True
    extra: dict = field(default_factory=dict)
    # per-channel detector normalisation in the model's channel order (RetinaFace: BGR 104/117/123, std 1)
    det_mean3: Optional[tuple] = None
    det_std3: Optional[tuple] = None
    det_bgr: bool = False


def letterbox_geom(h: int, w: int, off: int, S: int):
    """Reference _preprocess_detection sizes (onnxrt_backend.py:756-770): top-left, int()."""
    if h / w > 1.0:
        nh, nw = S, int(S / (h / w))
    else:
        nw, nh = S, int(S * (h / w))
    nh, nw = max(nh, 1), max(nw, 1)
    return ops.ImageGeom.letterbox(h, w, off, S, S, nh, nw), nh / h


def crop_minv(bbox, out: int) -> np.ndarray:
    """dst (out x out) -> src map of an integer bbox crop resized with cv2 linear (half-pixel)."""
    x1, y1, x2, y2 = [int(v) for v in bbox]
    bw, bh = max(x2 - x1, 1), max(y2 - y1, 1)
    sx, sy = bw / out, bh / out
    return np.array([[sx, 0, x1 + 0.5 * sx - 0.5], [0, sy, y1 + 0.5 * sy - 0.5], [0, 0, 1]], np.float32)


class MI355XFaceBackend:
    def __init__(self, resources: GenericResources, device: Optional[str] = None, max_batch: int = 64,
                 max_wait_ms: float = 2.0, max_faces_batch: int = 512, dp_devices: Optional[Sequence[str]] = None):
        self.resources = resources
        self.dp_devices = list(dp_devices or [])
        self._pool = None
        self._dp: dict = {}
        self.device_pref = device
        self.max_batch = max_batch
        self.max_wait_ms = max_wait_ms
        self.max_faces_batch = max_faces_batch
        self.det: Optional[SCRFD] = None
        self.rec: Optional[IResNet] = None
        self.spec = FaceSpec()
        self.is_initialized = False
        self.load_time = 0.0
        self._det_batcher: Optional[DynamicBatcher] = None
        self._emb_batcher: Optional[DynamicBatcher] = None
        self.align_mode = (os.environ.get("LUMEN_FACE_ALIGN") or
                           str((resources.extra or {}).get("face_align", "standard"))).lower()
        if self.align_mode not in ("standard", "reference"):
            raise ValueError(f"face_align must be 'standard' or 'reference', got {self.align_mode!r}")
        self.template = REFERENCE_TEMPLATE if (os.environ.get("LUMEN_FACE_REFERENCE_TEMPLATE") == "1" or
                                               self.align_mode == "reference") else vision.ARCFACE_DST

    # ------------------------------------------------------------------ lifecycle
    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        from ...parallel.engine import current_remote

        remote = current_remote()
        if remote is not None:
            # serving front end (parallel/engine.py): SCRFD + IResNet live in the GPU engine
            # processes; this process decodes the JPEGs and ships batches there
            self.device = torch.device("cpu")
            self._init_pool(remote)
            self.load_time = time.time() - t0
            self.is_initialized = True
            log.info("face pack %s served by %d GPU engine(s)", self.resources.model_name, remote.size)
            return
        self.device = pick_device(self.device_pref)
        if len(self.dp_devices) > 1:
            self._init_pool()
            self.load_time = time.time() - t0
            self.is_initialized = True
            log.info("face pack %s ready on %d DP workers %s in %.2fs", self.resources.model_name,
                     len(self.dp_devices), self.dp_devices, self.load_time)
            return
        r = self.resources
        cfgp = r.model_root_path / "lumen_face_config.json"
        from .specs import pack_spec

        spec = pack_spec(r.model_name, r.extra.get("insightface") or {})
        d, rc = spec["detection"], spec["recognition"]
        if cfgp.exists():
            import json

            meta = json.loads(cfgp.read_text())
            dcfg = SCRFDConfig(**{k: tuple(v) if isinstance(v, list) else v for k, v in meta["det"].items()})
            rcfg = IResNetConfig(**{k: tuple(v) if isinstance(v, list) else v for k, v in meta["rec"].items()})
            det, rec = SCRFD(dcfg), IResNet(rcfg)
            det.load_state_dict(load_safetensors(r.get_model_file("detection.safetensors")))
            rec.load_state_dict(load_safetensors(r.get_model_file("recognition.safetensors")))
            det_size, rec_size = dcfg.input_size, rcfg.input_size
        else:
            # the reference's InsightFace ONNX pack, run by the MI355X graph executor
            from .onnx_pack import OnnxArcFace, find_onnx_pair, make_detector

            dpath, rpath = find_onnx_pair(r.model_root_path)
            if dpath is None or rpath is None:
                raise ResourceNotFoundError(
                    f"{r.model_name}: neither lumen_face_config.json (+ safetensors) nor a detection/recognition "
                    f"ONNX pair found in {r.model_root_path}")
            det, rec = make_detector(dpath, self.device, d), OnnxArcFace(rpath, self.device, rc)
            det_size, rec_size = det.cfg.input_size, rec.cfg.input_size
        dm, dsd = d.get("mean", 127.5), d.get("std", 128.0)
        self.spec = FaceSpec(det_size=det_size, det_mean=float(np.mean(dm)),
                             det_std=float(np.mean(dsd)), rec_size=rec_size,
                             det_mean3=tuple(float(v) for v in np.broadcast_to(np.asarray(dm, np.float64), 3)),
                             det_std3=tuple(float(v) for v in np.broadcast_to(np.asarray(dsd, np.float64), 3)),
                             det_bgr=str(d.get("color_order", "rgb")).lower() == "bgr",
                             rec_mean=float(np.mean(rc.get("mean", 127.5))), rec_std=float(np.mean(rc.get("std", 127.5))),
                             rec_color=rc.get("color_order", "rgb"), align_landmarks=rc.get("align_landmarks", True))
        self.det, self.rec = det.to(self.device).eval(), rec.to(self.device).eval()
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self._det_batcher = DynamicBatcher(self._detect_batch, self.max_batch, self.max_wait_ms, "face-det")
        self._emb_batcher = DynamicBatcher(self._embed_batch, self.max_faces_batch, self.max_wait_ms, "face-emb")
        self.load_time = time.time() - t0
        self.is_initialized = True
        log.info("face pack %s ready on %s in %.2fs", r.model_name, self.device, self.load_time)

    def _init_pool(self, pool=None) -> None:
        from ...parallel.worker_pool import GPUWorkerPool

        self._pool = pool or GPUWorkerPool("lumen_amd.services.face.backend:dp_worker", self.dp_devices,
                                           kwargs={"resources": self.resources, "max_batch": self.max_batch})
        info = self._pool.submit("info", [None]).result()[0]
        self.spec = info["spec"]
        self._emb_dim = info["embedding_dim"]
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        conc = 2 * self._pool.size
        for kind, cap in (("detect", self.max_batch), ("det_emb", self.max_batch), ("embed", self.max_faces_batch)):
            self._dp[kind] = DynamicBatcher(self._pool_fn(kind), cap, self.max_wait_ms, f"face-dp-{kind}", conc)

    def _pool_fn(self, kind: str):
        def fn(items):
            with stage("dp_forward"):
                return self._pool.submit(kind, list(items)).result()
        return fn

    def close(self) -> None:
        for b in (self._det_batcher, self._emb_batcher, *self._dp.values()):
            if b is not None:
                b.close()
        self._dp = {}
        if self._pool is not None:
            self._pool.close()
            self._pool = None

    def _ensure(self):
        if not self.is_initialized:
            raise BackendNotInitializedError("Backend not initialized")

    # ------------------------------------------------------------------ batched device work
    def upload_async(self, images: Sequence[np.ndarray]):
        """Stage a batch's pixels for :meth:`detect_images` (``pre=``) from a prefetch thread: the
        pinned staging copy and the H2D run while the GPU works on the previous batch."""
        tl = self._tl()
        if getattr(tl, "pre_uploader", None) is None:
            from ...utils.image import PinnedUploader

            tl.pre_uploader = PinnedUploader(self.device)
        return tl.pre_uploader.upload_async(images)

    def _tl(self):
        """Per-thread staging state (uploaders, the last upload's image map): batches of different
        threads -- each on its own HIP stream -- may be in flight at once."""
        t = self.__dict__.get("_tls")
        if t is None:
            import threading

            t = self.__dict__.setdefault("_tls", threading.local())
        return t

    def decode_device(self, datas: Sequence[bytes]):
        """A batch of encoded images -> (images, pre): baseline JPEGs entropy-decoded on the host
        pool and reconstructed on the GPU by one batched launch (utils/jpeg.py), other formats
        through Pillow, every image in one flat device buffer.  ``images[k]`` is a
        :class:`~lumen_amd.utils.jpeg.DeviceImage` (pixels stay on the device) or the
        InvalidInputError of an undecodable payload; ``pre`` feeds :meth:`detect_images`."""
        from ...utils.jpeg import DeviceImage, decode_batch_to_device

        with stage("decode"):
            flat, offs, shapes, errors = decode_batch_to_device(list(datas), self.device)
        images = [InvalidInputError(f"Failed to decode image bytes: {errors[k]}") if k in errors
                  else DeviceImage(*shapes[k]) for k in range(len(datas))]
        return images, (flat, offs, None)

    def device_decode_ok(self) -> bool:
        """Batches of JPEG bytes can take :meth:`decode_device` (GPU device, standard alignment:
        the reference alignment mode crops host pixels)."""
        return self.device.type == "cuda" and self.align_mode != "reference" and \
            os.environ.get("LUMEN_FACE_DEVICE_JPEG", "1") != "0"

    @torch.no_grad()
    def detect_images(self, images: Sequence[np.ndarray], params: Sequence[DetParams], pre=None
                      ) -> list[list[FaceDetection]]:
        """Batched detection of decoded uint8 RGB images (one DetParams per image).  ``pre``: the
        images' device upload from :meth:`upload_async` (else uploaded here)."""
        if len(images) == 0:
            return []
        return self.detect_finish(self.detect_launch(images, params, pre))

    def detect_finish(self, st) -> list[list[FaceDetection]]:
        """Second half of :meth:`detect_images`: waits for the kept rows' D2H (queued by
        :meth:`detect_launch`) and parses them on the host."""
        images, pend = st
        with stage("det_parse"):
            return self._det_parse(len(images), pend)

    @torch.no_grad()
    def detect_launch(self, images: Sequence[np.ndarray], params: Sequence[DetParams], pre=None):
        """First half of :meth:`detect_images`: upload / preprocess / detector forward, all queued
        on the stream without waiting -- a pipelined caller queues batch i + 1's detector behind
        batch i's recogniser before it waits for batch i's embeddings."""
        N = len(images)
        S = self.spec.det_size
        geoms, scales, off = [], [], 0
        for im in images:
            g, s = letterbox_geom(im.shape[0], im.shape[1], off, S)
            geoms.append(g)
            scales.append(s)
            off += im.size
        tens = [torch.empty(im.shape, dtype=torch.uint8, device="meta") for im in images] if pre is not None \
            else [torch.from_numpy(np.ascontiguousarray(im)) for im in images]
        src = None
        if self.device.type == "cuda":
            # one pinned H2D for the batch, kept for the alignment warps of the same images
            tl = self._tl()
            if getattr(tl, "uploader", None) is None:
                from ...utils.image import PinnedUploader

                tl.uploader = PinnedUploader(self.device)
            if pre is not None:
                from ...utils.image import consume

                dev, offs, ready = pre
                consume(dev, ready)
            else:
                dev, offs = tl.uploader.upload(images)
            src = dev
            # (strong refs to the images keep their ids from being reused while the map lives); the two
            # most recent uploads are kept: a pipelined caller launches batch i + 1's detector before it
            # aligns batch i's faces (tools/face_ocr_bench.py --real-dets)
            up = (dev, {id(im): int(o) for im, o in zip(images, offs)}, list(images))
            tl.uploads = [up] + list(getattr(tl, "uploads", []))[:1]
        with stage("det_preprocess"):
            sp = self.spec
            x = ops.image_prep(tens, (S, S), mean=getattr(sp, "det_mean3", None) or (sp.det_mean,) * 3,
                               std=getattr(sp, "det_std3", None) or (sp.det_std,) * 3, scale=1.0,
                               filter="cv2_linear", layout="nhwc8", pad=0.0, geoms=geoms, out_dtype=self.dtype,
                               device=self.device, src=src, swap_rb=bool(getattr(sp, "det_bgr", False)))
        with stage("det_forward"):
            heads = self.det(x)
        with stage("det_decode_nms"):      # decode + NMS kernels + the kept rows' async D2H
            return images, self._det_post_launch(images, params, heads, scales)

    def _det_post_launch(self, images, params, heads, scales):
        """Queue decode + NMS per parameter group; -> [(image indices, NMS handle or rows)]."""
        img_scale = h2d(scales, self.device, torch.float32)
        img_hw = h2d([[im.shape[0], im.shape[1]] for im in images], self.device, torch.float32)
        A = self.det.cfg.anchors
        box_det = hasattr(self.det, "decode")       # RetinaFace-family / generic exports (onnx_pack)
        pend = []
        groups: dict = {}
        for i, p in enumerate(params):
            groups.setdefault(p.key(), []).append(i)
        for key, idx in groups.items():
            p = params[idx[0]]
            sel = h2d(idx, self.device, torch.long) if len(groups) > 1 else None
            n = len(idx)
            cand = torch.zeros((n, MAX_CAND, 16), dtype=torch.float32, device=self.device)
            count = torch.zeros((n,), dtype=torch.int32, device=self.device)
            isc = img_scale if sel is None else img_scale.index_select(0, sel)
            ihw = img_hw if sel is None else img_hw.index_select(0, sel)
            if box_det:
                out = heads if sel is None else self.det.select(heads, sel)
                self.det.decode(out, p.conf, isc, ihw, cand, count, float(p.size_min), float(p.size_max))
            else:
                for h, stride in zip(heads, self.det.cfg.strides):
                    hh = h if sel is None else h.index_select(0, sel)
                    vision.det_decode_head(hh, A, stride, p.conf, isc, ihw, cand, count, float(p.size_min),
                                           float(p.size_max))
            pend.append((idx, vision.nms_async(cand, count, p.nms) if cand.is_cuda
                         else vision.nms(cand, count, p.nms)))
        return pend

    @staticmethod
    def _det_parse(N, pend) -> list[list[FaceDetection]]:
        results: list[Optional[list[FaceDetection]]] = [None] * N
        for idx, h in pend:
            kept = vision.nms_wait(h) if isinstance(h, tuple) else h
            for j, rows in zip(idx, kept):
                faces = []
                for r in rows.tolist():
                    lm = [(r[5 + 2 * k], r[6 + 2 * k]) for k in range(5)]
                    faces.append(FaceDetection(bbox=(r[0], r[1], r[2], r[3]), confidence=min(max(r[4], 0.0), 1.0),
                                               landmarks=lm))
                results[j] = faces
        return results  # type: ignore[return-value]

    def _minv_for(self, img: np.ndarray, landmarks, bbox) -> np.ndarray:
        out = self.spec.rec_size
        if landmarks is not None and len(landmarks) == 5 and self.spec.align_landmarks:
            dst = self.template * (out / 112.0)
            M = vision.similarity_transform(np.asarray(landmarks, np.float32), dst)
            return vision.invert_affine(M)
        if bbox is None:
            bbox = (0, 0, img.shape[1], img.shape[0])
        return crop_minv(bbox, out)

    @torch.no_grad()
    def warp_faces(self, images: Sequence[np.ndarray], img_index: Sequence[int], minv: np.ndarray,
                   replicate: Optional[Sequence[bool]] = None) -> torch.Tensor:
        """Batched alignment warp -> recogniser input [F, R, R, 8].  ``replicate`` (per face)
        selects the edge-replicating border of a cv2.resize instead of the constant 0 of a
        cv2.warpAffine; faces of the two kinds are warped by one launch each."""
        R = self.spec.rec_size
        kw = dict(cpad=8, scale=1.0 / self.spec.rec_std, mean=self.spec.rec_mean / self.spec.rec_std, std=1.0,
                  swap_rb=self.spec.rec_color.lower() == "bgr", device=self.device)
        if self.device.type == "cuda":
            for last in getattr(self._tl(), "uploads", []):
                if all(id(im) in last[1] for im in images):
                    kw["src"] = (last[0], [last[1][id(im)] for im in images])     # reuse the detection upload
                    break
        if replicate is None or not any(replicate):
            return vision.warp_batch(images, img_index, minv, (R, R), **kw)
        rep = np.asarray(replicate, bool)
        parts, order = [], []
        for flag in (False, True):
            sel = np.nonzero(rep == flag)[0]
            if len(sel):
                parts.append(vision.warp_batch(images, [img_index[k] for k in sel], minv[sel], (R, R),
                                               replicate=flag, **kw))
                order.extend(sel.tolist())
        x = torch.cat(parts) if len(parts) > 1 else parts[0]
        inv = torch.empty(len(order), dtype=torch.long)
        inv[torch.tensor(order)] = torch.arange(len(order))
        return x.index_select(0, inv.to(x.device))

    @torch.no_grad()
    def embed_faces(self, images: Sequence[np.ndarray], img_index: Sequence[int], minv: np.ndarray,
                    replicate: Optional[Sequence[bool]] = None) -> np.ndarray:
        """Warp + embed F faces -> [F, D] fp32 (L2-normalised)."""
        if len(img_index) == 0:
            return np.zeros((0, self.rec.cfg.embedding), np.float32)
        with stage("align_warp"):
            x = self.warp_faces(images, img_index, minv, replicate)
            if x.dtype != self.dtype:
                x = x.to(self.dtype)
        with stage("rec_forward"):
            return self.rec(x).float().cpu().numpy()

    @torch.no_grad()
    def embed_faces_async(self, images: Sequence[np.ndarray], img_index: Sequence[int], minv: np.ndarray):
        """:meth:`embed_faces` without the wait: warp + recogniser + a D2H copy into pinned memory
        are queued; :meth:`embed_wait` returns the [F, D] embeddings."""
        x = self.warp_faces(images, img_index, minv)
        if x.dtype != self.dtype:
            x = x.to(self.dtype)
        emb = self.rec(x)
        host = torch.empty(emb.shape, dtype=torch.float32, pin_memory=True)
        host.copy_(emb, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    @staticmethod
    def embed_wait(h) -> np.ndarray:
        host, ev = h
        ev.synchronize()
        return host.numpy()

    def _detect_batch(self, items):
        imgs = [it[0] for it in items]
        return self.detect_images(imgs, [it[1] for it in items])

    def _reference_crop(self, img: np.ndarray, landmarks, bbox):
        """Reference geometry: (source image, dst->src map) of one face, or None for an
        empty crop (the reference then returns a zero vector)."""
        src = img
        if bbox is not None:
            h, w = img.shape[:2]
            x1, y1, x2, y2 = (int(v) for v in bbox)
            x1, x2 = max(0, min(x1, w)), max(0, min(x2, w))
            y1, y2 = max(0, min(y1, h)), max(0, min(y2, h))
            if x2 <= x1 or y2 <= y1:
                return None
            src = np.ascontiguousarray(img[y1:y2, x1:x2])
        out = self.spec.rec_size
        if landmarks is not None and len(landmarks) == 5 and self.spec.align_landmarks:
            # original-image landmarks, transform applied to the crop (reference behaviour);
            # cv2.warpAffine: border 0
            M = vision.similarity_transform(np.asarray(landmarks, np.float32), REFERENCE_TEMPLATE * (out / 112.0))
            return src, vision.invert_affine(M), False
        # cv2.resize of the crop (half-pixel centres, edge-replicating)
        return src, crop_minv((0, 0, src.shape[1], src.shape[0]), out), True

    def _embed_batch(self, items):
        # items: (image, landmarks, bbox); identical image objects are uploaded once
        if self.align_mode == "reference":
            srcs, minvs, reps, slot = [], [], [], []
            for img, lm, bb in items:
                r = self._reference_crop(img, lm, bb)
                if r is None:
                    slot.append(-1)
                    continue
                slot.append(len(srcs))
                srcs.append(r[0])
                minvs.append(r[1])
                reps.append(r[2])
            emb = self.embed_faces(srcs, list(range(len(srcs))), np.stack(minvs), reps) if srcs else None
            dim = self.rec.cfg.embedding
            return [emb[k] if k >= 0 else np.zeros(dim, np.float32) for k in slot]
        emb = self.embed_faces(*self._standard_geom(items))
        return list(emb)

    def _standard_geom(self, items):
        """(unique images, per-face image index, [F, 2, 3] dst->src maps) of (image, landmarks,
        bbox) items; identical image objects are listed (and uploaded) once."""
        uniq: dict = {}
        images, index, minvs = [], [], []
        for img, lm, bb in items:
            k = id(img)
            if k not in uniq:
                uniq[k] = len(images)
                images.append(img)
            index.append(uniq[k])
            minvs.append(self._minv_for(img, lm, bb))
        return images, index, np.stack(minvs)

    # ------------------------------------------------------------------ public API (reference contract)
    def _payload(self, image_bytes: bytes):
        """What a worker batch item carries: a serving front end decodes here (its own core),
        a DP worker pool gets the JPEG and decodes in the worker."""
        from ...parallel.engine import RemotePool

        if isinstance(self._pool, RemotePool):
            # baseline JPEGs travel as bytes: the engine decodes its merged batch with one GPU
            # reconstruction (dp_worker "detect" / "det_emb"); anything else decodes here
            from ...utils import jpeg

            if os.environ.get("LUMEN_FACE_DEVICE_JPEG", "1") != "0" and jpeg.info(bytes(image_bytes)) is not None:
                return bytes(image_bytes)
            return self.decode(image_bytes)
        return bytes(image_bytes)

    def decode(self, image_bytes: bytes) -> np.ndarray:
        if not image_bytes:
            raise InvalidInputError("image_bytes cannot be empty")
        try:
            with stage("decode"):
                return decode_rgb(image_bytes)
        except ValueError as e:
            raise InvalidInputError(f"Failed to decode image bytes: {e}") from e

    def image_to_faces(self, image_bytes: bytes, detection_confidence_threshold: float = 0.7,
                       nms_threshold: float = 0.4, face_size_min: int = 50, face_size_max: int = 1000
                       ) -> list[FaceDetection]:
        self._ensure()
        params = DetParams(detection_confidence_threshold, nms_threshold, face_size_min, face_size_max)
        if self._pool is not None:
            if not image_bytes:
                raise InvalidInputError("image_bytes cannot be empty")
            return self._dp["detect"]((self._payload(image_bytes), params))
        img = self.decode(image_bytes)
        return self.detect_decoded(img, params)

    def detect_decoded(self, img: np.ndarray, params: DetParams) -> list[FaceDetection]:
        self._ensure()
        if self._pool is not None:
            return self._dp["detect"]((img, params))
        return self._det_batcher((img, params))

    def detect_and_embed(self, image_bytes: bytes, params: DetParams, max_faces: int = -1
                         ) -> list[tuple[FaceDetection, np.ndarray]]:
        """Detect + embed every face of one image (decoded once; one recogniser batch).
        A failed embedding yields zero vectors like the reference (face_model.py:357-364)."""
        self._ensure()
        if self._pool is not None:
            if not image_bytes:
                raise InvalidInputError("image_bytes cannot be empty")
            return self._dp["det_emb"]((self._payload(image_bytes), params, int(max_faces)))
        img = self.decode(image_bytes)
        faces = self.detect_decoded(img, params)
        if 0 < max_faces < len(faces):
            faces = faces[:max_faces]
        if not faces:
            return []
        try:
            embs = self.embed_detections(img, faces)
        except Exception as e:  # noqa: BLE001
            log.warning("face embedding failed: %s", e)
            embs = [np.zeros((self.get_info().embedding_dim or 512,), np.float32) for _ in faces]
        return list(zip(faces, embs))

    def face_to_embedding(self, face_image: Optional[bytes] = None, cropped_face_array: Optional[np.ndarray] = None,
                          landmarks: Optional[list] = None) -> np.ndarray:
        self._ensure()
        if face_image is None and cropped_face_array is None:
            raise InvalidInputError("Either face_image or cropped_face_array must be provided")
        if self._pool is not None and face_image is not None:
            return self._dp["embed"]((bytes(face_image), landmarks, None))
        img = self.decode(face_image) if face_image is not None else \
            np.ascontiguousarray(np.clip(cropped_face_array, 0, 255).astype(np.uint8))
        if self._pool is not None:
            return self._dp["embed"]((img, landmarks, None))
        return self._emb_batcher((img, landmarks, None))

    def embed_detections(self, img: np.ndarray, faces: Sequence[FaceDetection]) -> list[np.ndarray]:
        """Embed detected faces of one decoded image (aligned from the full image)."""
        self._ensure()
        items = [(img, f.landmarks, f.bbox) for f in faces]
        if self._pool is not None:
            return self._dp["embed"].map(items)
        return self._emb_batcher.map(items)

    def embed_batch_detections(self, images: Sequence[np.ndarray], dets: Sequence[Sequence[FaceDetection]],
                               max_faces: Sequence[int]) -> list[list[tuple[FaceDetection, np.ndarray]]]:
        """Every face of a batch of decoded images (detections capped at max_faces[i] when > 0)
        aligned + embedded as ONE recogniser batch -> per image [(FaceDetection, embedding)].
        A failed embedding yields zero vectors like the reference (face_model.py:357-364)."""
        kept, flat, owner = self._flatten_dets(images, dets, max_faces)
        embs: list = []
        if flat:
            try:
                embs = self._embed_batch(flat)
            except Exception as e:  # noqa: BLE001
                log.warning("face embedding failed: %s", e)
                embs = [np.zeros((self.rec.cfg.embedding,), np.float32) for _ in flat]
        return self._per_image(kept, owner, embs)

    @staticmethod
    def _flatten_dets(images, dets, max_faces):
        kept, flat, owner = [], [], []
        for k, (img, d) in enumerate(zip(images, dets)):
            mf = int(max_faces[k])
            d = list(d[:mf]) if 0 < mf < len(d) else list(d)
            kept.append(d)
            for f in d:
                flat.append((img, f.landmarks, f.bbox))
                owner.append(k)
        return kept, flat, owner

    @staticmethod
    def _per_image(kept, owner, embs):
        per: list = [[] for _ in kept]
        for k, e in zip(owner, embs):
            per[k].append(e)
        return [list(zip(kept[k], per[k])) for k in range(len(kept))]

    @torch.no_grad()
    def embed_batch_detections_async(self, images: Sequence[np.ndarray], dets: Sequence[Sequence[FaceDetection]],
                                     max_faces: Sequence[int]):
        """:meth:`embed_batch_detections` without the wait (standard alignment on a GPU): the
        host geometry runs here, warp + recogniser + the embeddings' D2H are queued, and
        :meth:`embed_batch_detections_wait` assembles the per-image result.  A pipelined caller
        queues batch i + 1's detector between the two (tools/face_ocr_bench.py --real-dets)."""
        kept, flat, owner = self._flatten_dets(images, dets, max_faces)
        if flat and self.align_mode != "reference" and self.device.type == "cuda":
            try:
                with stage("align_rec_launch"):
                    return "pend", self.embed_faces_async(*self._standard_geom(flat)), kept, owner
            except Exception as e:  # noqa: BLE001 -- the synchronous path below logs + zero-fills
                log.warning("async face embedding launch failed (%s); embedding synchronously", e)
        return "done", self.embed_batch_detections(images, dets, max_faces)

    def embed_batch_detections_wait(self, h) -> list[list[tuple[FaceDetection, np.ndarray]]]:
        if h[0] == "done":
            return h[1]
        _, eh, kept, owner = h
        with stage("rec_wait"):
            return self._per_image(kept, owner, list(self.embed_wait(eh)))

    def detect_and_embed_images(self, images: Sequence[np.ndarray], params: Sequence[DetParams],
                                max_faces: int = -1) -> list[list[tuple[FaceDetection, np.ndarray]]]:
        """Batched detect + embed of decoded images on THIS process's device (one detector batch,
        one recogniser batch): the per-rank body of the SPMD data-parallel path
        (services/face/spmd.py) and of the DP worker's "det_emb" task."""
        dets = self.detect_images(images, params)
        return self.embed_batch_detections(images, dets, [max_faces] * len(images))

    def get_runtime_info(self) -> BackendInfo:
        return self.get_info()

    def get_info(self) -> BackendInfo:
        r = self.resources
        dev = getattr(self, "device", None)
        cuda = dev is not None and dev.type == "cuda"
        emb = self.rec.cfg.embedding if self.rec is not None else \
            (getattr(self, "_emb_dim", None) or r.get_embedding_dim() or 512)
        return BackendInfo(runtime=runtime_name(dev) if dev is not None else "mi355x-hip", device=str(dev or self.device_pref),
                           model_id=r.model_id, model_name=r.model_name, version=r.model_info.version,
                           precisions=("bf16",) if cuda or dev is None else ("fp32",), embedding_dim=emb,
                           extra={"det_size": str(self.spec.det_size), "rec_size": str(self.spec.rec_size),
                                  "detector": "scrfd", "max_batch": str(self.max_batch),
                                  "dp_workers": str(len(self.dp_devices) if self._pool is not None else 1)})


def engine_spec(resources: GenericResources, max_batch: int = 64) -> tuple:
    """(factory path, kwargs) of the GPU engine side of this backend (parallel/engine.py)."""
    return "lumen_amd.services.face.backend:dp_worker", {"resources": resources, "max_batch": max_batch}


def create_backend(settings, resources: GenericResources, runtime: Optional[str] = None) -> MI355XFaceBackend:
    """Factory (reference backends/factory.py:21-141 registers only onnx)."""
    rt = runtime or resources.runtime
    if rt not in ("onnx", "torch", "rknn"):
        raise ValueError(f"unsupported runtime '{rt}'")
    if rt == "rknn":
        raise DeviceUnavailableError("RKNN runtime is not available on MI355X builds")
    from ...resources.config import AmdRuntimeSettings

    from ...runtime import placement

    amd = AmdRuntimeSettings.from_env()
    dev = getattr(settings, "device", None) if settings is not None else None
    dev, dp_devs = placement.resolve(dev, placement.dp_size_env())
    return MI355XFaceBackend(resources, device=dev, max_batch=min(amd.max_batch, 64), max_wait_ms=amd.max_wait_ms,
                             dp_devices=dp_devs)


def dp_worker(device: str, resources: GenericResources, max_batch: int = 64):
    """GPUWorkerPool factory: one detector + recogniser on ``device``; fn(kind, items):

    "detect":  [(jpeg bytes | RGB array, DetParams)] -> [list[FaceDetection]]
    "det_emb": [(jpeg bytes, DetParams, max_faces)] -> [list[(FaceDetection, embedding)]]
               (every face of the batch aligned + embedded as ONE recogniser batch)
    "embed":   [(jpeg bytes | RGB array, landmarks | None, bbox | None)] -> [embedding]
    "info":    -> [{"spec": FaceSpec, "embedding_dim": int}]
    A payload that fails to decode yields an InvalidInputError for that request only."""
    b = MI355XFaceBackend(resources, device=device, max_batch=max_batch)
    b.initialize()

    def load(x):
        if isinstance(x, np.ndarray):
            return x
        try:
            return b.decode(x)
        except InvalidInputError as e:
            return e

    @torch.no_grad()
    def fn(kind, items):
        if kind == "info":
            return [{"spec": b.spec, "embedding_dim": int(b.rec.cfg.embedding)}] * len(items)   # one per requester
        dev_path = kind in ("detect", "det_emb") and b.device_decode_ok() and bool(items) and \
            all(isinstance(it[0], (bytes, bytearray, memoryview)) for it in items)
        if dev_path:
            # the whole batch's JPEGs: host entropy decode on the pool + ONE GPU reconstruction
            imgs, (flat, offs, _) = b.decode_device([bytes(it[0]) for it in items])
        else:
            imgs = [load(it[0]) for it in items]
        ok = [k for k, im in enumerate(imgs) if not isinstance(im, BaseException)]
        out: list = [imgs[k] for k in range(len(items))]          # decode errors stay in place
        pre = (flat, [offs[k] for k in ok], None) if dev_path else None
        if kind == "embed":
            if ok:
                embs = b._embed_batch([(imgs[k], items[k][1], items[k][2]) for k in ok])
                for k, e in zip(ok, embs):
                    out[k] = e
            return out
        dets = b.detect_images([imgs[k] for k in ok], [items[k][1] for k in ok], pre=pre) if ok else []
        if kind == "detect":
            for k, d in zip(ok, dets):
                out[k] = d
            return out
        if kind != "det_emb":
            raise ValueError(f"unknown face task kind {kind!r}")
        res = b.embed_batch_detections([imgs[k] for k in ok], dets, [items[k][2] for k in ok])
        for k, r in zip(ok, res):
            out[k] = r
        return out

    return fn
