"""MI355X CLIP backend (L2): weights -> CLIPModel on the GPU, tokenizer, preprocessing.

Contract of the reference ``BaseClipBackend`` (packages/lumen-clip/src/lumen_clip/
backends/base.py:47-292): ``initialize``, ``image_to_vector``, ``text_to_vector``,
``image_batch_to_vectors``, ``text_batch_to_vectors``, ``get_info``,
``get_temperature``; vectors are unit-normalised fp32 numpy arrays.

MI355X specifics: image decode on CPU threads, then ONE fused
resize+normalise+patchify HIP kernel for the whole batch, the bf16 tower on
MFMA kernels and the L2-normalise epilogue on device; concurrent requests from
all gRPC streams are merged by a :class:`~lumen_amd.runtime.batcher.DynamicBatcher`
that owns the device.  With ``LUMEN_DP_SIZE = N > 1`` the batcher feeds a
:class:`~lumen_amd.parallel.worker_pool.GPUWorkerPool` instead: N worker
processes, one per GPU, each holding a replica of the towers, every merged
batch split into N contiguous shards (image-batch data parallelism).  The same backend serves runtime ``torch`` and ``onnx``
configs (one native execution path, no multi-backend dispatch); ``device: cpu``
selects the fp32 PyTorch reference path (BASELINE config #1).
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from ...models.clip import CLIPModel
from ...runtime.batcher import DynamicBatcher
from ...runtime.metrics import stage
from ...utils.h2d import h2d
from ...utils.image import decode_many, decode_rgb
from ...resources.exceptions import ResourceError
from .resources import ModelResources, load_weights

log = logging.getLogger("lumen.clip.backend")


# exception hierarchy of the reference (packages/lumen-clip/src/lumen_clip/backends/backend_exceptions.py:7-59)
class BackendError(Exception):
    """Base class for all backend errors."""


class BackendNotInitializedError(BackendError):
    """Backend used before initialize()."""


class InvalidInputError(BackendError):
    """Input data invalid or malformed."""


class InferenceError(BackendError):
    """A forward pass failed (HIP launch error, OOM, ...)."""


class ModelLoadingError(BackendError):
    """Weights / tokenizer / config could not be loaded."""


class DeviceUnavailableError(BackendError):
    """The requested device does not exist on this host."""


class BackendDependencyError(BackendError):
    """A runtime kind whose optional dependencies are not part of this build."""

    def __init__(self, runtime: str) -> None:
        super().__init__(f"Backend '{runtime}' is not available in the MI355X build "
                         f"(supported runtimes: onnx, torch — both served by the native HIP engine)")
        self.runtime = runtime


@dataclass
class BackendInfo:
    runtime: str
    device: Optional[str]
    model_id: str
    model_name: str
    version: str = "1.0.0"
    precisions: tuple = ("bf16",)
    image_embedding_dim: Optional[int] = None
    text_embedding_dim: Optional[int] = None
    supports_image_batch: bool = True
    extra_metadata: Optional[dict] = None


def pick_device(pref: Optional[str]) -> torch.device:
    if pref and pref.startswith("cpu"):
        return torch.device("cpu")
    if torch.cuda.is_available():
        if pref and pref.startswith("cuda"):
            d = torch.device(pref)
            if d.index is not None and d.index >= torch.cuda.device_count():
                raise DeviceUnavailableError(f"{pref} requested but only {torch.cuda.device_count()} GPU(s) visible")
            return d
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


class MI355XClipBackend:
    def __init__(self, resources: ModelResources, device: Optional[str] = None, batch_size: int = 8,
                 max_batch: int = 256, max_wait_ms: float = 2.0, precision: Optional[str] = None, dp_size: int = 1,
                 dp_devices: Optional[Sequence[str]] = None):
        self.resources = resources
        self.dp_devices = list(dp_devices or [])
        self.dp_size = max(1, len(self.dp_devices) or int(dp_size))
        self._pool = None
        self.device_pref = device
        self.batch_size = batch_size
        self.max_batch = max_batch
        self.max_wait_ms = max_wait_ms
        self.precision = precision
        self.model: Optional[CLIPModel] = None
        self.tokenizer = None
        self.context_length = 77
        self.load_time = 0.0
        self._img_batcher: Optional[DynamicBatcher] = None
        self._txt_batcher: Optional[DynamicBatcher] = None
        self.shard_bank = False        # BioCLIP: each DP worker holds a slice of the label bank
        self.remote_key: Optional[str] = None   # multi-model service: this model's part of the engine
        self.is_initialized = False

    # ------------------------------------------------------------------ lifecycle
    def initialize(self) -> None:
        if self.is_initialized:
            return
        t0 = time.time()
        self.device = pick_device(self.device_pref)
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        cfg = self.resources.clip_config()
        mean, std = self.resources.get_normalization_stats()
        cfg.image_mean, cfg.image_std = tuple(mean), tuple(std)
        self.cfg = cfg
        self.context_length = cfg.context_length
        from ...parallel.engine import current_remote

        remote = current_remote()
        if remote is not None and self.remote_key:
            remote = remote.prefixed(self.remote_key)
        if remote is not None:
            # serving front end (parallel/engine.py): the towers live in the GPU engine processes;
            # this process decodes, tokenises and ships batches there
            self._pool = remote
            self.device = torch.device("cpu")
            info = remote.submit("info", [None]).result()[0]
            self._logit_scale = float(info["logit_scale"])
        elif self.dp_size > 1:
            from ...parallel.worker_pool import GPUWorkerPool, default_devices

            r = self.resources
            devs = self.dp_devices or (["cpu"] * self.dp_size if self.device.type == "cpu"
                                       else default_devices(self.dp_size))
            self._pool = GPUWorkerPool("lumen_amd.services.clip.backend:dp_worker", devs,
                                       kwargs={"cache_dir": str(r.model_root_path.parent.parent),
                                               "model": r.model_name, "runtime": r.runtime,
                                               "dataset": r.dataset, "shard_bank": self.shard_bank})
            sd = load_weights(r.model_root_path, self.precision)
            self._logit_scale = float(sd["logit_scale"]) if "logit_scale" in sd else cfg.logit_scale
        else:
            try:
                m = CLIPModel(cfg, dtype=dtype, device="cpu")
                m.load_state_dict_any(load_weights(self.resources.model_root_path, self.precision))
            except (OSError, KeyError, ValueError, RuntimeError, ResourceError) as e:
                raise ModelLoadingError(f"loading {self.resources.model_name} from "
                                        f"{self.resources.model_root_path}: {e}") from e
            m.center_crop = torch_runtime_crop(self.resources.runtime)
            self.model = m.to(self.device)
            self._logit_scale = self.model.logit_scale
        self._load_tokenizer()
        # with DP workers: 2 dispatchers per GPU, each batch goes whole to the least-loaded worker; one
        # GPU in-process: 2 dispatchers, so one batch's stacking / H2D / D2H overlaps the other's tower
        conc = (2 * self._pool.size if self._pool is not None and remote is not None else
                2 * self.dp_size if self._pool is not None else (2 if self.device.type == "cuda" else 1))
        self._img_batcher = DynamicBatcher(self._encode_images, self.max_batch, self.max_wait_ms, "clip-image", conc)
        self._txt_batcher = DynamicBatcher(self._encode_texts, self.max_batch, self.max_wait_ms, "clip-text", conc)
        self.load_time = time.time() - t0
        self.is_initialized = True
        log.info("CLIP %s ready on %s in %.2fs (dp %d)", self.resources.model_name, self.device, self.load_time,
                 self.dp_size)

    def close(self) -> None:
        for b in (self._img_batcher, self._txt_batcher):
            if b is not None:
                b.close()
        if self._pool is not None:
            self._pool.close()
            self._pool = None

    def _load_tokenizer(self) -> None:
        p = self.resources.tokenizer_path
        if p is None:
            raise ModelLoadingError(f"tokenizer.json missing in {self.resources.model_root_path}")
        from tokenizers import Tokenizer

        tok = Tokenizer.from_file(str(p))
        tok.enable_truncation(max_length=self.context_length)
        # OpenAI BPE pads with 0 (EOT-argmax pooling ignores it); CN-CLIP's WordPiece pads with
        # [PAD]=0 and the BERT tower masks keys past the non-pad length
        pad = "[PAD]" if self.cfg.text_arch == "bert" else "<pad>"
        tok.enable_padding(pad_id=0, pad_token=pad, length=self.context_length)
        self.tokenizer = tok

    def _ensure(self):
        if not self.is_initialized:
            raise BackendNotInitializedError("backend not initialized")

    @property
    def remote(self) -> bool:
        """True in a serving front end: batches go to the GPU engine processes (decoded here)."""
        from ...parallel.engine import is_remote

        return is_remote(self._pool)

    # ------------------------------------------------------------------ batched workers
    def tokenize(self, texts: Sequence[str]) -> torch.Tensor:
        encs = self.tokenizer.encode_batch(list(texts))
        ids = np.array([e.ids[: self.context_length] for e in encs], dtype=np.int64)
        return torch.from_numpy(ids)

    def _encode_texts(self, texts: Sequence[str]) -> list:
        with stage("tokenize"):
            ids = self.tokenize(texts)
        if self._pool is not None:
            with stage("dp_forward"):
                return self._pool.submit("text", list(ids.numpy())).result()
        with torch.no_grad(), stage("forward"):      # H2D + text tower + D2H (synchronising)
            emb = self.model.encode_text_ids(ids.to(self.device)).float().cpu().numpy()
        return list(emb)

    def _encode_images(self, payloads: Sequence[bytes]) -> list:
        if self._pool is not None:
            with stage("dp_forward"):
                return self._pool.submit("image", list(payloads)).result()
        raw = [i for i, p in enumerate(payloads) if not isinstance(p, np.ndarray)]
        imgs = list(payloads)
        if raw:                                       # batch API: decode here (single requests arrive decoded)
            with stage("decode"):
                for i, a in zip(raw, decode_many([payloads[i] for i in raw])):
                    imgs[i] = a
        with torch.no_grad(), stage("forward"):      # H2D + resize/normalise + tower + D2H
            tens = [torch.from_numpy(i) for i in imgs]
            emb = self.model.encode_image_uint8(tens).float().cpu().numpy()
        return list(emb)

    # ------------------------------------------------------------------ public API
    def image_to_vector(self, image_bytes: bytes) -> np.ndarray:
        self._ensure()
        if not image_bytes:
            raise InvalidInputError("empty image payload")
        if self._pool is not None and not self.remote:  # DP workers decode in their own processes
            return self._img_batcher(image_bytes)
        if self.remote:
            # serving front end: a baseline JPEG travels as bytes and the engine decodes the whole
            # merged batch on the GPU (utils.jpeg.decode_batch_to_device); anything else decodes here
            from ...utils.jpeg import info as jpeg_info

            if jpeg_info(image_bytes) is not None:
                v = self._img_batcher(bytes(image_bytes))
                if v is None:
                    raise InvalidInputError("Failed to decode image")
                return v
        # decoded on the caller's (gRPC) thread: Pillow releases the GIL, so concurrent requests decode
        # in parallel and the batch's critical path is only the GPU work; a bad payload fails alone
        with stage("decode"):
            try:
                img = decode_rgb(image_bytes)
            except ValueError as e:
                raise InvalidInputError(str(e)) from e
        return self._img_batcher(img)

    def image_batch_to_vectors(self, images: Sequence[bytes]) -> np.ndarray:
        self._ensure()
        if self._pool is not None:       # every chunk in flight at once, spread over the GPUs
            n = self._pool.size
            per = min(self.max_batch, max(1, -(-len(images) // n)))
            with stage("dp_forward"):
                futs = [self._pool.submit("image", list(images[i:i + per])) for i in range(0, len(images), per)]
                out = [e for f in futs for e in f.result()]
            return np.stack(out).astype(np.float32)
        out = []
        for i in range(0, len(images), self.max_batch):
            out.extend(self._encode_images(images[i:i + self.max_batch]))
        return np.stack(out).astype(np.float32)

    def text_to_vector(self, text: str) -> np.ndarray:
        self._ensure()
        return self._txt_batcher(text)

    def text_batch_to_vectors(self, texts: Sequence[str]) -> np.ndarray:
        self._ensure()
        out = []
        for i in range(0, len(texts), self.max_batch):
            out.extend(self._encode_texts(texts[i:i + self.max_batch]))
        return np.stack(out).astype(np.float32) if out else np.zeros((0, self.cfg.embed_dim), np.float32)

    def get_temperature(self) -> float:
        return float(np.exp(self._logit_scale)) if self.is_initialized else 100.0

    def get_info(self) -> BackendInfo:
        r = self.resources
        dim = self.cfg.embed_dim if self.is_initialized else r.get_embedding_dim()
        return BackendInfo(runtime="mi355x-hip" if getattr(self, "device", None) is not None and self.device.type == "cuda"
                           else "torch-cpu-reference", device=str(getattr(self, "device", self.device_pref)),
                           model_id=r.model_id, model_name=r.model_name, image_embedding_dim=dim,
                           text_embedding_dim=dim,
                           precisions=("bf16",) if getattr(self, "device", None) is not None and self.device.type == "cuda"
                           else ("fp32",),
                           extra_metadata={"image_size": str(r.get_image_size()),
                                           "context_length": str(self.context_length)})


def torch_runtime_crop(runtime) -> bool:
    """The reference's two CLIP preprocessors: its torch runtime (open_clip / HF processors)
    resizes the shortest side and centre-crops; its ONNX runtime squashes to the model size."""
    return str(getattr(runtime, "value", runtime)).lower() == "torch"


def dp_worker(device: str, cache_dir: str, model: str, runtime: str, dataset: Optional[str] = None,
              shard_bank: bool = False, rank: int = 0, world: int = 1):
    """GPUWorkerPool factory: one CLIP replica on ``device``; fn(kind, items) -> embeddings.

    kind "image": encoded image bytes (decoded on this worker's CPU threads);
    kind "text": token-id arrays [ctx];
    kind "bank_topk" (``shard_bank``): items = [(queries [B, D], k, scale, softmax)] -> this
    worker's label-bank shard candidates (rows rank/world of the memory-mapped bank .npy)."""
    from ...resources.config import ModelConfig, Runtime
    from .resources import ResourceLoader

    res = ResourceLoader.load_model_resources(cache_dir, ModelConfig(model=model, runtime=Runtime(runtime),
                                                                     dataset=dataset))
    dev = torch.device(device)
    cfg = res.clip_config()
    mean, std = res.get_normalization_stats()
    cfg.image_mean, cfg.image_std = tuple(mean), tuple(std)
    m = CLIPModel(cfg, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32, device="cpu")
    m.load_state_dict_any(load_weights(res.model_root_path))
    m.center_crop = torch_runtime_crop(runtime)
    m = m.to(dev)
    bank = None
    if shard_bank and res.label_embeddings is not None:
        from ...runtime.label_bank import LabelBank, orient_bank

        emb = orient_bank(res.label_embeddings, len(res.labels) if res.labels is not None else 0, cfg.embed_dim)
        bank = LabelBank(emb, dev, shard=(rank, world))

    @torch.no_grad()
    def fn(kind, items):
        if kind == "bank_topk":
            if bank is None:
                raise RuntimeError("this worker holds no label-bank shard")
            return [bank.topk_local(q, k, scale, sm) for q, k, scale, sm in items]
        if kind == "info":
            # one answer per item: the engine may merge several front ends' info calls in a batch
            return [{"logit_scale": float(m.logit_scale), "embed_dim": int(cfg.embed_dim)}] * len(items)
        if kind == "image":
            if dev.type == "cuda" and cfg.vision_arch != "fastvit" and items and \
                    all(isinstance(it, (bytes, bytearray)) for it in items):
                # encoded payloads (a serving front end or a DP caller): the whole batch decodes on the
                # device -- parallel host entropy decode, one IDCT + colour launch -- and the patch
                # preprocessing reads the decoded pixels in place; an undecodable payload answers None
                from ...utils.jpeg import decode_batch_to_device

                flat, _offs, shapes, errs = decode_batch_to_device(list(items), dev)
                out = list(m.encode_image_uint8(shapes, src=flat).float().cpu().numpy())
                for k in errs:
                    out[k] = None
                return out
            # encoded images (DP workers decode here) or uint8 HWC arrays (decoded by a serving front end)
            raw = [k for k, it in enumerate(items) if not isinstance(it, np.ndarray)]
            imgs = list(items)
            if raw:
                for k, a in zip(raw, decode_many([items[k] for k in raw])):
                    imgs[k] = a
            emb = m.encode_image_uint8([torch.from_numpy(np.ascontiguousarray(i)) for i in imgs])
        elif kind == "text":
            emb = m.encode_text_ids(h2d(np.stack(items), dev))
        else:
            raise ValueError(f"unknown CLIP task kind {kind!r}")
        return list(emb.float().cpu().numpy())

    return fn


def engine_spec(resources: ModelResources, shard_bank: bool = False) -> tuple:
    """(factory path, kwargs) of the GPU engine side of this backend (parallel/engine.py).
    ``shard_bank``: every engine holds its rank / world slice of the stored label bank (BioCLIP's
    TreeOfLife bank), queried by broadcast from the front ends (runtime/label_bank.PoolShardedBank)."""
    r = resources
    return ("lumen_amd.services.clip.backend:dp_worker",
            {"cache_dir": str(r.model_root_path.parent.parent), "model": r.model_name, "runtime": r.runtime,
             "dataset": r.dataset, "shard_bank": bool(shard_bank)})


def bio_shards_bank(resources: ModelResources) -> bool:
    """A BioCLIP model with a stored bank: sharded over the GPU workers / engines."""
    return resources.labels is not None and len(resources.labels) > 0 and resources.label_embeddings is not None


def create_backend(backend_settings, resources: ModelResources, runtime: Optional[str] = None,
                   precision: Optional[str] = None) -> MI355XClipBackend:
    """Factory (reference backends/factory.py:21-141): runtime must be onnx|torch|rknn."""
    rt = runtime or resources.runtime
    if rt not in ("onnx", "torch", "rknn"):
        raise ValueError(f"unsupported runtime '{rt}' (expected onnx|torch|rknn)")
    if rt == "rknn":
        raise BackendDependencyError("rknn")
    from ...resources.config import AmdRuntimeSettings

    from ...runtime import placement

    amd = AmdRuntimeSettings.from_env()
    dev = getattr(backend_settings, "device", None) if backend_settings is not None else None
    dev, dp_devs = placement.resolve(dev, placement.dp_size_env())
    bs = getattr(backend_settings, "batch_size", 8) if backend_settings is not None else 8
    return MI355XClipBackend(resources, device=dev, batch_size=bs or 8, max_batch=amd.max_batch,
                             max_wait_ms=amd.max_wait_ms, precision=precision, dp_devices=dp_devs)
