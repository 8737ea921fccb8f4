"""MI355X VLM backend (L2): chat template, tokenizer, vision + decoder on the engine.

Contract of the reference ``BaseFastVLMBackend`` / ``FastVLMONNXBackend``
(packages/lumen-vlm/src/lumen_vlm/backends/base.py:63-553, onnxrt_backend.py:55-811):
``ChatMessage``, ``GenerationConfig`` / ``KVCacheConfig`` / ``VisionConfig`` from
``model_info.extra_metadata``, ``GenerationRequest`` defaults (max_new_tokens 512,
temperature 0, top_p 1, repetition_penalty 1), Jinja2 chat template from
``tokenizer_config.json`` with the ``<|role|>`` fallback, tokenize / detokenize with
the HF ``tokenizers`` library, stop-sequence truncation, ``GenerationChunk`` /
``GenerationResult``.

Differences (deliberate): finish reasons follow the TextGenerationV1
schema (``eos_token`` / ``length`` / ``stop_sequence``; the reference reports
"length" on EOS and "max_length"/"stop_seq" on the stream path); repetition_penalty
is applied (accepted but ignored by the reference); when the rendered prompt has no
``<image>`` token the image is placed before the first user message (the reference
silently drops the image); streaming yields per-token chunks as they are produced.

Device work runs on :class:`~lumen_amd.runtime.engine.LLMEngine` (continuous
batching over a paged KV cache) — concurrent requests share decode steps.
"""
from __future__ import annotations

import json
import logging
import os
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Iterable, Iterator, Mapping, Optional, Sequence

import numpy as np
import torch

from ...models.llm import TPInfo
from ...models.vlm import ENCODE_AHEAD, VLM, VLM_PRESETS, EncodedImage, PreparedPrefill, VLMConfig
from ...resources.exceptions import ResourceNotFoundError
from ...runtime.engine import LLMEngine, SamplingParams
from ...runtime.kv_cache import PagedKVCache
from ...runtime.metrics import current_timer, stage
from ...utils.image import decode_rgb
from ...utils.jpeg import decode_image
from ..common import GenericResources, load_safetensors, pick_device, runtime_name

log = logging.getLogger("lumen.vlm.backend")

DEFAULT_MAX_NEW_TOKENS = 512


class BackendError(Exception):
    pass


class BackendNotInitializedError(BackendError):
    pass


class InvalidInputError(BackendError):
    pass


class ModelLoadingError(BackendError):
    pass


class InferenceError(BackendError):
    pass


@dataclass(frozen=True)
class ChatMessage:
    role: str
    content: str

    def to_mapping(self) -> dict:
        return {"role": self.role, "content": self.content}


@dataclass(frozen=True)
class GenerationConfig:
    bos_token_id: int
    eos_token_id: int
    pad_token_id: int
    image_token_index: int
    vocab_size: int
    max_position_embeddings: Optional[int] = None

    @classmethod
    def from_dict(cls, d: Mapping) -> "GenerationConfig":
        req = ["bos_token_id", "eos_token_id", "pad_token_id", "image_token_index", "vocab_size"]
        miss = [k for k in req if k not in d]
        if miss:
            raise ModelLoadingError(f"generation_config missing required keys: {miss}")
        return cls(*(int(d[k]) for k in req), max_position_embeddings=d.get("max_position_embeddings"))


@dataclass(frozen=True)
class KVCacheConfig:
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    hidden_size: int
    head_dim: int

    @classmethod
    def from_dict(cls, d: Mapping) -> "KVCacheConfig":
        req = ["num_hidden_layers", "num_attention_heads", "num_key_value_heads", "hidden_size", "head_dim"]
        miss = [k for k in req if k not in d]
        if miss:
            raise ModelLoadingError(f"kv_cache_config missing keys: {miss}")
        return cls(*(int(d[k]) for k in req))


@dataclass(frozen=True)
class VisionConfigMeta:
    image_size: int
    patch_size: int
    mean: tuple
    std: tuple

    @classmethod
    def from_dict(cls, d: Mapping) -> "VisionConfigMeta":
        req = ["image_size", "patch_size", "mean", "std"]
        miss = [k for k in req if k not in d]
        if miss:
            raise ModelLoadingError(f"vision_config missing keys: {miss}")
        for k in ("mean", "std"):
            if len(d[k]) != 3:
                raise ModelLoadingError(f"vision_config entries must have 3 values, got {d[k]}")
        return cls(int(d["image_size"]), int(d["patch_size"]), tuple(float(x) for x in d["mean"]),
                   tuple(float(x) for x in d["std"]))


@dataclass
class GenerationRequest:
    messages: Sequence[ChatMessage]
    image_bytes: bytes
    add_generation_prompt: bool = True
    max_new_tokens: int = DEFAULT_MAX_NEW_TOKENS
    temperature: float = 0.0
    top_p: float = 1.0
    repetition_penalty: float = 1.0
    stop_sequences: Optional[Sequence[str]] = None
    do_sample: bool = False
    stream: bool = False
    extra: dict = field(default_factory=dict)


@dataclass
class GenerationChunk:
    text: str
    tokens: list = field(default_factory=list)
    is_final: bool = False
    metadata: dict = field(default_factory=dict)


@dataclass
class GenerationResult:
    text: str
    tokens: list
    finish_reason: str
    metadata: dict = field(default_factory=dict)


@dataclass
class BackendInfo:
    runtime: str
    device: Optional[str] = None
    model_id: Optional[str] = None
    model_name: Optional[str] = None
    version: Optional[str] = None
    precisions: list = field(default_factory=list)
    max_new_tokens: Optional[int] = None
    max_context_length: Optional[int] = None
    vision_image_size: Optional[int] = None
    vision_patch_size: Optional[int] = None
    vocab_size: Optional[int] = None
    extra: dict = field(default_factory=dict)

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k in ("runtime", "device", "model_id", "model_name", "version",
                                             "max_new_tokens", "max_context_length", "vision_image_size",
                                             "vision_patch_size", "vocab_size")}
        d["precisions"] = list(self.precisions)
        d.update(self.extra)
        return d


def stop_on_sequences(text: str, stop_sequences: Optional[Sequence[str]]) -> tuple[str, str]:
    """reference base.py:530-541: cut at the first listed stop sequence found."""
    if not stop_sequences:
        return text, ""
    for s in stop_sequences:
        if not s:
            continue
        i = text.find(s)
        if i != -1:
            return text[:i], s
    return text, ""


class IncrementalText:
    """Streaming detokenization at O(window) per token: the text of the tokens since the previous
    emission boundary, decoded together with the token before it (so a leading-space piece keeps
    its space), minus that prefix's own text, is the new text; a tail ending in U+FFFD (an
    incomplete UTF-8 sequence) is held back until a later token completes it."""

    def __init__(self, detok):
        self.detok = detok
        self.tokens: list = []
        self.prefix = 0        # window start
        self.read = 0          # tokens whose text is in self.text
        self.text = ""

    def push(self, tok) -> str:
        self.tokens.append(int(tok))
        return self._advance(hold=True)

    def flush(self) -> str:
        return self._advance(hold=False)

    def _advance(self, hold: bool) -> str:
        if self.read == len(self.tokens):
            return ""
        prev = self.detok(self.tokens[self.prefix:self.read])
        cur = self.detok(self.tokens[self.prefix:])
        if (hold and cur.endswith("\ufffd")) or len(cur) <= len(prev) or not cur.startswith(prev):
            if not hold and not cur.startswith(prev):   # tokenizer re-spelled the window: resync
                self.text = self.detok(self.tokens)
                self.prefix = self.read = len(self.tokens)
            return ""
        delta = cur[len(prev):]
        self.text += delta
        self.prefix, self.read = self.read, len(self.tokens)
        return delta


def _engine_stages(r) -> None:
    """Engine-side stage times of a finished request onto the request's timer: admission
    queue, prefill (incl. vision tower) to first token, and the decode phase."""
    t = current_timer()
    if t is None or r.t_first is None:
        return
    adm = r.t_admit or r.t_submit
    t.merge({"queue": (adm - r.t_submit) * 1000, "prefill": (r.t_first - adm) * 1000,
             "decode_tokens": ((r.t_done or r.t_first) - r.t_first) * 1000})


class MI355XVLMBackend:
    IMAGE_TOKEN = "<image>"

    def __init__(self, resources: GenericResources, device: Optional[str] = None,
                 max_new_tokens: Optional[int] = None, tp: Optional[TPInfo] = None, kv_blocks: int = 0,
                 max_batch: int = 64, tp_size: int = 1):
        self.resources = resources
        self.tp_size = max(1, int(tp_size))   # leader: spawn a TP group of this size at initialize()
        self._tp_group = None
        self._device_preference = device
        self._max_new_tokens = max_new_tokens
        self.tp = tp or TPInfo()
        self.kv_blocks = kv_blocks
        self.max_batch = max_batch
        self._initialized = False
        self._tokenizer = None
        tc = resources.configs.get("tokenizer_config.json") or {}
        t = tc.get("chat_template")
        self._chat_template = t if isinstance(t, str) and t.strip() else None
        from jinja2 import Environment, StrictUndefined

        self._jinja = Environment(trim_blocks=True, lstrip_blocks=True, undefined=StrictUndefined)
        meta = resources.extra
        self.generation_config = GenerationConfig.from_dict(meta.get("generation_config", {}))
        self.kv_cache_config = KVCacheConfig.from_dict(meta.get("kv_cache_config", {}))
        self.vision_config = VisionConfigMeta.from_dict(meta.get("vision_config", {}))
        self.model: Optional[VLM] = None
        self.engine: Optional[LLMEngine] = None
        self._remote = None            # serving front end: generation runs on a GPU engine (engine_worker)
        self.load_time = 0.0

    # ------------------------------------------------------------------ lifecycle
    @property
    def is_initialized(self) -> bool:
        return self._initialized

    @property
    def device_preference(self):
        return self._device_preference

    def ensure_initialized(self) -> None:
        if not self._initialized:
            raise BackendNotInitializedError("Backend must be initialized before calling inference APIs.")

    def _vlm_config(self) -> VLMConfig:
        r = self.resources
        cfgp = r.model_root_path / "lumen_vlm_config.json"
        if cfgp.exists():
            return VLMConfig.from_dict(json.loads(cfgp.read_text()))
        preset = (r.extra.get("lumen_preset") or "").strip()
        if preset in VLM_PRESETS:
            return VLM_PRESETS[preset]
        hfp = r.model_root_path / "config.json"
        if hfp.exists():
            from ...models.vlm import vlm_config_from_hf

            return vlm_config_from_hf(json.loads(hfp.read_text()))
        raise ResourceNotFoundError(f"{r.model_name}: no lumen_vlm_config.json, preset or HF config.json")

    def _tp_spec(self) -> dict:
        r = self.resources
        return {"cache_dir": str(r.model_root_path.parent.parent), "model": r.model_name, "runtime": r.runtime,
                "precision": r.precision, "kv_blocks": self.kv_blocks, "max_batch": self.max_batch}

    def _build(self) -> None:
        """Model (this rank's TP shard), tokenizer, paged KV cache, TP communicator."""
        self.device = pick_device(self._device_preference) if self._tp_group is None else self._tp_group.state.device
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        cfg = self._vlm_config()
        self.cfg = cfg
        m = VLM(cfg, self.tp, dtype=dtype, device=self.device)
        root = self.resources.model_root_path
        wp = root / "model.safetensors"
        from ...runtime import shard_cache
        from ...utils import onnx_import

        fp8 = (self.resources.precision or "").lower() in ("fp8", "e4m3", "fp8_e4m3") or \
            os.environ.get("LUMEN_VLM_FP8", "0") == "1"
        # pre-sharded cache: TP ranks / fp8 builds reload their own (sharded, quantised) tensors
        cached = None
        if shard_cache.enabled() and (self.tp.enabled or fp8) and self.device.type == "cuda" and \
                not self.resources.extra.get("random_init"):
            # key: the compute dtype AND the configured precision -- two non-fp8 precisions pick
            # different ONNX pack files from the same directory (find_vlm_pack)
            prec = (self.resources.precision or "default").lower().replace("/", "_")
            cached = (shard_cache.shard_path(root, self.tp.world, self.tp.rank, f"{'fp8' if fp8 else 'bf16'}-{prec}"),
                      shard_cache.source_fingerprint(root), cfg.to_dict())
        if cached is not None and shard_cache.valid(*cached):
            extra = shard_cache.load(m, cached[0], self.device)
            m.llm.weight_dtype = extra.get("weight_dtype", m.llm.weight_dtype)
            if fp8 and cfg.vision_arch != "fastvit" and os.environ.get("LUMEN_VIT_FP8", "1") != "0":
                m.vision.w8a8 = True      # the MX vision chain quantises its (bf16, cached) weights on first use
            log.info("VLM rank %d/%d weights from shard cache %s", self.tp.rank, self.tp.world, cached[0])
        else:
            pack = onnx_import.find_vlm_pack(root, self.resources.precision)
            if wp.exists():
                m.load_pack_state_dict(load_safetensors(wp))
            elif pack is not None:
                # the reference's FastVLM ONNX pack: initializers mapped onto the native FastViTHD +
                # projector + decoder (the graphs are not executed)
                log.info("VLM weights from ONNX pack %s", [p.name for p in pack])
                onnx_import.load_vlm(m, *pack)
            elif self.resources.extra.get("random_init"):
                m.random_init(int(self.resources.extra.get("seed", 0)))
            else:
                raise ResourceNotFoundError(f"{self.resources.model_name}: model.safetensors / onnx pack missing")
            if fp8:
                m.quantize_fp8()   # fp8 decoder + W8A8 ViT tower (config precision "fp8")
            if cached is not None:
                shard_cache.save(m, cached[0], cached[1], cached[2], {"weight_dtype": m.llm.weight_dtype})
        self.model = m.eval()
        if self.tp.enabled:
            from ...parallel.comm import Communicator

            self.model.llm.comm = Communicator(self.tp.group, self.device)
        self.tokenizer()
        lc = cfg.llm
        from ...runtime.kv_cache import kv_dtype_from_env

        kv_dtype = kv_dtype_from_env(dtype) if self.device.type == "cuda" else dtype   # LUMEN_KV_DTYPE=fp8
        self.kv = PagedKVCache(lc.num_layers, self.model.llm.Hkv, lc.head_dim, num_blocks=self.kv_blocks or None,
                               device=self.device, dtype=kv_dtype)

    def initialize(self) -> None:
        if self._initialized:
            return
        t0 = time.time()
        from ...parallel.engine import current_remote

        remote = current_remote()
        if remote is not None and self.tp_size <= 1:
            # serving front end (parallel/engine.py): the VLM and its continuous-batching engine live
            # in a GPU engine process (:func:`engine_worker`); requests are shipped there whole
            self._remote = remote
            self.device = torch.device("cpu")
            self.load_time = time.time() - t0
            self._initialized = True
            log.info("VLM %s served by %d GPU engine(s)", self.resources.model_name, remote.size)
            return
        sync = None
        if self.tp_size > 1 and not self.tp.enabled:
            from ...parallel.tp import TPServingGroup

            devs = None
            if self._device_preference and str(self._device_preference).startswith("cpu"):
                devs = ["cpu"] * self.tp_size
            self._tp_group = TPServingGroup(self.tp_size, self._tp_spec(), devices=devs)
            self.tp = self._tp_group.state.tp_info()
        self._build()
        if self.tp.enabled:
            from ...runtime.engine import TPSync, tp_sync_capacity

            sync = TPSync(self.tp.group, src=0,
                          capacity=tp_sync_capacity(self.max_batch, self.model.llm.cfg.max_position))
        self.engine = LLMEngine(self.model.llm, self.kv, self._build_prefill, max_batch=self.max_batch, tp_sync=sync,
                                follower_args=self._follower_args)
        self.load_time = time.time() - t0
        self._initialized = True
        log.info("VLM %s ready on %s in %.2fs (TP %d, KV cache %d tokens, %.1f GB)", self.resources.model_name,
                 self.device, self.load_time, self.tp.world, self.kv.capacity_tokens, self.kv.bytes / 1e9)

    def run_follower(self) -> None:
        """TP ranks > 0: build this rank's shard and replay the leader's steps until it stops."""
        from ...runtime.engine import TPSync, follower_loop, tp_sync_capacity

        self._build()
        self._initialized = True
        sync = TPSync(self.tp.group, src=0, capacity=tp_sync_capacity(self.max_batch, self.model.llm.cfg.max_position))
        follower_loop(self.model.llm, self.kv, self._build_prefill, sync, max_batch=self.max_batch)
        self._initialized = False

    def close(self) -> None:
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        if self._tp_group is not None:
            self._tp_group.close()
            self._tp_group = None
        self._initialized = False

    # ------------------------------------------------------------------ prompt / tokens
    def build_prompt(self, messages: Sequence[ChatMessage], add_generation_prompt: bool = True) -> str:
        if not messages:
            raise InvalidInputError("Chat messages cannot be empty.")
        if self._chat_template:
            from jinja2 import TemplateError

            try:
                # compiled once per template string: Environment.from_string recompiles every call
                # (~1-4 ms of Python per request, inside every request's time to first token)
                ct = self.__dict__.get("_tmpl_cache")
                if ct is None or ct[0] is not self._chat_template:
                    ct = self._tmpl_cache = (self._chat_template, self._jinja.from_string(self._chat_template))
                out = ct[1].render(messages=[m.to_mapping() for m in messages],
                                   add_generation_prompt=add_generation_prompt)
                if not isinstance(out, str):
                    raise TemplateError(f"Template rendered non-string value ({type(out)})")
                return out.strip()
            except TemplateError as e:
                log.warning("Chat template rendering failed (%s). Falling back to naive prompt.", e)
        parts = [f"<|{m.role}|>\n{m.content.strip()}\n" for m in messages]
        if add_generation_prompt:
            parts.append("<|assistant|>\n")
        return "".join(parts)

    def tokenizer(self):
        if self._tokenizer is None:
            p = Path(self.resources.model_root_path) / "tokenizer.json"
            if not p.exists():
                raise ResourceNotFoundError(f"Tokenizer file not found at {p}. FastVLM backends require tokenizer.json.")
            from tokenizers import Tokenizer

            try:
                self._tokenizer = Tokenizer.from_file(str(p))
            except Exception as e:  # pragma: no cover
                raise ModelLoadingError(f"Failed to load tokenizer from {p}: {e}") from e
        return self._tokenizer

    def tokenize(self, text: str, *, add_special_tokens: bool = False) -> list[int]:
        try:
            return self.tokenizer().encode(text, add_special_tokens=add_special_tokens).ids
        except Exception as e:
            raise InvalidInputError(f"Tokenization failed: {e}") from e

    def detokenize(self, ids: Sequence[int]) -> str:
        tok = self.tokenizer()
        # Tokenizer.get_vocab_size materialises the whole vocabulary: ~12-60 ms for a 128k-token
        # (Llama-3) vocab, paid on every streamed token before it was cached per tokenizer object
        cv = self.__dict__.get("_vocab_size")
        if cv is None or cv[0] is not tok:
            cv = self._vocab_size = (tok, tok.get_vocab_size(with_added_tokens=True))
        V = cv[1]
        try:
            return tok.decode([int(i) for i in ids if 0 <= int(i) < V], skip_special_tokens=True)
        except Exception as e:
            raise InvalidInputError(f"Detokenization failed: {e}") from e

    def stop_on_sequences(self, text, stop_sequences):
        return stop_on_sequences(text, stop_sequences)

    def build_generation_request(self, *, messages: Sequence[ChatMessage], image_bytes: bytes,
                                 **overrides: Any) -> GenerationRequest:
        if not image_bytes:
            raise InvalidInputError("Image payload is empty.")
        kw = dict(messages=messages, image_bytes=image_bytes,
                  add_generation_prompt=overrides.pop("add_generation_prompt", True),
                  max_new_tokens=overrides.pop("max_new_tokens", self._max_new_tokens or DEFAULT_MAX_NEW_TOKENS),
                  temperature=overrides.pop("temperature", 0.0), top_p=overrides.pop("top_p", 1.0),
                  repetition_penalty=overrides.pop("repetition_penalty", 1.0),
                  stop_sequences=overrides.pop("stop_sequences", None), do_sample=overrides.pop("do_sample", False),
                  stream=overrides.pop("stream", False), extra=overrides.pop("extra", {}))
        if overrides:
            raise InvalidInputError(f"Unknown generation overrides: {list(overrides)}")
        return GenerationRequest(**kw)

    def _with_image_token(self, messages: Sequence[ChatMessage]) -> list[ChatMessage]:
        if any(self.IMAGE_TOKEN in m.content for m in messages):
            return list(messages)
        out, placed = [], False
        for m in messages:
            if not placed and m.role == "user":
                out.append(ChatMessage(m.role, f"{self.IMAGE_TOKEN}\n{m.content}"))
                placed = True
            else:
                out.append(m)
        if not placed:
            out.insert(0, ChatMessage("user", self.IMAGE_TOKEN))
        return out

    # ------------------------------------------------------------------ generation
    def _build_prefill(self, args) -> torch.Tensor:
        ids, img = args[0], args[1]
        if isinstance(img, PreparedPrefill):
            return img.x
        if len(args) > 2:                    # TP follower: no image here, rank 0 broadcasts its features
            return self.model.build_prefill(ids, [], n_images=args[2])
        tens = [img if isinstance(img, (torch.Tensor, EncodedImage)) else torch.from_numpy(img)] \
            if img is not None else []
        return self.model.build_prefill(ids, tens)

    @staticmethod
    def _follower_args(args):
        ids, img = args[0], args[1]
        return (ids, None, 1 if img is not None else 0)

    def jpeg_draft_size(self):
        """JPEG DCT-domain downscaled decode (libjpeg scale 1/2, 1/4, 1/8) down to no less than the
        vision input on both sides: the image is padded to a square and resized to that input
        anyway, so decoding a 4032 x 3024 photo at full resolution only to shrink it 12x wastes
        most of the time to first token (1024 x 768: 5.0 ms -> ~1.5 ms).  The reference decodes at
        full size (PIL, onnxrt_backend.py:161-214); LUMEN_VLM_JPEG_DRAFT=0 restores that."""
        if os.environ.get("LUMEN_VLM_JPEG_DRAFT", "1") == "0" or self.model is None:
            return None
        s = int(self.model.cfg.vision.image_size)
        return (s, s)

    def _submit(self, req: GenerationRequest):
        self.ensure_initialized()
        if self._tp_group is not None and self._tp_group.failed:
            raise BackendError(f"tensor-parallel group unavailable: {self._tp_group.failed}")
        with stage("tokenize"):
            prompt = self.build_prompt(self._with_image_token(req.messages), req.add_generation_prompt)
            ids = self.tokenize(prompt)
        try:
            with stage("decode"):
                # baseline JPEGs: parallel host entropy decode + GPU reconstruction (utils/jpeg.py);
                # others: Pillow, DCT-scaled towards the vision input
                img = decode_image(req.image_bytes, self.device, draft_to=self.jpeg_draft_size())
        except ValueError as e:
            raise InvalidInputError(str(e)) from e
        full, starts = self.model.expand_image_tokens(ids, 1)
        if starts and ENCODE_AHEAD and self._tp_group is None and torch.device(self.device).type == "cuda":
            # the prompt's embeddings and the image encoder are queued now, in this request's
            # thread, while the engine admits it
            with stage("encode"):
                pre = self.model.prepare_prefill(ids, [img])
            if pre is not None:
                img = pre
        gc = self.generation_config
        stops = {gc.eos_token_id}
        extra_eos = self.resources.extra.get("stop_token_ids") or []
        stops.update(int(t) for t in extra_eos)
        sp = SamplingParams(max_new_tokens=max(1, int(req.max_new_tokens)), temperature=float(req.temperature),
                            top_p=float(req.top_p), repetition_penalty=float(req.repetition_penalty),
                            stop_token_ids=tuple(stops), seed=req.extra.get("seed"))
        r = self.engine.submit((ids, img if starts else None), len(full), sp)
        return r, len(full)

    def _remote_result(self, request: GenerationRequest) -> GenerationResult:
        """One generation on the engine, completed on its own (not with a merged batch)."""
        from dataclasses import replace

        gen = self._remote.stream("generate", replace(request, stream=False))
        try:
            while True:
                next(gen)
        except StopIteration as e:
            return e.value

    def _stream_remote(self, request: GenerationRequest) -> Iterator[GenerationChunk]:
        """The engine's token stream: every chunk is yielded as the engine produces it (shm
        channel partial records, parallel/shm_channel.py); closing this generator (a cancelled
        client) abandons the request and the engine stops generating it."""
        from dataclasses import replace

        yield from self._remote.stream("generate_stream", replace(request, stream=True))

    def generate(self, request: GenerationRequest):
        if self._remote is not None:
            self.ensure_initialized()
            return self._stream_remote(request) if request.stream else self._remote_result(request)
        if request.stream:
            return self._generate_stream(request)
        r, n_in = self._submit(request)
        for _ in r.stream():
            pass
        _engine_stages(r)
        text = self.detokenize(r.tokens)
        cut, stop = stop_on_sequences(text, request.stop_sequences)
        reason = "stop_sequence" if stop else (r.finish_reason or "stop")
        return GenerationResult(text=cut, tokens=list(r.tokens), finish_reason=reason,
                                metadata={"tokens_generated": len(r.tokens), "input_tokens": n_in,
                                          "ttft_ms": (r.t_first - r.t_submit) * 1000 if r.t_first else None})

    def _generate_stream(self, request: GenerationRequest) -> Iterator[GenerationChunk]:
        r, n_in = self._submit(request)
        inc = IncrementalText(self.detokenize)
        stops = [x for x in (request.stop_sequences or []) if x]
        longest = max((len(x) for x in stops), default=0)
        emitted = 0                     # characters of inc.text already yielded
        pending: list = []              # tokens not yet carried by a chunk (text held back)
        step = 0
        finished = False
        try:
            for kind, val in r.stream():
                if kind == "token":
                    pending.append(val)
                    inc.push(val)
                    if stops:
                        # a stop sequence can only end inside the new text: search the tail
                        lo = max(0, emitted - longest)
                        cut, stop = stop_on_sequences(inc.text[lo:], stops)
                        if stop:
                            cut = inc.text[:lo] + cut
                            if len(cut) > emitted:
                                yield GenerationChunk(text=cut[emitted:], tokens=pending, metadata={"step": step, "t_wall": time.time()})
                            self.engine.cancel(r)
                            for _ in r.stream():
                                pass
                            finished = True
                            _engine_stages(r)
                            yield GenerationChunk(text="", is_final=True, metadata={"reason": "stop_sequence",
                                                                                   "input_tokens": n_in})
                            return
                    if len(inc.text) == emitted:
                        continue                # held back: an incomplete UTF-8 tail
                    yield GenerationChunk(text=inc.text[emitted:], tokens=pending, metadata={"step": step, "t_wall": time.time()})
                    emitted, pending = len(inc.text), []
                    step += 1
                else:
                    finished = True
                    inc.flush()
                    if len(inc.text) > emitted or pending:
                        yield GenerationChunk(text=inc.text[emitted:], tokens=pending, metadata={"step": step, "t_wall": time.time()})
                    _engine_stages(r)
                    yield GenerationChunk(text="", is_final=True, metadata={"reason": val, "input_tokens": n_in})
        finally:
            if not finished:            # the consumer went away (client cancel): stop generating
                self.engine.cancel(r)

    def get_info(self) -> BackendInfo:
        gc, vc = self.generation_config, self.vision_config
        dev = getattr(self, "device", None)
        return BackendInfo(runtime=runtime_name(dev) if dev is not None else "mi355x-hip",
                           device=str(dev or self._device_preference), model_id=self.resources.model_info.name,
                           model_name=self.resources.model_info.name, version=self.resources.model_info.version,
                           precisions=(["bf16", "fp8"] if self.model is not None and self.model.llm.weight_dtype == "fp8"
                                       else ["bf16"]) if dev is None or dev.type == "cuda" else ["fp32"],
                           max_new_tokens=self._max_new_tokens or DEFAULT_MAX_NEW_TOKENS,
                           max_context_length=gc.max_position_embeddings, vision_image_size=vc.image_size,
                           vision_patch_size=vc.patch_size, vocab_size=gc.vocab_size,
                           extra={"tp_size": str(self.tp.world),
                                  "kv_cache_tokens": str(self.kv.capacity_tokens)
                                  if self._initialized and getattr(self, "kv", None) is not None else "0",
                                  "served_by": "engine" if self._remote is not None else "in-process"})


def engine_spec(backend: "MI355XVLMBackend") -> Optional[tuple]:
    """GPU engine side of a single-GPU VLM (parallel/engine.py): :func:`engine_worker`, with one
    engine batch loop per request the continuous-batching engine may hold.  A tensor-parallel VLM
    leads its TP group from the serving parent instead (None: mixed topology, hub/server.py)."""
    if backend.tp_size > 1:
        return None
    return ("lumen_amd.services.vlm.backend:engine_worker",
            {"resources": backend.resources, "max_new_tokens": backend._max_new_tokens, "kv_blocks": backend.kv_blocks,
             "max_batch": backend.max_batch},
            {"threads": max(2, min(backend.max_batch, 32))})


def engine_worker(device: str, resources: GenericResources, max_new_tokens: Optional[int] = None, kv_blocks: int = 0,
                  max_batch: int = 64):
    """Engine factory: the VLM on ``device``.  Generations are ``solo`` kinds (parallel/engine.py):
    each request's slot runs on its own thread on the continuous-batching LLMEngine and completes
    alone -- a short answer does not wait for a long one that arrived in the same front-end batch --
    and ``generate_stream`` hands every chunk to the front end as it is produced."""
    from dataclasses import replace

    b = MI355XVLMBackend(resources, device=device, max_new_tokens=max_new_tokens, kv_blocks=kv_blocks,
                         max_batch=max_batch)
    b.initialize()

    def fn(kind, items):
        if kind == "generate":
            out = []
            for req in items:
                try:
                    out.append(b.generate(replace(req, stream=False)))
                except Exception as e:  # noqa: BLE001 - reported per request
                    out.append(e)
            return out
        if kind == "info":
            return [b.get_info().as_dict()] * len(items)
        raise ValueError(f"unknown VLM task kind {kind!r}")

    def stream(kind, req, emit):
        if kind == "generate":
            return b.generate(replace(req, stream=False))
        if kind != "generate_stream":
            raise ValueError(f"unknown VLM stream kind {kind!r}")
        gen = b.generate(replace(req, stream=True))
        try:
            for chunk in gen:
                if not emit(chunk):     # the front end abandoned the request
                    break
        finally:
            gen.close()                 # cancels the engine request if it is still running
        return None

    fn.stream, fn.solo_kinds = stream, ("generate", "generate_stream")
    return fn


def create_backend(settings, resources: GenericResources, runtime: Optional[str] = None) -> MI355XVLMBackend:
    """Factory (reference backends/factory.py:15-82, onnx only; max_new_tokens fixed 512)."""
    rt = runtime or resources.runtime
    if rt not in ("onnx", "torch", "rknn"):
        raise ValueError(f"unsupported runtime '{rt}'")
    if rt == "rknn":
        raise BackendError("RKNN runtime is not available on MI355X builds")
    from ...resources.config import AmdRuntimeSettings

    amd = AmdRuntimeSettings.from_env()
    dev = getattr(settings, "device", None) if settings is not None else None
    return MI355XVLMBackend(resources, device=dev, max_new_tokens=DEFAULT_MAX_NEW_TOKENS, kv_blocks=amd.kv_blocks,
                            max_batch=min(amd.max_batch, 64), tp_size=amd.tp_size)
