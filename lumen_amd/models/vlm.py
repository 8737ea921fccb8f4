"""LLaVA-family vision-language model: ViT image encoder -> MLP projector -> decoder LLM.

Reference pipeline (packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py):
prompt -> tokens; image -> pad-to-square (black, centred) + bicubic resize -> /255
-> vision encoder (FastViTHD, 256 tokens) -> projector; token embeddings; the
vision embeddings replace the ``<image>`` token (:240-296); prefill; decode loop.

Presets:
* ``fastvlm-0.5b``  — Qwen2-0.5B decoder with FastViTHD (models/fastvit.py: the
  reparameterised conv/RepMixer/attention hybrid, 1024 px -> 16 x 16 x 3072 conv_exp map
  = 256 visual tokens) -> 2-layer GELU projector (3072 -> 896).  ``cfg.vision`` keeps the
  token geometry (image_size 1024, patch_size = the tower's stride 64).
* ``llava-llama3-8b`` — north-star config: CLIP ViT-L/14-336 (penultimate layer,
  576 tokens, CLS dropped) -> 2-layer GELU MLP projector -> Llama-3-8B.
* ``tiny`` — CPU tests.

MI355X path: one fused pad/resize/normalise/patchify kernel, the ViT on the MFMA
kernels, projector GEMMs whose second GEMM writes straight into the rows of the
LLM's prefill embedding buffer that the ``<image>`` token occupies.
"""
from __future__ import annotations

import logging
import os
import threading

from dataclasses import asdict, dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch
from torch import nn

from .. import ops
from ..utils.h2d import h2d, h2d_ahead
from .clip import VisionConfig, VisionTower
from .fastvit import FASTVIT_PRESETS, FastViTConfig, FastViTTower
from .llm import LLM, LLM_PRESETS, LLMConfig, TPInfo

log = logging.getLogger("lumen.vlm")

# The image encoder (patch GEMM -> tower -> projector) of a small image count replayed from a
# hipGraph: ~170 launches of ~8 us host time each become one, so the tower no longer waits on the
# host at the start of a request (profiles/r5_ttft_*).  LUMEN_VISION_GRAPH=0: eager launches.
_VISION_GRAPH = os.environ.get("LUMEN_VISION_GRAPH", "1") == "1"
# tensor parallel: a ViT image tower runs split over the TP group (clip.run_blocks_tp) instead of on rank 0
# with a feature broadcast (VERDICT r5 missing 3; tests/test_parallel_cpu.py, tests/test_tp_gpu.py)
TP_TOWER = True
_VISION_GRAPH_MAX_B = 4
# the service / benchmarks encode a request's image in the request's thread (encode_ahead)
ENCODE_AHEAD = os.environ.get("LUMEN_VLM_ENCODE_AHEAD", "1") == "1"


class PreparedPrefill:
    """A request's whole prefill input x [T, hidden] (text embeddings + image rows), built in the
    request's thread (:meth:`VLM.prepare_prefill`) so that its uploads and the image encoder are
    queued before the engine admits the request; the engine's prefill builder passes it through."""

    __slots__ = ("x",)

    def __init__(self, x: torch.Tensor):
        self.x = x

    @property
    def shape(self):
        return tuple(self.x.shape)


class EncodedImage:
    """Projected embeddings [N_img, hidden] of one image, encoded ahead of the prefill
    (:meth:`VLM.encode_ahead`, in the request's thread while the engine admits it); the prefill
    builder splices the rows instead of running the tower."""

    __slots__ = ("emb",)

    def __init__(self, emb: torch.Tensor):
        self.emb = emb

    @property
    def shape(self):
        return tuple(self.emb.shape)


@dataclass
class VLMConfig:
    vision: VisionConfig = field(default_factory=lambda: VisionConfig(image_size=1024, patch_size=64, width=768,
                                                                      layers=12, heads=12, act="gelu"))
    llm: LLMConfig = field(default_factory=LLMConfig)
    feature_layer: int = -2
    image_token_id: int = 151646
    image_mean: tuple = (0.0, 0.0, 0.0)
    image_std: tuple = (1.0, 1.0, 1.0)
    pad_value: float = 0.0          # pad-to-square fill (pixel units)
    resize_filter: str = "pil_bicubic"
    vision_arch: str = "vit"        # "vit" (LLaVA CLIP towers) | "fastvit" (FastViTHD)
    fastvit: Optional[FastViTConfig] = None

    @property
    def vision_width(self) -> int:
        return self.fastvit.final_features if self.vision_arch == "fastvit" else self.vision.width

    @property
    def num_image_tokens(self) -> int:
        return (self.vision.image_size // self.vision.patch_size) ** 2

    def to_dict(self):
        return asdict(self)

    @staticmethod
    def from_dict(d: dict) -> "VLMConfig":
        v = VisionConfig(**d.get("vision", {}))
        l = LLMConfig.from_dict(d.get("llm", {}))
        rest = {k: d[k] for k in ("feature_layer", "image_token_id", "pad_value", "resize_filter", "vision_arch")
                if k in d}
        if d.get("fastvit"):
            rest["fastvit"] = FastViTConfig.from_dict(d["fastvit"])
        for k in ("image_mean", "image_std"):
            if k in d:
                rest[k] = tuple(d[k])
        return VLMConfig(vision=v, llm=l, **rest)


def vlm_config_from_hf(c: dict) -> VLMConfig:
    """FastVLM (``llava_qwen2`` with the FastViTHD / MobileCLIP-L tower) HF ``config.json`` ->
    VLMConfig, for reference ONNX packs that ship no lumen config."""
    fv = FASTVIT_PRESETS["fastvithd"]
    size = int(c.get("image_size") or (c.get("vision_config") or {}).get("image_size") or 1024)
    return VLMConfig(vision=VisionConfig(image_size=size, patch_size=64, width=fv.final_features, layers=0, heads=1),
                     llm=LLMConfig.from_hf(c.get("text_config") or c), vision_arch="fastvit", fastvit=fv,
                     image_token_id=int(c.get("image_token_index", 151646)))


VLM_PRESETS = {
    "fastvlm-0.5b": VLMConfig(vision=VisionConfig(image_size=1024, patch_size=64, width=3072, layers=0, heads=1),
                              vision_arch="fastvit", fastvit=FASTVIT_PRESETS["fastvithd"]),
    "llava-llama3-8b": VLMConfig(vision=VisionConfig(image_size=336, patch_size=14, width=1024, layers=24, heads=16,
                                                     act="quick_gelu"),
                                 llm=LLM_PRESETS["llama3-8b"], image_token_id=128002,
                                 image_mean=(0.48145466, 0.4578275, 0.40821073),
                                 image_std=(0.26862954, 0.26130258, 0.27577711), pad_value=116.0),
    "tiny": VLMConfig(vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=2, act="gelu"),
                      llm=LLM_PRESETS["tiny"], image_token_id=259),
    "tiny-h8": VLMConfig(vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=2, act="gelu"),
                         llm=LLM_PRESETS["tiny-h8"], image_token_id=259),
    "tiny-gqa8": VLMConfig(vision=VisionConfig(image_size=32, patch_size=8, width=64, layers=2, heads=2, act="gelu"),
                           llm=LLM_PRESETS["tiny-gqa8"], image_token_id=259),
    "tiny-fastvit": VLMConfig(vision=VisionConfig(image_size=64, patch_size=16, width=128, layers=0, heads=1),
                              vision_arch="fastvit", fastvit=FASTVIT_PRESETS["tiny-ln"], llm=LLM_PRESETS["tiny"],
                              image_token_id=259),
}


class VLM(nn.Module):
    def __init__(self, cfg: VLMConfig, tp: Optional[TPInfo] = None, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        kw = dict(dtype=dtype, device=device)
        self.vision = FastViTTower(cfg.fastvit, None, dtype, device) if cfg.vision_arch == "fastvit" \
            else VisionTower(cfg.vision, 16, dtype, device)
        Wv, Hd = cfg.vision_width, cfg.llm.hidden_size
        self.proj1_w = nn.Parameter(torch.zeros(Hd, Wv, **kw), requires_grad=False)
        self.proj1_b = nn.Parameter(torch.zeros(Hd, dtype=torch.float32, device=device), requires_grad=False)
        self.proj2_w = nn.Parameter(torch.zeros(Hd, Hd, **kw), requires_grad=False)
        self.proj2_b = nn.Parameter(torch.zeros(Hd, dtype=torch.float32, device=device), requires_grad=False)
        self.llm = LLM(cfg.llm, tp, dtype, device)
        self._vgraphs: dict = {}
        self._vgraph_lock = threading.Lock()

    def invalidate_graphs(self) -> None:
        """Drop the captured image-encoder graphs (they hold the weights' tensors; call after any
        weight load / quantisation)."""
        with self._vgraph_lock:
            self._vgraphs.clear()

    @torch.no_grad()
    def random_init(self, seed: int = 0):
        """Vision + projector replicated on every rank (same seed); LLM shards per rank."""
        g = torch.Generator().manual_seed(seed)
        dev = self.proj1_w.device
        vis_cpu = FastViTTower(self.cfg.fastvit, None, torch.float32, "cpu") if self.cfg.vision_arch == "fastvit" \
            else VisionTower(self.cfg.vision, 16, torch.float32, "cpu")
        vis_cpu.random_init(g)
        self.vision.load_state_dict({k: v.to(self.vision.state_dict()[k].dtype) for k, v in vis_cpu.state_dict().items()})
        Wv, Hd = self.cfg.vision_width, self.cfg.llm.hidden_size
        self.proj1_w.copy_((torch.randn(Hd, Wv, generator=g) * Wv ** -0.5).to(self.proj1_w.dtype).to(dev))
        self.proj2_w.copy_((torch.randn(Hd, Hd, generator=g) * Hd ** -0.5).to(self.proj2_w.dtype).to(dev))
        self.llm.random_init(seed)
        self.invalidate_graphs()

    @torch.no_grad()
    def quantize_fp8(self) -> None:
        """fp8 VLM: the W8A8 / fp8-weight decoder (LLM.quantize_fp8) and, for a ViT tower, the MX W8A8
        vision chain (clip.run_blocks_mx; LUMEN_VIT_FP8=0 keeps the tower bf16)."""
        self.llm.quantize_fp8()
        if self.cfg.vision_arch != "fastvit" and os.environ.get("LUMEN_VIT_FP8", "1") != "0":
            self.vision.w8a8 = True
        self.invalidate_graphs()

    @property
    def device(self):
        return self.proj1_w.device

    # ------------------------------------------------------------------ vision
    def preprocess(self, images: Sequence[torch.Tensor]) -> torch.Tensor:
        """uint8 HWC images -> patch rows: pad to a centred square (pad_value), resize, normalise."""
        v = self.vision
        s = self.cfg.vision.image_size
        geoms, off = [], 0
        for im in images:
            geoms.append(ops.ImageGeom.pad_square(im.shape[0], im.shape[1], off, s))
            off += im.numel()
        if self.cfg.vision_arch == "fastvit":
            return ops.image_prep(list(images), (s, s), mean=self.cfg.image_mean, std=self.cfg.image_std,
                                  filter=self.cfg.resize_filter, layout="nhwc8", pad=self.cfg.pad_value, geoms=geoms,
                                  out_dtype=v.stem0.w.dtype, device=self.device)
        return ops.image_prep(list(images), (s, s), mean=self.cfg.image_mean, std=self.cfg.image_std,
                              filter=self.cfg.resize_filter, layout="patches", patch=self.cfg.vision.patch_size,
                              kpad=v.kpad, pad=self.cfg.pad_value, geoms=geoms, out_dtype=v.patch_w.dtype,
                              device=self.device)

    def _encode_tower(self, pre: torch.Tensor, B: int, out: Optional[torch.Tensor] = None,
                      tp: Optional[tuple] = None) -> torch.Tensor:
        """preprocessed pixels -> projected embeddings [B * N_img, hidden] (``tp``: the ViT blocks
        tensor-parallel over the group, clip.run_blocks_tp)"""
        if self.cfg.vision_arch == "fastvit":     # conv_exp map [B, 16, 16, 3072]: NHWC rows = image tokens
            feats = self.vision.forward_features(pre)
        else:
            feats = self.vision.forward_features(pre, B, self.cfg.feature_layer, tp=tp)
        f = feats.reshape(B * self.cfg.num_image_tokens, -1)
        if not f.is_contiguous():
            f = f.contiguous()
        h = ops.linear(f, self.proj1_w, self.proj1_b, act="gelu")
        return ops.linear(h, self.proj2_w, self.proj2_b, out=out)

    def _graph_ok(self, pre: torch.Tensor, B: int) -> bool:
        return _VISION_GRAPH and pre.is_cuda and B <= _VISION_GRAPH_MAX_B and not torch.cuda.is_current_stream_capturing()

    def _graph_encode(self, pre: torch.Tensor, B: int, out: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """the tower from the graph of this (B, input shape, tower precision); None when it cannot be
        captured (eager from then on for this key).  The static input / output are used under the
        lock, so concurrent requests cannot interleave their copies with another's replay."""
        key = (B, tuple(pre.shape), pre.dtype, bool(getattr(self.vision, "w8a8", False)))
        with self._vgraph_lock:
            ent = self._vgraphs.get(key)
            if ent is None:
                ent = self._capture(pre, B)
                self._vgraphs[key] = ent
            if ent is False:
                return None
            # the lock orders the host-side enqueues only: wait on the device for the previous user's
            # replay / copy-out (possibly on another stream) before reusing the static buffers
            cur = torch.cuda.current_stream(pre.device)
            if ent.get("ev") is not None:
                cur.wait_event(ent["ev"])
            ent["in"].copy_(pre)
            ent["g"].replay()
            if out is not None:
                out.copy_(ent["out"])
            else:
                out = ent["out"].clone()
            ent["ev"] = torch.cuda.Event()
            ent["ev"].record(cur)
            return out

    def _capture(self, pre: torch.Tensor, B: int):
        try:
            static_in = pre.clone()
            cur = torch.cuda.current_stream(pre.device)
            # this model's own capture stream: the split-K tickets / workspaces keyed by the
            # stream are baked into the graph, so no other graph or eager thread may ever use it
            if getattr(self, "_cap_stream", None) is None:
                self._cap_stream = ops.private_stream(pre.device)
            side = self._cap_stream
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._encode_tower(static_in, B)     # warm-up: weight caches, workspaces, autotune
            cur.wait_stream(side)
            g = torch.cuda.CUDAGraph()
            # thread_local: other threads keep launching meanwhile; one capture at a time per process
            with ops.CAPTURE_LOCK, torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                static_out = self._encode_tower(static_in, B)
            return {"g": g, "in": static_in, "out": static_out}
        except Exception as e:  # noqa: BLE001 - an op that cannot be captured: eager launches
            log.warning("image encoder graph capture failed (%s); eager launches", e)
            return False

    @torch.no_grad()
    def encode_images(self, images: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """-> projected image embeddings [B * N_img, hidden] (or written into ``out`` rows)."""
        B = len(images)
        pre = self.preprocess(images)
        if self._graph_ok(pre, B):
            r = self._graph_encode(pre, B, out)
            if r is not None:
                return r
        return self._encode_tower(pre, B, out=out)

    @torch.no_grad()
    def prepare_prefill(self, ids: Sequence[int], images: Sequence[torch.Tensor]):
        """:meth:`build_prefill` run now, in the caller's thread (single-rank GPU models), wrapped
        as a :class:`PreparedPrefill`; otherwise None (the engine builds the input itself)."""
        if self.llm.tp.enabled or self.device.type != "cuda":
            return None
        return PreparedPrefill(self.build_prefill(ids, images))

    @torch.no_grad()
    def encode_ahead(self, images: Sequence[torch.Tensor]) -> list:
        """Run the image encoder now (in the caller's thread, on its stream) and return
        :class:`EncodedImage` stand-ins for :meth:`build_prefill`: the tower's GPU work then starts
        while the engine is still admitting the request.  Single-rank models only (under tensor
        parallelism the images follow the TP group's own schedule)."""
        if self.llm.tp.enabled or not images or self.device.type != "cuda":
            return list(images)
        N = self.cfg.num_image_tokens
        emb = self.encode_images(images)
        return [EncodedImage(emb[i * N:(i + 1) * N]) for i in range(len(images))]

    def tp_tower_ok(self) -> bool:
        """Whether the image tower runs tensor-parallel under this model's TP group (a ViT whose heads /
        MLP width split over the ranks; FastViT towers stay on rank 0)."""
        tp = self.llm.tp
        if not (TP_TOWER and tp.enabled) or self.cfg.vision_arch == "fastvit":
            return False
        from .clip import tp_blocks_ok

        v = self.vision
        n = len(v.blocks) + self.cfg.feature_layer + 1 if self.cfg.feature_layer < 0 else self.cfg.feature_layer
        probe = torch.empty((1, self.cfg.vision.width), device=self.device)
        return tp_blocks_ok(probe, v.blocks[:n], self.cfg.vision.heads, tp.world, False)

    def _encode_tp(self, images: Sequence[torch.Tensor], n: int, out: torch.Tensor) -> None:
        """The TP group's image tower: rank 0 preprocesses the images and broadcasts the patch rows
        (~0.7 MB per 336 px image, vs 4.7 MB of 8B-decoder features), then EVERY rank runs the
        tensor-parallel blocks (clip.run_blocks_tp: its heads / MLP slice, 2 all-reduces per block) and
        the replicated projector, so every rank ends with identical features and none waits on rank
        0's whole tower."""
        import torch.distributed as dist

        tp = self.llm.tp
        v = self.vision
        if tp.rank == 0:
            pre = self.preprocess(list(images[:n]))
        else:
            pre = torch.empty((n * v.num_patches, v.kpad), device=self.device, dtype=v.patch_w.dtype)
        staged = pre.cpu() if dist.get_backend(tp.group) == "gloo" and pre.is_cuda else pre
        dist.broadcast(staged, src=dist.get_global_rank(tp.group, 0) if tp.group is not None else 0, group=tp.group)
        if staged is not pre:
            pre.copy_(staged)
        self._encode_tower(pre, n, out=out, tp=(tp.rank, tp.world, self.llm._all_reduce))

    # ------------------------------------------------------------------ prefill inputs
    def expand_image_tokens(self, ids: Sequence[int], n_images: int) -> tuple[list[int], list[int]]:
        """Replace each ``<image>`` id by N_img placeholder positions -> (ids, image row starts)."""
        N = self.cfg.num_image_tokens
        out, starts = [], []
        used = 0
        for t in ids:
            if t == self.cfg.image_token_id and used < n_images:
                starts.append(len(out))
                out.extend([self.cfg.image_token_id] * N)
                used += 1
            else:
                out.append(int(t))
        return out, starts

    @torch.no_grad()
    def build_prefill(self, ids: Sequence[int], images: Sequence[torch.Tensor],
                      n_images: Optional[int] = None, shard_images: bool = False) -> torch.Tensor:
        """Token embeddings with image rows spliced in -> x [T, hidden] on the model device.

        Tensor parallel: every rank embeds the text (vocab-parallel lookup + all-reduce).
        ``shard_images`` (every rank holds all the images): rank r runs the vision tower +
        projector on images r, r + world, ... only, and ONE all-reduce of the zero-filled
        [n * N_img, hidden] block (disjoint rows: the sum is exact) hands every rank all the
        features -- a multi-image prompt's towers run in parallel across the TP group.
        Otherwise only TP rank 0 holds the images (``n_images`` tells the others how many): with a
        ViT tower (:meth:`tp_tower_ok`) rank 0 broadcasts the patch rows and the whole group runs the
        tower tensor-parallel (:meth:`_encode_tp`); a FastViT tower runs on rank 0 and its features
        are broadcast."""
        n = len(images) if n_images is None else int(n_images)
        full, starts = self.expand_image_tokens(ids, n)
        dev = self.device
        t = h2d_ahead(full, dev, torch.long)
        x = self.llm.embed_tokens(t)
        N = self.cfg.num_image_tokens
        if not starts:
            return x
        tp = self.llm.tp
        contiguous = all(s == starts[0] + i * N for i, s in enumerate(starts))
        if tp.enabled:
            import torch.distributed as dist

            buf = x[starts[0]:starts[0] + N * len(starts)] if contiguous else \
                torch.empty((N * len(starts), x.shape[1]), device=dev, dtype=x.dtype)
            if shard_images:
                buf.zero_()
                for i in range(tp.rank, len(starts), tp.world):
                    self.encode_images([images[i]], out=buf[i * N:(i + 1) * N])
                staged = buf.cpu() if dist.get_backend(tp.group) == "gloo" and buf.is_cuda else buf
                dist.all_reduce(staged, group=tp.group)
                if staged is not buf:
                    buf.copy_(staged)
                if not contiguous:
                    for i, s in enumerate(starts):
                        x[s:s + N] = buf[i * N:(i + 1) * N]
                return x
            if self.tp_tower_ok():
                self._encode_tp(images, len(starts), buf)
                if not contiguous:
                    for i, s in enumerate(starts):
                        x[s:s + N] = buf[i * N:(i + 1) * N]
                return x
            if tp.rank == 0:
                self.encode_images(images[:len(starts)], out=buf)
            staged = buf.cpu() if dist.get_backend(tp.group) == "gloo" and buf.is_cuda else buf
            dist.broadcast(staged, src=dist.get_global_rank(tp.group, 0), group=tp.group)
            if staged is not buf:
                buf.copy_(staged)
            if not contiguous:
                for i, s in enumerate(starts):
                    x[s:s + N] = buf[i * N:(i + 1) * N]
            return x
        imgs = images[:len(starts)]
        if any(isinstance(im, EncodedImage) for im in imgs):
            raw = [im for im in imgs if not isinstance(im, EncodedImage)]
            enc = iter(self.encode_ahead(raw)) if raw else iter(())
            for i, s in enumerate(starts):
                im = imgs[i] if isinstance(imgs[i], EncodedImage) else next(enc)
                x[s:s + N] = im.emb
            return x
        if contiguous:
            self.encode_images(imgs, out=x[starts[0]:starts[0] + N * len(starts)])
        else:
            emb = self.encode_images(imgs)
            for i, s in enumerate(starts):
                x[s:s + N] = emb[i * N:(i + 1) * N]
        return x

    # ------------------------------------------------------------------ weights
    def export_state_dict(self) -> dict:
        """Synthetic-pack layout: ``vision.*`` / ``mm_projector.*`` + HF decoder names."""
        sd = {f"vision.{k}": v for k, v in self.vision.state_dict().items()}
        sd["mm_projector.0.weight"], sd["mm_projector.0.bias"] = self.proj1_w, self.proj1_b
        sd["mm_projector.2.weight"], sd["mm_projector.2.bias"] = self.proj2_w, self.proj2_b
        l = self.llm
        assert l.tp.world == 1
        sd["model.embed_tokens.weight"] = l.embed
        sd["model.norm.weight"] = l.norm
        if l.lm_head is not None:
            sd["lm_head.weight"] = l.lm_head
        D = l.cfg.head_dim
        for i, ly in enumerate(l.layers):
            p = f"model.layers.{i}."
            q, k, v = torch.split(ly.qkv_w, [ly.H * D, ly.Hkv * D, ly.Hkv * D], 0)
            sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.v_proj.weight"] = q, k, v
            if ly.qkv_b is not None:
                bq, bk, bv = torch.split(ly.qkv_b, [ly.H * D, ly.Hkv * D, ly.Hkv * D], 0)
                sd[p + "self_attn.q_proj.bias"], sd[p + "self_attn.k_proj.bias"], sd[p + "self_attn.v_proj.bias"] = bq, bk, bv
            sd[p + "self_attn.o_proj.weight"] = ly.o_w
            gu = ly.gu_w.view(ly.I // 8, 2, 8, -1)
            sd[p + "mlp.gate_proj.weight"] = gu[:, 0].reshape(ly.I, -1)
            sd[p + "mlp.up_proj.weight"] = gu[:, 1].reshape(ly.I, -1)
            sd[p + "mlp.down_proj.weight"] = ly.down_w
            sd[p + "input_layernorm.weight"] = ly.ln1
            sd[p + "post_attention_layernorm.weight"] = ly.ln2
        return {k: v.detach().contiguous() for k, v in sd.items()}

    @torch.no_grad()
    def load_pack_state_dict(self, sd: dict) -> None:
        vis = {k[len("vision."):]: v for k, v in sd.items() if k.startswith("vision.")}
        own = self.vision.state_dict()
        self.vision.load_state_dict({k: vis[k].to(own[k].dtype) for k in own})
        for dst, key in ((self.proj1_w, "mm_projector.0.weight"), (self.proj1_b, "mm_projector.0.bias"),
                         (self.proj2_w, "mm_projector.2.weight"), (self.proj2_b, "mm_projector.2.bias")):
            dst.copy_(sd[key].to(dst.dtype))
        self.llm.load_hf_state_dict(sd)
        self.invalidate_graphs()


# ============================================================================= synthetic pack
CHATML_TEMPLATE = ("{% for message in messages %}<|im_start|>{{ message['role'] }}\n{{ message['content'] }}"
                   "<|im_end|>\n{% endfor %}{% if add_generation_prompt %}<|im_start|>assistant\n{% endif %}")


def write_vlm_model(root, name: str, preset: Optional[str] = None, seed: int = 0, weights: Optional[bool] = None):
    """Synthetic VLM pack: byte-level BPE tokenizer with ChatML specials, chat template,
    ``lumen_vlm_config.json``, ``model.safetensors`` (small presets) or ``random_init``
    (large presets are random-initialised on the device at load), ``model_info.json``
    with the generation / kv-cache / vision metadata the reference backends read."""
    import copy
    import json
    from pathlib import Path

    from ..resources.model_info import ModelInfo
    from ..resources.synthetic import write_byte_bpe_tokenizer

    root = Path(root)
    root.mkdir(parents=True, exist_ok=True)
    n = name.lower()
    preset = preset or ("tiny" if "tiny" in n else "llava-llama3-8b" if ("llava" in n or "8b" in n) else "fastvlm-0.5b")
    cfg = copy.deepcopy(VLM_PRESETS[preset])
    # full-size presets: the tokenizer covers the decoder's whole vocabulary (random-init decoders then
    # generate decodable text, so service benchmarks see real streamed chunks); tiny ones stay byte-only
    tok = write_byte_bpe_tokenizer(root / "tokenizer.json", bos="<|im_start|>", eos="<|im_end|>",
                                   extra_special=["<|endoftext|>", "<image>"], add_bos_eos=False,
                                   fill_vocab=0 if "tiny" in preset else cfg.llm.vocab_size)
    from tokenizers import Tokenizer

    t = Tokenizer.from_file(str(root / "tokenizer.json"))
    cfg.image_token_id = t.token_to_id("<image>")
    cfg.llm.eos_token_id = tok["eos_id"]
    cfg.llm.bos_token_id = tok["bos_id"]
    (root / "tokenizer_config.json").write_text(json.dumps({"chat_template": CHATML_TEMPLATE,
                                                            "eos_token": "<|im_end|>", "bos_token": None}, indent=2))
    (root / "lumen_vlm_config.json").write_text(json.dumps(cfg.to_dict(), indent=2))
    if weights is None:
        weights = preset in ("tiny", "tiny-h8", "tiny-gqa8")
    files = ["tokenizer.json", "tokenizer_config.json", "lumen_vlm_config.json"]
    if weights:
        m = VLM(cfg, dtype=torch.float32, device="cpu")
        m.random_init(seed)
        from safetensors.torch import save_file

        save_file({k: v.to(torch.bfloat16) if v.is_floating_point() and v.dim() > 1 else v
                   for k, v in m.export_state_dict().items()}, str(root / "model.safetensors"))
        files.append("model.safetensors")
    lc = cfg.llm
    info = {
        "name": name, "version": "1.0.0", "description": f"synthetic {preset} VLM pack (random init)",
        "model_type": "vlm", "source": {"format": "custom", "repo_id": f"synthetic/{name}"},
        "runtimes": {"onnx": {"available": True, "files": files, "devices": ["cuda", "cpu"]},
                     "torch": {"available": True, "files": files, "devices": ["cuda", "cpu"]}},
        "extra_metadata": {
            "synthetic": True, "random_init": not weights, "seed": seed, "lumen_preset": preset,
            "generation_config": {"bos_token_id": lc.bos_token_id, "eos_token_id": lc.eos_token_id,
                                  "pad_token_id": tok["eos_id"], "image_token_index": cfg.image_token_id,
                                  "vocab_size": lc.vocab_size, "max_position_embeddings": lc.max_position},
            "kv_cache_config": {"num_hidden_layers": lc.num_layers, "num_attention_heads": lc.num_heads,
                                "num_key_value_heads": lc.num_kv_heads, "hidden_size": lc.hidden_size,
                                "head_dim": lc.head_dim},
            "vision_config": {"image_size": cfg.vision.image_size, "patch_size": cfg.vision.patch_size,
                              "mean": list(cfg.image_mean), "std": list(cfg.image_std)},
        },
    }
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info, indent=2))
    return root
