"""Reference (InsightFace) ONNX face packs on the MI355X graph executor.

A pack directory that holds the reference's ONNX files (``detection*.onnx`` / ``det_*.onnx``
/ ``scrfd*.onnx`` and ``recognition*.onnx`` / ``w600k*.onnx`` / ``glintr*.onnx``) instead
of the native ``lumen_face_config.json`` + safetensors is served through
:class:`lumen_amd.runtime.onnx_graph.OnnxGraph`.  The adapters give the backend the same
call contract as the native towers:

* detector: SCRFD's nine outputs (score / bbox / kps per stride 8/16/32, InsightFace order;
  reference insightface_specs.py output index map) -> one fused NHWC head per stride
  ``[N, H, W, 15A]`` (score logits | bbox distances | kps distances), which the HIP
  ``det_decode`` + NMS kernels consume unchanged;
* detector, any other ``type`` (reference ``detector_type`` "retinaface", the default of a
  non-SCRFD pack; onnxrt_backend.py:810-880): outputs picked by the ``outputs`` index map
  (``boxes`` / ``scores`` / ``landmarks``) and returned as ``(scores [N, P], boxes [N, P, 4],
  landmarks [N, P, 10] | None)``.  ``box_encoding`` says what the boxes are:
  ``"decoded"`` (the reference's contract: corner boxes in input pixels, or normalised to the
  original image with ``normalized_boxes``) -> ``vision.det_decode_boxes``; ``"priors"`` (a raw
  RetinaFace export: centre / size regressions against the prior grid of ``steps`` /
  ``min_sizes`` with ``variance``) -> ``vision.det_decode_priors``.  Two-column class scores
  (background, face) take the face column (softmax first when they are logits);
* recogniser: aligned 112x112 crops -> L2-normalised embeddings.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional

import torch

from ... import ops
from ...runtime.onnx_graph import OnnxGraph

DET_HINTS = ("det", "scrfd", "retina")
REC_HINTS = ("rec", "w600k", "glint", "arcface", "r50", "r100", "mbf")


def find_onnx_pair(root: Path) -> tuple[Optional[Path], Optional[Path]]:
    files = sorted(Path(root).rglob("*.onnx"))
    det = next((f for f in files if any(h in f.name.lower() for h in DET_HINTS)), None)
    rec = next((f for f in files if f != det and any(h in f.name.lower() for h in REC_HINTS)), None)
    return det, rec


@dataclass
class _DetCfg:
    input_size: int = 640
    strides: list = field(default_factory=lambda: [8, 16, 32])
    anchors: int = 2


@dataclass
class _RecCfg:
    input_size: int = 112
    embedding: int = 512


def _to_nchw3(x: torch.Tensor) -> torch.Tensor:
    """NHWC8 (image_prep / warp_batch layout) -> NCHW fp32 RGB."""
    return x[..., :3].permute(0, 3, 1, 2).float().contiguous()


class OnnxSCRFD:
    def __init__(self, path, device, spec: dict):
        self.g = OnnxGraph(path, device)
        self.cfg = _DetCfg(int(spec.get("input_size", (640, 640))[0]), list(spec.get("strides", [8, 16, 32])),
                           int(spec.get("num_anchors", 2)))
        self.outmap = spec.get("outputs") or [{"stride": s, "score": i, "bbox": i + 3, "kps": i + 6}
                                              for i, s in enumerate(self.cfg.strides)]

    def eval(self):
        return self

    def to(self, _):
        return self

    def _run(self, x: torch.Tensor) -> list:
        outs = self.g.run({self.g.model.graph.inputs[0]: x})
        if outs[0].dim() == 2:               # batch-1 export ([P, C] outputs)
            outs = [o.unsqueeze(0) for o in outs]
        return outs

    def __call__(self, x: torch.Tensor) -> list:
        xn = _to_nchw3(x)
        N, S, A = xn.shape[0], self.cfg.input_size, self.cfg.anchors
        outs = self._run(xn)
        if outs[0].shape[0] != N:            # fixed-batch-1 graph: run image by image
            per = [self._run(xn[i:i + 1]) for i in range(N)]
            outs = [torch.cat([p[j] for p in per]) for j in range(len(per[0]))]
        heads = []
        for m in self.outmap:
            s = int(m["stride"])
            H = W = S // s
            sc = outs[m["score"]].float().reshape(N, H, W, A).clamp(1e-7, 1 - 1e-7)
            logit = torch.log(sc) - torch.log1p(-sc)            # decode kernel applies the sigmoid
            bb = outs[m["bbox"]].float().reshape(N, H, W, 4 * A)
            kp = outs[m["kps"]].float().reshape(N, H, W, 10 * A) if m.get("kps") is not None and \
                m["kps"] < len(outs) else torch.zeros(N, H, W, 10 * A, device=sc.device)
            heads.append(torch.cat([logit, bb, kp], dim=-1).contiguous())
        return heads


@dataclass
class _BoxDetCfg:
    input_size: int = 640
    strides: list = field(default_factory=list)
    anchors: int = 1


class OnnxBoxDetector:
    """Non-SCRFD detector export (RetinaFace family / generic): see the module docstring."""

    def __init__(self, path, device, spec: dict):
        self.g = OnnxGraph(path, device)
        self.cfg = _BoxDetCfg(int(spec.get("input_size", (640, 640))[0]))
        self.kind = "priors" if str(spec.get("box_encoding", "decoded")).lower() == "priors" else "decoded"
        om = spec.get("outputs")
        if not isinstance(om, dict):        # a SCRFD-style list does not apply: reference defaults
            om = {}
        self.idx = {"boxes": om.get("boxes", 0), "scores": om.get("scores", 1), "landmarks": om.get("landmarks", 2)}
        self.normalized = bool(spec.get("normalized_boxes", False))
        self.score_act = str(spec.get("score_activation", "auto")).lower()
        self.var = tuple(float(v) for v in spec.get("variance", (0.1, 0.2)))
        self.priors = None
        if self.kind == "priors":
            from ...ops.vision import retinaface_priors

            S = self.cfg.input_size
            self.priors = retinaface_priors((S, S), tuple(spec.get("steps", (8, 16, 32))),
                                            tuple(tuple(m) for m in spec.get("min_sizes", ((16, 32), (64, 128),
                                                                                            (256, 512))))
                                            ).to(device)

    def eval(self):
        return self

    def to(self, _):
        return self

    def _run(self, x: torch.Tensor) -> list:
        return self.g.run({self.g.model.graph.inputs[0]: x})

    def _scores(self, sc: torch.Tensor, N: int) -> torch.Tensor:
        sc = sc.float().reshape(N, -1, sc.shape[-1]) if sc.dim() >= 2 and sc.shape[-1] in (1, 2) else \
            sc.float().reshape(N, -1, 1)
        if sc.shape[-1] == 2:
            logits = self.score_act == "softmax" or (self.score_act == "auto" and
                                                     bool(((sc < 0) | (sc > 1)).any()))
            if logits:
                sc = torch.softmax(sc, -1)
            sc = sc[..., 1:]
        elif self.score_act == "sigmoid":
            sc = torch.sigmoid(sc)
        return sc[..., 0].contiguous()

    def __call__(self, x: torch.Tensor):
        xn = _to_nchw3(x)
        N = xn.shape[0]
        outs = self._run(xn)
        b0 = outs[self.idx["boxes"]]
        if b0.dim() >= 2 and b0.shape[0] != N and N > 1:    # fixed-batch-1 graph: image by image
            per = [self._run(xn[i:i + 1]) for i in range(N)]
            outs = [torch.cat([p[j] for p in per]) for j in range(len(per[0]))]
        boxes = outs[self.idx["boxes"]].float()
        C = boxes.shape[-1]
        boxes = boxes.reshape(N, -1, C)
        si, li = self.idx["scores"], self.idx["landmarks"]
        if si is not None and si < len(outs):
            scores = self._scores(outs[si], N)
        elif C >= 5:                                          # [x1 y1 x2 y2 score] rows
            scores = boxes[..., 4].contiguous()
        else:
            scores = torch.ones(boxes.shape[:2], device=boxes.device)
        boxes = boxes[..., :4].contiguous()
        kps = None
        if li is not None and li < len(outs):
            k = outs[li].float()
            if k.numel() == boxes.shape[0] * boxes.shape[1] * 10:
                kps = k.reshape(N, -1, 10).contiguous()
        P = min(boxes.shape[1], scores.shape[1])
        return scores[:, :P].contiguous(), boxes[:, :P].contiguous(), None if kps is None else kps[:, :P].contiguous()

    def decode(self, out, thresh, img_scale, img_hw, cand, count, min_size, max_size):
        """Candidate rows of one batch (``vision`` decode kernels), as the SCRFD heads' decode."""
        from ...ops import vision

        scores, boxes, kps = out
        if self.kind == "priors":
            S = float(self.cfg.input_size)
            vision.det_decode_priors(scores, boxes, kps, self.priors, thresh, img_scale, img_hw, cand, count, (S, S),
                                     var=self.var, min_size=min_size, max_size=max_size)
        else:
            vision.det_decode_boxes(scores, boxes, kps, thresh, img_scale, img_hw, cand, count,
                                    (-1.0, -1.0) if self.normalized else (1.0, 1.0), min_size, max_size)

    @staticmethod
    def select(out, sel):
        return tuple(None if t is None else t.index_select(0, sel) for t in out)


def make_detector(path, device, spec: dict):
    """The ONNX detector adapter for a pack's detection spec (``type``: "scrfd" or any other)."""
    if str(spec.get("type", "scrfd")).lower() == "scrfd":
        return OnnxSCRFD(path, device, spec)
    return OnnxBoxDetector(path, device, spec)


class OnnxArcFace:
    def __init__(self, path, device, spec: dict):
        self.g = OnnxGraph(path, device)
        self.cfg = _RecCfg(int(spec.get("input_size", (112, 112))[0]), int(spec.get("embedding_dim", 512)))

    def eval(self):
        return self

    def to(self, _):
        return self

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        xn = _to_nchw3(x)
        name = self.g.model.graph.inputs[0]
        e = self.g.run({name: xn})[0]
        if e.shape[0] != xn.shape[0]:
            e = torch.cat([self.g.run({name: xn[i:i + 1]})[0] for i in range(xn.shape[0])])
        e = e.float().reshape(xn.shape[0], -1).contiguous()
        return ops.l2_normalize_(e)
