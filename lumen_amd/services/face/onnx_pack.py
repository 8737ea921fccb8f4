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
