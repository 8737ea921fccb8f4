"""Reference PP-OCR ONNX packs (``detection*.onnx`` DBNet + ``recognition*.onnx`` SVTR /
PP-LCNet CTC recogniser) on the MI355X graph executor, behind the same call contract as
the native towers (reference packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py:
det output ``[N, 1, H, W]`` probability map; rec output ``[N, T, C]`` softmax scores)."""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import torch

from ...runtime.onnx_graph import OnnxGraph


def find_onnx_pair(root: Path) -> tuple[Optional[Path], Optional[Path]]:
    files = sorted(Path(root).rglob("*.onnx"))
    det = next((f for f in files if "det" in f.name.lower()), None)
    rec = next((f for f in files if f != det and ("rec" in f.name.lower() or "svtr" in f.name.lower())), None)
    return det, rec


def _to_nchw3(x: torch.Tensor) -> torch.Tensor:
    return x[..., :3].permute(0, 3, 1, 2).float().contiguous()


class OnnxDBNet:
    def __init__(self, path, device):
        self.g = OnnxGraph(path, device)

    def eval(self):
        return self

    def to(self, _):
        return self

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        p = self.g.run({self.g.model.graph.inputs[0]: _to_nchw3(x)})[0]
        return p.float().reshape(p.shape[0], p.shape[-2], p.shape[-1])


class OnnxCTCRecognizer:
    def __init__(self, path, device):
        self.g = OnnxGraph(path, device)
        self.time_stride = 4

    def eval(self):
        return self

    def to(self, _):
        return self

    def __call__(self, x: torch.Tensor, valid_w=None) -> torch.Tensor:
        xn = _to_nchw3(x)
        p = self.g.run({self.g.model.graph.inputs[0]: xn})[0].float()
        if p.dim() == 4:                      # [N, 1, T, C] exports
            p = p.squeeze(1)
        self.time_stride = max(1, xn.shape[-1] // p.shape[1])
        # softmax scores -> log-probabilities: the CTC kernel's softmax of these is the scores
        return torch.log(p.clamp_min(1e-30)).contiguous()
