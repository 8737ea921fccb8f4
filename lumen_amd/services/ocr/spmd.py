"""SPMD image-batch data parallelism for OCR detect + recognise (BASELINE config #4 at DP=N,
the OCR counterpart of :mod:`lumen_amd.services.face.spmd`).

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL on ROCm): every rank owns a
contiguous shard of the global image batch and runs the batched DBNet detector, the GPU DB
post-processing, the fused crop warp and the SVTR recogniser + CTC on its own GPU
(``MI355XOcrBackend._predict_batch``).  Results are variable-length text lines, so each rank
packs them into one fixed-shape fp32 tensor -- per text line: the 4 box corners, the confidence,
the text length and the text's Unicode code points (all < 2^24, exact in fp32) -- and ONE
``all_gather_into_tensor`` (plus one for the per-image line counts) gives every rank all images'
lines in global order.  The reference recognises one image at a time in its gRPC handler
(``packages/lumen-ocr/src/lumen_ocr/general_ocr/ocr_service.py``); the only cross-GPU traffic
here is that result gather.

Row layout per line: [x0, y0, x1, y1, x2, y2, x3, y3, conf, n, cp[0:L]] with L the global
maximum text length (one tiny all-reduce together with the maximum line count).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ...parallel.data_parallel import shard_range
from .backend import OcrParams, OcrResult

HEAD = 10      # box (8) + confidence (1) + text length (1)


def pack_lines(results: Sequence[Sequence[OcrResult]], n_pad: int, maxr: int, maxlen: int
               ) -> tuple[torch.Tensor, torch.Tensor]:
    """[OcrResult] per image -> rows [n_pad, maxr, 10 + maxlen] fp32, counts [n_pad] int32."""
    rows = np.zeros((n_pad, max(maxr, 1), HEAD + max(maxlen, 1)), np.float32)
    counts = np.zeros((n_pad,), np.int32)
    for i, lines in enumerate(results):
        counts[i] = len(lines)
        for j, r in enumerate(lines):
            rows[i, j, 0:8] = np.asarray(r.box, np.float32).reshape(-1)[:8]
            rows[i, j, 8] = r.confidence
            cps = [ord(c) for c in r.text]
            rows[i, j, 9] = len(cps)
            rows[i, j, HEAD:HEAD + len(cps)] = cps
    return torch.from_numpy(rows), torch.from_numpy(counts)


def unpack_lines(rows: np.ndarray, counts: np.ndarray) -> list[list[OcrResult]]:
    out = []
    for i in range(rows.shape[0]):
        lines = []
        for j in range(int(counts[i])):
            r = rows[i, j]
            n = int(r[9])
            box = [(int(r[2 * k]), int(r[2 * k + 1])) for k in range(4)]
            text = "".join(chr(int(c)) for c in r[HEAD:HEAD + n])
            lines.append(OcrResult(box=box, text=text, confidence=float(r[8])))
        out.append(lines)
    return out


class SPMDOcrRunner:
    """Collective over ``comm`` (a :class:`lumen_amd.parallel.Communicator` of the DP group):
    every rank calls :meth:`run` with the SAME global image list and gets every image's lines."""

    def __init__(self, backend, comm, device: Optional[torch.device] = None):
        self.be = backend
        self.comm = comm
        self.device = device if device is not None else backend.device

    def run_local(self, images: Sequence[np.ndarray], params: Sequence[OcrParams]):
        a, b = shard_range(len(images), self.comm.rank, self.comm.world)
        local = self.be._predict_batch(list(zip(images[a:b], params[a:b]))) if b > a else []
        return local, (a, b)

    def gather(self, local: Sequence[Sequence[OcrResult]], n_global: int) -> list[list[OcrResult]]:
        world = self.comm.world
        per = -(-n_global // world)
        mx = torch.tensor([max((len(ls) for ls in local), default=0),
                           max((len(r.text) for ls in local for r in ls), default=0)], dtype=torch.int32,
                          device=self.device)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.comm.group)
        maxr, maxlen = (max(int(v), 1) for v in mx.tolist())
        rows, counts = pack_lines(local, per, maxr, maxlen)
        rows, counts = rows.to(self.device), counts.to(self.device)
        all_rows = torch.empty((world * per,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=self.device)
        all_counts = torch.empty((world * per,), dtype=counts.dtype, device=self.device)
        self.comm.all_gather_into(all_rows, rows)
        self.comm.all_gather_into(all_counts, counts)
        r_np, c_np = all_rows.cpu().numpy(), all_counts.cpu().numpy()
        keep = np.concatenate([np.arange(r * per, r * per + (shard_range(n_global, r, world)[1] -
                                                               shard_range(n_global, r, world)[0]))
                               for r in range(world)])
        return unpack_lines(r_np[keep], c_np[keep])

    def run(self, images: Sequence[np.ndarray], params: Sequence[OcrParams]) -> list[list[OcrResult]]:
        local, _ = self.run_local(images, params)
        return self.gather(local, len(images))
