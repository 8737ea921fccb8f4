"""SPMD image-batch data parallelism for face detect + embed (BASELINE config #3: "DP=8
image-batch over xGMI (RCCL all-gather)").

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL on ROCm): every rank owns
a contiguous shard of the global image batch, runs the batched detector + recogniser on its
own GPU (``MI355XFaceBackend.detect_and_embed_images``), packs its results into one fixed-shape
fp32 tensor and ONE ``all_gather_into_tensor`` gives every rank all images' faces in global
order.  The reference does detect -> crop -> embed one image at a time in the gRPC handler
(``packages/lumen-face/src/lumen_face/general_face/face_service.py:516-574``); here the whole
batch is one launch sequence per GPU and the only cross-GPU traffic is the result gather
(per face 15 + D floats: bbox, confidence, 5 landmarks, embedding).

Packed row layout per face: [x1, y1, x2, y2, conf, lx0, ly0, ..., lx4, ly4, emb[0:D]];
per image up to ``maxf`` rows (the global maximum face count, one tiny all-reduce), plus an
int32 face count per image.  Shards differ by at most one image; the gather pads every rank
to ceil(n / world) images and the padding is dropped on unpack.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ...parallel.data_parallel import shard_range
from .backend import DetParams, FaceDetection

HEAD = 15      # bbox (4) + confidence (1) + 5 landmarks (10)


def pack_faces(results: Sequence[Sequence[tuple]], n_pad: int, maxf: int, dim: int) -> tuple[torch.Tensor, torch.Tensor]:
    """[(FaceDetection, emb)] per image -> rows [n_pad, maxf, 15 + dim] fp32, counts [n_pad] int32."""
    rows = np.zeros((n_pad, max(maxf, 1), HEAD + dim), np.float32)
    counts = np.zeros((n_pad,), np.int32)
    for i, faces in enumerate(results):
        counts[i] = len(faces)
        for j, (f, e) in enumerate(faces):
            rows[i, j, 0:4] = f.bbox
            rows[i, j, 4] = f.confidence
            if f.landmarks is not None:
                rows[i, j, 5:15] = np.asarray(f.landmarks, np.float32).reshape(-1)[:10]
            rows[i, j, HEAD:] = e
    return torch.from_numpy(rows), torch.from_numpy(counts)


def unpack_faces(rows: np.ndarray, counts: np.ndarray) -> list[list[tuple[FaceDetection, np.ndarray]]]:
    out = []
    for i in range(rows.shape[0]):
        faces = []
        for j in range(int(counts[i])):
            r = rows[i, j]
            lm = [(float(r[5 + 2 * k]), float(r[6 + 2 * k])) for k in range(5)]
            faces.append((FaceDetection(bbox=tuple(float(x) for x in r[0:4]), confidence=float(r[4]), landmarks=lm),
                          r[HEAD:].copy()))
        out.append(faces)
    return out


class SPMDFaceRunner:
    """Collective over ``comm`` (a :class:`lumen_amd.parallel.Communicator` of the DP group):
    every rank calls :meth:`run` with the SAME global image list and gets every image's faces."""

    def __init__(self, backend, comm, device: Optional[torch.device] = None):
        self.be = backend
        self.comm = comm
        self.device = device if device is not None else backend.device
        self.dim = int(backend.rec.cfg.embedding)

    def run_local(self, images: Sequence[np.ndarray], params: Sequence[DetParams], max_faces: int = -1):
        a, b = shard_range(len(images), self.comm.rank, self.comm.world)
        return self.be.detect_and_embed_images(list(images[a:b]), list(params[a:b]), max_faces), (a, b)

    def gather(self, local: Sequence[Sequence[tuple]], n_global: int) -> list[list[tuple[FaceDetection, np.ndarray]]]:
        world = self.comm.world
        per = -(-n_global // world)
        mx = torch.tensor([max((len(f) for f in local), default=0)], dtype=torch.int32, device=self.device)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.comm.group)
        maxf = max(int(mx.item()), 1)
        rows, counts = pack_faces(local, per, maxf, self.dim)
        # ONE all-gather: each image's face count rides in an extra leading row of its block
        # (exact in fp32), uploaded through pinned memory
        blk = torch.zeros((per, maxf + 1, rows.shape[2]), dtype=torch.float32)
        blk[:, 0, 0] = counts.float()
        blk[:, 1:] = rows
        from ...utils.h2d import h2d

        blk = h2d(blk, self.device)
        all_blk = torch.empty((world * per,) + tuple(blk.shape[1:]), dtype=blk.dtype, device=self.device)
        self.comm.all_gather_into(all_blk, blk)
        a_np = all_blk.cpu().numpy()
        r_np, c_np = a_np[:, 1:], a_np[:, 0, 0].astype(np.int32)
        keep = np.concatenate([np.arange(r * per, r * per + (shard_range(n_global, r, world)[1] -
                                                               shard_range(n_global, r, world)[0]))
                               for r in range(world)])
        return unpack_faces(r_np[keep], c_np[keep])

    def run(self, images: Sequence[np.ndarray], params: Sequence[DetParams], max_faces: int = -1):
        local, _ = self.run_local(images, params, max_faces)
        return self.gather(local, len(images))
