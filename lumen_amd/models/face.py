"""Face models: SCRFD-style detector and ArcFace IResNet-50/100 recogniser (NHWC, bf16).

Detector (SCRFD family, reference packs antelopev2 / buffalo_l use SCRFD-10G:
packages/lumen-face/src/lumen_face/backends/insightface_specs.py:11-159):
ResNet-style backbone with three output strides (8/16/32), a top-down FPN and a
head shared across strides predicting, per anchor (A=2 per location),
a class logit, 4 box distances and 10 keypoint distances; all three heads are
one fused conv whose NHWC output is decoded in place by the det_decode kernel
(sigmoid + anchor-centre distance2bbox/kps + un-letterbox + size filter).
The layer graph is a faithful-in-kind re-implementation for random-init
benchmarking; output semantics match the reference's 9-output SCRFD decode.

Recogniser (insightface iresnet50 / iresnet100 = buffalo_l w600k_r50 / antelopev2
glintr100): conv3x3+BN+PReLU stem, IBasicBlocks [3,4,14,3] / [3,13,30,3]
(BN -> conv3x3 -> BN -> PReLU -> conv3x3(stride) -> BN, + shortcut), BN,
flatten 7x7x512 -> FC 512 -> BN1d; BNs after convs are folded into the
implicit-GEMM epilogue, the pre-conv BN of each block is a channel affine, the
final BN1d is folded into the FC, and the 512-d embedding is L2-normalised.
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Optional

import numpy as np
import torch
from torch import nn

from .. import ops
from ..ops import cnn
from .layers import ChannelAffine, ConvBN, Linear, fold_bn

# (r5's 2-stream recogniser -- batch halves block-interleaved on two HIP streams -- tied the single stream,
# 3,318-3,346 vs 3,325-3,344 img/s: the face pipeline already overlaps the next batch's detector with this
# batch's recogniser, profiles/r5_face_micro_v1.txt; it was removed in r6)


# =============================================================================== recogniser
@dataclass
class IResNetConfig:
    layers: tuple = (3, 4, 14, 3)          # r50; r100 = (3, 13, 30, 3)
    widths: tuple = (64, 128, 256, 512)
    embedding: int = 512
    input_size: int = 112


IRESNET_PRESETS = {"r50": IResNetConfig(), "r100": IResNetConfig(layers=(3, 13, 30, 3)),
                   "r18": IResNetConfig(layers=(2, 2, 2, 2)), "tiny": IResNetConfig(layers=(1, 1, 1, 1),
                                                                                    widths=(16, 32, 32, 64),
                                                                                    embedding=64)}


class IBasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.bn1 = ChannelAffine(cin)
        self.conv1 = ConvBN(cin, cout, 3, 1, prelu=True)          # conv1 + bn2 + prelu
        self.conv2 = ConvBN(cout, cout, 3, stride)                 # conv2 + bn3 (+ shortcut)
        self.down = ConvBN(cin, cout, 1, stride, pad=0) if (stride != 1 or cin != cout) else None

    def forward(self, x, xb=None, next_aff=None, next_in_place: bool = False):
        """x: block input; xb: bn1(x) when the previous conv's epilogue already produced it.
        ``next_aff`` (scale, shift): the next layer's pre-conv BN, emitted by conv2's epilogue as
        a second output (returns (out, bn(out))) or, ``next_in_place``, instead of out."""
        sc = self.down(x) if self.down is not None else x
        h = xb if xb is not None else self.bn1(x)
        h = self.conv1(h)
        if next_aff is None:
            return self.conv2(h, residual=sc)
        if next_in_place:
            return self.conv2(h, residual=sc, aff=next_aff)
        return self.conv2(h, residual=sc, aff=next_aff, aff_out=True)


class IResNet(nn.Module):
    def __init__(self, cfg: IResNetConfig = IResNetConfig()):
        super().__init__()
        self.cfg = cfg
        w0 = cfg.widths[0]
        self.stem = ConvBN(3, w0, 3, 1, prelu=True)
        blocks = []
        cin = w0
        for n, w in zip(cfg.layers, cfg.widths):
            for i in range(n):
                blocks.append(IBasicBlock(cin, w, 2 if i == 0 else 1))
                cin = w
        self.blocks = nn.ModuleList(blocks)
        self.bn_out = ChannelAffine(cin)
        hw = cfg.input_size // 16
        self.fc = Linear(cin * hw * hw, cfg.embedding)

    def random_init(self, g: torch.Generator):
        for m in self.modules():
            if isinstance(m, (ConvBN, ChannelAffine)):
                m.random_init(g)
            elif isinstance(m, Linear):
                m.random_init(g)
        # keep the residual stream well scaled at random init
        for b in self.blocks:
            b.conv2.w.data.mul_(0.2)

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: NHWC8 [F, 112, 112, 8] bf16 -> L2-normalised fp32 [F, 512].

        On the GPU every pre-conv BatchNorm (bn1 of each block, the final bn_out) is produced by the
        epilogue of the conv that writes its input -- the stem / the previous block's conv2 writes
        the block output AND its affine -- so no channel-affine pass re-reads the activations (the CPU
        reference runs the separate channel affine)."""
        if not x.is_cuda:
            h = self.stem(x)
            for b in self.blocks:
                h = b(h)
            h = self.bn_out(h)
        else:
            for h in self._fused_steps(x):
                pass
        emb = self.fc(h.reshape(h.shape[0], -1), out_dtype=torch.float32)
        return ops.l2_normalize_(emb.contiguous())

    def _fused_steps(self, x: torch.Tensor):
        """The fused-BN block chain over x, one ``yield`` per block (the last yields the output rows)."""
        b0 = self.blocks[0].bn1
        h, hb = self.stem(x, aff=(b0.scale, b0.shift), aff_out=True)
        n = len(self.blocks)
        for i, b in enumerate(self.blocks):
            if i + 1 < n:
                nb = self.blocks[i + 1].bn1
                h, hb = b(h, hb, (nb.scale, nb.shift))
            else:
                h = b(h, hb, (self.bn_out.scale, self.bn_out.shift), next_in_place=True)
            yield h

    def load_insightface_state_dict(self, sd: dict) -> None:
        """insightface ``iresnet`` PyTorch weights (conv1/bn1/prelu, layerX.Y.*, bn2, fc, features)."""
        def bn(p):
            return {k: sd.get(f"{p}.{k}") for k in ("weight", "bias", "running_mean", "running_var")}

        self.stem.load_torch(sd["conv1.weight"], None, bn("bn1"), sd["prelu.weight"])
        i = 0
        for li, n in enumerate(self.cfg.layers):
            for j in range(n):
                p = f"layer{li + 1}.{j}"
                b = self.blocks[i]
                b.bn1.load_bn(bn(f"{p}.bn1"))
                b.conv1.load_torch(sd[f"{p}.conv1.weight"], None, bn(f"{p}.bn2"), sd[f"{p}.prelu.weight"])
                b.conv2.load_torch(sd[f"{p}.conv2.weight"], None, bn(f"{p}.bn3"))
                if b.down is not None:
                    b.down.load_torch(sd[f"{p}.downsample.0.weight"], None, bn(f"{p}.downsample.1"))
                i += 1
        self.bn_out.load_bn(bn("bn2"))
        # FC expects NCHW flatten (c*HW + p); our activations flatten NHWC (p*C + c)
        C = self.cfg.widths[-1]
        hw = self.cfg.input_size // 16
        w = sd["fc.weight"].float().reshape(-1, C, hw * hw).permute(0, 2, 1).reshape(-1, C * hw * hw)
        b = sd.get("fc.bias")
        feat = bn("features")
        if feat["running_mean"] is not None:
            w, b = fold_bn(w, b, feat)
        self.fc.load_torch(w, b)


# =============================================================================== detector
@dataclass
class SCRFDConfig:
    input_size: int = 640
    stem: int = 32
    widths: tuple = (64, 128, 256)       # strides 8, 16, 32
    depths: tuple = (2, 2, 2)
    fpn: int = 64
    head_convs: int = 2
    anchors: int = 2
    strides: tuple = (8, 16, 32)


SCRFD_PRESETS = {"10g": SCRFDConfig(), "tiny": SCRFDConfig(input_size=128, stem=16, widths=(32, 32, 64),
                                                         depths=(1, 1, 1), fpn=32, head_convs=1)}


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = ConvBN(cin, cout, 3, stride, act="relu")
        self.c2 = ConvBN(cout, cout, 3, 1, act=None, post_act="relu")   # relu(bn(conv) + shortcut)
        self.down = ConvBN(cin, cout, 1, stride, pad=0) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        sc = self.down(x) if self.down is not None else x
        return self.c2(self.c1(x), residual=sc)


class SCRFD(nn.Module):
    def __init__(self, cfg: SCRFDConfig = SCRFDConfig()):
        super().__init__()
        self.cfg = cfg
        s = cfg.stem
        self.stem = nn.ModuleList([ConvBN(3, s, 3, 2, act="relu"), ConvBN(s, s, 3, 1, act="relu"),
                                   ConvBN(s, s * 2 if s * 2 <= cfg.widths[0] else s, 3, 2, act="relu")])
        cin = self.stem[-1].cout
        stages = []
        for i, (w, d) in enumerate(zip(cfg.widths, cfg.depths)):
            blocks = []
            for j in range(d):
                blocks.append(BasicBlock(cin, w, 2 if j == 0 else 1))
                cin = w
            stages.append(nn.ModuleList(blocks))
        self.stages = nn.ModuleList(stages)
        self.lateral = nn.ModuleList([ConvBN(w, cfg.fpn, 1, 1, pad=0) for w in cfg.widths])
        self.fpn_out = nn.ModuleList([ConvBN(cfg.fpn, cfg.fpn, 3, 1, act="relu") for _ in cfg.widths])
        self.head_convs = nn.ModuleList([ConvBN(cfg.fpn, cfg.fpn, 3, 1, act="relu") for _ in range(cfg.head_convs)])
        A = cfg.anchors
        self.head_out = ConvBN(cfg.fpn, A * 15, 3, 1)       # [cls A | bbox 4A | kps 10A] (padded to 32)

    def random_init(self, g: torch.Generator):
        for m in self.modules():
            if isinstance(m, ConvBN):
                m.random_init(g)
        A = self.cfg.anchors
        # bias the class logits negative (few positives), distances ~1 stride
        self.head_out.b.data[:A] = -4.0
        self.head_out.b.data[A:5 * A] = 1.0

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> list[torch.Tensor]:
        """x NHWC8 [N, S, S, 8] -> list of fused head maps [N, S/s, S/s, 32] (fp32) for strides 8/16/32."""
        h = x
        for c in self.stem:
            h = c(h)
        feats = []
        for st in self.stages:
            for b in st:
                h = b(h)
            feats.append(h)
        lat = [l(f) for l, f in zip(self.lateral, feats)]
        # top-down: P5 -> P4 -> P3
        for i in range(len(lat) - 1, 0, -1):
            lat[i - 1] = cnn.upsample_add(lat[i], lat[i - 1], 2)
        outs = []
        for i, p in enumerate(lat):
            t = self.fpn_out[i](p)
            for hc in self.head_convs:
                t = hc(t)
            outs.append(self.head_out(t, out_dtype=torch.float32))
        return outs


# =============================================================================== synthetic artefacts
def write_face_model(root: Path, name: str, det_preset: str = "10g", rec_preset: Optional[str] = None,
                     seed: int = 0) -> Path:
    """Random-init SCRFD + IResNet pack in the reference's directory layout."""
    from safetensors.torch import save_file

    from ..resources.model_info import ModelInfo

    root = Path(root)
    root.mkdir(parents=True, exist_ok=True)
    rec_preset = rec_preset or ("r100" if "antelope" in name.lower() else "r50")
    if "tiny" in name.lower():
        det_preset, rec_preset = "tiny", "tiny"
    g = torch.Generator().manual_seed(seed)
    det = SCRFD(SCRFD_PRESETS[det_preset])
    det.random_init(g)
    rec = IResNet(IRESNET_PRESETS[rec_preset])
    rec.random_init(g)
    save_file({k: v.contiguous() for k, v in det.state_dict().items()}, str(root / "detection.safetensors"))
    save_file({k: v.contiguous() for k, v in rec.state_dict().items()}, str(root / "recognition.safetensors"))
    dcfg, rcfg = SCRFD_PRESETS[det_preset], IRESNET_PRESETS[rec_preset]
    meta = {"det": asdict(dcfg), "rec": asdict(rcfg), "det_preset": det_preset, "rec_preset": rec_preset}
    (root / "lumen_face_config.json").write_text(json.dumps(meta, indent=2))
    files = ["detection.safetensors", "recognition.safetensors", "lumen_face_config.json"]
    info = {
        "name": name, "version": "1.0.0", "description": f"synthetic SCRFD-{det_preset} + IResNet-{rec_preset} face pack",
        "model_type": "face", "embedding_dim": rcfg.embedding,
        "source": {"format": "custom", "repo_id": f"synthetic/{name}"},
        "runtimes": {"torch": {"available": True, "files": files, "devices": ["cuda", "cpu"]},
                     "onnx": {"available": True, "files": files, "devices": ["cuda", "cpu"]}},
        "extra_metadata": {"synthetic": True,
                           "insightface": {"detection": {"type": "scrfd", "input_size": [dcfg.input_size] * 2,
                                                         "mean": 127.5, "std": 128.0, "strides": list(dcfg.strides),
                                                         "num_anchors": dcfg.anchors},
                                           "recognition": {"input_size": [112, 112], "mean": 127.5, "std": 127.5,
                                                           "embedding_size": rcfg.embedding}}},
    }
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info, indent=2))
    return root
