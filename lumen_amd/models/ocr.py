"""OCR models: DBNet text detector + SVTR-LCNet CTC recogniser (NHWC, bf16).

Reference behaviour: packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py
(PP-OCR det/rec ONNX pair).  The detector is a PP-LCNet-style backbone
(depthwise-separable blocks with hardswish and SE in the last stage) producing
strides 4/8/16/32, a DB-FPN neck (1x1 laterals, top-down nearest-upsample adds,
3x3 smoothing convs whose outputs are upsampled straight into channel slices of
one stride-4 concat buffer) and the DB head (3x3 conv-BN-ReLU, two 2x2 stride-2
transposed convs, sigmoid) -> probability map at input resolution.
The recogniser is an LCNet backbone with (2, 1) strides that collapses height
48 -> 1 while keeping width/8 time steps, an SVTR-style global-attention neck
(pre-LN transformer blocks over the width sequence, padded steps masked through
the attention kernel's kv_len) and a CTC classifier whose logits feed the fused
softmax/arg-max/collapse kernel.

Transposed convs (kernel 2, stride 2) are GEMMs [HW, Cin] x [Cin, 4*Cout] followed
by a pixel shuffle; BN after them is folded into the GEMM rows.  Layer graphs are
faithful in kind (random-init benchmarking); output semantics match the
reference (prob map; [B, T, C] class scores with blank = 0).
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Optional, Sequence

import torch
from torch import nn

from .. import ops
from ..ops import cnn
from .clip import _Block, run_blocks
from ..ops import vision
from .layers import ConvBN, DWConvBN, Linear


# ============================================================================= blocks
class SE(nn.Module):
    """squeeze-excite: avgpool -> FC(C/r) ReLU -> FC(C) hardsigmoid -> channel scale."""

    def __init__(self, c: int, r: int = 4):
        super().__init__()
        self.fc1 = Linear(c, c // r, act="relu")
        self.fc2 = Linear(c // r, c, act="hardsigmoid", dtype=torch.bfloat16)

    def random_init(self, g):
        self.fc1.random_init(g)
        self.fc2.random_init(g)

    def forward(self, x):
        s = cnn.global_avgpool(x).to(self.fc1.w.dtype if x.is_cuda else torch.float32)
        s = self.fc2(self.fc1(s), out_dtype=torch.float32)
        return cnn.channel_scale_(x, s)


class DSBlock(nn.Module):
    """depthwise kxk (stride) hardswish -> [SE] -> pointwise 1x1 hardswish (LCNet)."""

    def __init__(self, cin: int, cout: int, k: int, stride, se: bool):
        super().__init__()
        self.dw = DWConvBN(cin, k, stride, act="hardswish")
        self.se = SE(cin) if se else None
        self.pw = ConvBN(cin, cout, 1, 1, pad=0, act="hardswish")

    def random_init(self, g):
        self.dw.random_init(g)
        self.pw.random_init(g)
        if self.se is not None:
            self.se.random_init(g)

    def forward(self, x):
        h = self.dw(x)
        if self.se is not None:
            h = self.se(h)
        return self.pw(h)


class ConvT2(nn.Module):
    """2x2 stride-2 transposed conv (+folded BN) as GEMM + pixel shuffle."""

    def __init__(self, cin: int, cout: int, act=None, out_dtype=None):
        super().__init__()
        self.cin, self.cout, self.out_dtype = cin, cout, out_dtype
        self.g = Linear(cin, 4 * cout, act=act)

    def random_init(self, g):
        self.g.random_init(g, std=(2.0 / self.cin) ** 0.5)

    def load_torch(self, w: torch.Tensor, b: Optional[torch.Tensor] = None, bn: Optional[dict] = None):
        """w: ConvTranspose2d weight [Cin, Cout, 2, 2]."""
        wf, bf = w.float(), (b.float() if b is not None else torch.zeros(w.shape[1]))
        if bn is not None:
            s = bn["weight"].float() / torch.sqrt(bn["running_var"].float() + 1e-5)
            wf = wf * s.view(1, -1, 1, 1)
            bf = bf * s + bn["bias"].float() - bn["running_mean"].float() * s
        self.g.load_torch(wf.permute(2, 3, 1, 0).reshape(4 * self.cout, self.cin), bf.repeat(4))

    def gemm(self, x):
        N, H, W, C = x.shape
        return self.g(x.reshape(-1, C), out_dtype=self.out_dtype).reshape(N, H, W, 4 * self.cout)

    def forward(self, x):
        return cnn.pixel_shuffle_up(self.gemm(x), self.cout, 2)


# ============================================================================= detector
@dataclass
class DBNetConfig:
    stem: int = 16
    # (kernel, out_channels, stride, se)
    blocks: tuple = ((3, 32, 1, 0), (3, 64, 2, 0), (3, 64, 1, 0), (3, 128, 2, 0), (3, 128, 1, 0),
                     (5, 256, 2, 0), (5, 256, 1, 0), (5, 256, 1, 0), (5, 512, 2, 1), (5, 512, 1, 1))
    taps: tuple = (2, 4, 7, 9)   # block outputs at strides 4 / 8 / 16 / 32
    fpn: int = 96
    branch: int = 32


DBNET_PRESETS = {"mobile": DBNetConfig(),
                 "tiny": DBNetConfig(stem=16, blocks=((3, 16, 1, 0), (3, 32, 2, 0), (3, 32, 2, 0), (3, 64, 2, 0),
                                                      (3, 64, 2, 1)), taps=(1, 2, 3, 4), fpn=32, branch=16)}


class DBNet(nn.Module):
    def __init__(self, cfg: DBNetConfig = DBNetConfig()):
        super().__init__()
        self.cfg = cfg
        self.stem = ConvBN(3, cfg.stem, 3, 2, act="hardswish")
        blocks, cin = [], cfg.stem
        for k, c, s, se in cfg.blocks:
            blocks.append(DSBlock(cin, c, k, s, bool(se)))
            cin = c
        self.blocks = nn.ModuleList(blocks)
        tap_c = [cfg.blocks[i][1] for i in cfg.taps]
        self.lateral = nn.ModuleList([ConvBN(c, cfg.fpn, 1, 1, pad=0) for c in tap_c])
        self.smooth = nn.ModuleList([ConvBN(cfg.fpn, cfg.branch, 3, 1) for _ in tap_c])
        cat = cfg.branch * len(tap_c)
        self.head_conv = ConvBN(cat, cat // 4, 3, 1, act="relu")
        self.up1 = ConvT2(cat // 4, cat // 4, act="relu")
        self.up2 = ConvT2(cat // 4, 1, act="sigmoid", out_dtype=torch.float32)

    def random_init(self, g: torch.Generator):
        for m in self.modules():
            if isinstance(m, (ConvBN, DWConvBN)):
                m.random_init(g)
            elif isinstance(m, (SE, ConvT2)):
                m.random_init(g)

    def _head_weights(self, device):
        """(w1 [4C, C], b1 [4C], w2p [4, 64, 8], b2 [4]) of the fused head tail, rebuilt when the
        ConvT2 weights change (load / random_init bump the parameters' versions)."""
        g1, g2 = self.up1.g, self.up2.g
        key = (str(device), g1.w.data_ptr(), g1.w._version, g1.b._version, g2.w.data_ptr(), g2.w._version,
               g2.b._version)
        c = getattr(self, "_head_cache", None)
        if c is None or c[0] != key:
            C = self.up1.cout
            w1 = g1.w[:4 * C, :C].to(device=device, dtype=torch.bfloat16).contiguous()
            b1 = g1.b[:4 * C].to(device=device, dtype=torch.float32).contiguous()
            w2p = cnn.db_head_pack_up2(g2.w[:4, :C]).to(device)
            b2 = g2.b[:4].to(device=device, dtype=torch.float32).contiguous()
            c = self._head_cache = (key, (w1, b1, w2p, b2))
        return c[1]

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x NHWC8 [N, H, W, 8] (H, W multiples of 32) -> probability map fp32 [N, H, W]."""
        h = self.stem(x)
        feats = []
        for i, b in enumerate(self.blocks):
            h = b(h)
            if i in self.cfg.taps:
                feats.append(h)
        lat = [l(f) for l, f in zip(self.lateral, feats)]
        for i in range(len(lat) - 1, 0, -1):
            lat[i - 1] = cnn.upsample_add(lat[i], lat[i - 1], 2)
        N, H4, W4, _ = lat[0].shape
        br = self.cfg.branch
        cat = torch.empty((N, H4, W4, br * len(lat)), device=x.device, dtype=lat[0].dtype)
        # finest level last in the concat, coarse levels upsampled straight into their slice
        L = len(lat)
        for i, p in enumerate(lat):
            sl = cat[..., (L - 1 - i) * br:(L - i) * br]
            if i == 0:
                self.smooth[i](p, out=sl)
            else:
                cnn.upsample_add(self.smooth[i](p), None, 2 ** i, out=sl)
        h = self.head_conv(cat)
        if h.is_cuda and h.shape[-1] in (16, 32) and self.up1.cout == h.shape[-1] and self.up2.cout == 1:
            # up1 + ReLU + shuffle + up2 + sigmoid + the final interleave in one MFMA pass (ops.cnn.db_head_up)
            return cnn.db_head_up(h, *self._head_weights(h.device))
        h = self.up1(h)
        y = self.up2.gemm(h)                         # [N, H/2, W/2, 4] fp32, sigmoid applied
        N, Hh, Wh, _ = y.shape
        return y.view(N, Hh, Wh, 2, 2).permute(0, 1, 3, 2, 4).reshape(N, 2 * Hh, 2 * Wh)


# ============================================================================= recogniser
@dataclass
class RecConfig:
    height: int = 48
    stem: int = 16
    # (kernel, out_channels, (stride_h, stride_w), se); stem is stride 2
    blocks: tuple = ((3, 32, (1, 1), 0), (3, 64, (2, 2), 0), (3, 64, (1, 1), 0), (3, 128, (2, 2), 0),
                     (3, 128, (1, 1), 0), (5, 256, (2, 1), 0), (5, 256, (1, 1), 0), (5, 256, (1, 1), 0),
                     (5, 512, (1, 1), 1), (5, 512, (1, 1), 1))
    dim: int = 128
    heads: int = 4
    depth: int = 2
    mlp: int = 256
    num_classes: int = 6625        # ppocr_keys_v1 (6623) + space + blank


REC_PRESETS = {"mobile": RecConfig(),
               "tiny": RecConfig(stem=16, blocks=((3, 32, (2, 2), 0), (3, 32, (2, 2), 0), (3, 64, (2, 1), 1)),
                                 dim=64, heads=2, depth=1, mlp=128, num_classes=97)}


def _stride_h(s):
    return s[0] if isinstance(s, (tuple, list)) else s


class SVTRRecognizer(nn.Module):
    def __init__(self, cfg: RecConfig = RecConfig()):
        super().__init__()
        self.cfg = cfg
        self.stem = ConvBN(3, cfg.stem, 3, 2, act="hardswish")
        blocks, cin, h = [], cfg.stem, cfg.height // 2
        for k, c, s, se in cfg.blocks:
            blocks.append(DSBlock(cin, c, k, tuple(s), bool(se)))
            cin = c
            h = (h + _stride_h(s) - 1) // _stride_h(s)
        self.blocks = nn.ModuleList(blocks)
        self.feat_h = h
        self.proj = ConvBN(cin, cfg.dim, 1, 1, pad=0, act="hardswish")
        self.tblocks = nn.ModuleList([_Block(cfg.dim, cfg.mlp, torch.bfloat16, None) for _ in range(cfg.depth)])
        self.ln_w = nn.Parameter(torch.ones(cfg.dim, dtype=torch.bfloat16), requires_grad=False)
        self.ln_b = nn.Parameter(torch.zeros(cfg.dim, dtype=torch.bfloat16), requires_grad=False)
        self.cls = Linear(cfg.dim, cfg.num_classes)
        with torch.no_grad():  # padded class columns never win the arg-max / add no softmax mass
            self.cls.b.data[cfg.num_classes:] = -1e9

    @property
    def time_stride(self) -> int:
        s = 2
        for _, _, st, _ in self.cfg.blocks:
            s *= st[1] if isinstance(st, (tuple, list)) else st
        return s

    def random_init(self, g: torch.Generator):
        for m in self.modules():
            if isinstance(m, (ConvBN, DWConvBN)):
                m.random_init(g)
            elif isinstance(m, SE):
                m.random_init(g)
        for b in self.tblocks:
            b.random_init(g, self.cfg.depth)
        self.cls.random_init(g, std=0.05)
        self.cls.b.data[self.cfg.num_classes:] = -1e9

    @torch.no_grad()
    def forward(self, x: torch.Tensor, valid_w: Optional[Sequence[int]] = None) -> torch.Tensor:
        """x NHWC8 [B, 48, W, 8] -> class logits fp32 [B, T, Cpad] (T = W / time_stride; columns
        >= num_classes carry -1e9).  ``valid_w`` masks width padding in the attention."""
        hn, B, T = self.features(x, valid_w)
        logits = ops.linear(hn, self.cls.w, self.cls.b, out_dtype=torch.float32)
        return logits.view(B, T, -1)

    @torch.no_grad()
    def ctc_decode(self, x: torch.Tensor, valid_w: Optional[Sequence[int]] = None, blank: int = 0):
        """x -> greedy CTC (ids per crop, mean confidence per crop).  On the GPU the classifier is
        fused with the per-step arg-max (csrc/postproc.hip cls_argmax_kernel): the [B, T, classes]
        logits (~650 MB fp32 for a PP-OCR batch) are never written."""
        hn, B, T = self.features(x, valid_w)
        return self.ctc_from_features(hn, B, T, valid_w, blank)

    @torch.no_grad()
    def ctc_from_features(self, hn: torch.Tensor, B: int, T: int, valid_w: Optional[Sequence[int]] = None,
                          blank: int = 0):
        """classifier + greedy CTC of :meth:`features` output (fused on the GPU, see ctc_decode)."""
        ts = self.time_stride
        tlen = None if valid_w is None else [-(-int(w) // ts) for w in valid_w]
        if hn.is_cuda and self.cls.cin_p in (64, 128, 256) and hn.shape[1] == self.cls.cin_p:
            return vision.cls_ctc_greedy(hn, self.cls.w, self.cls.b, self.cfg.num_classes, B, T, blank=blank,
                                         tlen=tlen)
        logits = ops.linear(hn, self.cls.w, self.cls.b, out_dtype=torch.float32).view(B, T, -1)
        return vision.ctc_greedy(logits, blank=blank, from_logits=True, tlen=tlen)

    def features(self, x: torch.Tensor, valid_w: Optional[Sequence[int]] = None):
        """x -> final-LayerNorm sequence features [B*T, dim] bf16 (the classifier input), B, T."""
        h = self.stem(x)
        for b in self.blocks:
            h = b(h)
        B, Hf, T, C = h.shape
        if Hf > 1:
            h = cnn.pool2d(h, (Hf, 1), (Hf, 1), 0, is_max=False)
        h = self.proj(h)                                # [B, 1, T, D]
        D = self.cfg.dim
        seq = h.reshape(B * T, D).contiguous()
        kv = None
        if valid_w is not None:
            ts = self.time_stride
            kv = torch.tensor([max(1, min(T, -(-int(w) // ts))) for w in valid_w], dtype=torch.int32,
                              device=x.device)
        run_blocks(seq, self.tblocks, B, T, self.cfg.heads, "gelu", 1e-6, kv_len=kv)
        return ops.layer_norm(seq, self.ln_w, self.ln_b, 1e-6), B, T


# ============================================================================= synthetic pack
def synthetic_vocab(n: int) -> list[str]:
    """n printable characters: ASCII first, then CJK unified ideographs."""
    chars = [chr(c) for c in range(33, 127)]
    c = 0x4E00
    while len(chars) < n:
        chars.append(chr(c))
        c += 1
    return chars[:n]


def write_ocr_model(root: Path, name: str, preset: Optional[str] = None, seed: int = 0) -> Path:
    from safetensors.torch import save_file

    from ..resources.model_info import ModelInfo

    root = Path(root)
    root.mkdir(parents=True, exist_ok=True)
    preset = preset or ("tiny" if "tiny" in name.lower() else "mobile")
    g = torch.Generator().manual_seed(seed)
    dcfg, rcfg = DBNET_PRESETS[preset], REC_PRESETS[preset]
    det, rec = DBNet(dcfg), SVTRRecognizer(rcfg)
    det.random_init(g)
    rec.random_init(g)
    save_file({k: v.contiguous() for k, v in det.state_dict().items()}, str(root / "detection.safetensors"))
    save_file({k: v.contiguous() for k, v in rec.state_dict().items()}, str(root / "recognition.safetensors"))
    vocab = synthetic_vocab(rcfg.num_classes - 2)     # + space + blank
    (root / "ppocr_keys_v1.txt").write_text("\n".join(vocab) + "\n", encoding="utf-8")
    meta = {"det": asdict(dcfg), "rec": asdict(rcfg), "preset": preset}
    (root / "lumen_ocr_config.json").write_text(json.dumps(meta, indent=2))
    files = ["detection.safetensors", "recognition.safetensors", "lumen_ocr_config.json", "ppocr_keys_v1.txt"]
    info = {
        "name": name, "version": "1.0.0", "description": f"synthetic DBNet + SVTR-LCNet ({preset}) OCR pack",
        "model_type": "ocr", "source": {"format": "custom", "repo_id": f"synthetic/{name}"},
        "runtimes": {"onnx": {"available": True, "files": files, "devices": ["cuda", "cpu"]},
                     "torch": {"available": True, "files": files, "devices": ["cuda", "cpu"]}},
        "extra_metadata": {"synthetic": True,
                           "det_config": {"limit_side_len": 960, "thresh": 0.3, "box_thresh": 0.6,
                                          "unclip_ratio": 1.5},
                           "rec_config": {"image_shape": [3, 48, 320], "character_dict_path": "ppocr_keys_v1.txt",
                                          "use_space_char": True}},
    }
    ModelInfo.model_validate(info)
    (root / "model_info.json").write_text(json.dumps(info, indent=2))
    return root
