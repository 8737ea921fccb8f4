"""FastViT-family image towers on NHWC HIP kernels: the MobileCLIP / MobileCLIP2 "MCi"
image encoders (MobileCLIP2-S0/S2 = MCi0/MCi2, S3/S4 = MCi3/MCi4) and FastVLM's FastViTHD.

Reference behaviour: the reference runs these towers inside exported ONNX graphs / the
timm ``fastvit_mci*`` trunk of open_clip (lumen-clip ``MobileCLIP2-S2`` / ``-S4``,
packages/lumen-clip/README.md:117-125; FastVLM ``vision_encoder.onnx``,
packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py).  Here the network runs in
its *reparameterised* inference form, which is what makes it cheap on the GPU:

* every multi-branch MobileOne block (k x k conv+BN branches, 1x1 scale branch, BN
  identity branch) is one conv with bias,
* a RepMixer block (``x + g * (mixer(x) - norm(x))``) is ONE depthwise conv with the
  identity folded into its centre tap, RepCPE likewise,
* BatchNorms after convs fold into the conv, the BatchNorm before attention folds
  into the QKV projection, LayerScale gammas fold into the projection / fc2 weights,
* so a block is: depthwise conv (mixer) -> depthwise 7x7 -> 1x1 conv + GELU (implicit
  GEMM on MFMA) -> 1x1 conv with the residual add in the epilogue; an attention block
  runs the flash-attention kernel directly on the NHWC activation (NHWC rows ARE the
  token rows: no flatten/transposes).

Grouped convs with channel multiplier 2 (PatchEmbed's 7x7 stride-2 ``ReparamLargeKernelConv``,
the final 3x3 ``conv_exp``) run as a depthwise conv over the channel-duplicated input.
:func:`reparameterize` turns training-form timm / ml-fastvlm state dicts (``rbr_conv``,
``rbr_scale``, ``rbr_skip``, ``large_conv``/``small_conv``, ``mixer``/``norm``,
``pos_enc``) into fused tensors; already-reparameterised checkpoints (``reparam_conv``)
load directly.  Architecture tables follow timm's fastvit_mci0..4; the MCi3/MCi4 and
FastViTHD tables are not pinned against released weights here (no checkpoints offline).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops
from ..ops import cnn
from .layers import ConvBN, Linear


@dataclass
class FastViTConfig:
    layers: tuple = (4, 12, 24, 4)
    dims: tuple = (80, 160, 320, 640)
    mlp_ratios: tuple = (3.0, 3.0, 3.0, 3.0)
    downsamples: tuple = (False, True, True, True)
    se_downsamples: tuple = (False, False, True, True)
    pos_embs: tuple = (False, False, False, True)
    token_mixers: tuple = ("repmixer", "repmixer", "repmixer", "attention")
    attn_norm: str = "bn"            # "bn" (MCi0-2) | "ln" (LayerNorm over channels: MCi3/4, FastViTHD)
    stem_scale_branch: bool = True
    lkc_use_act: bool = True
    cls_ratio: float = 2.0
    head_dim: int = 32
    image_size: int = 256
    mixer_kernel: int = 3
    down_kernel: int = 7
    cpe_kernel: int = 7
    mlp_kernel: int = 7
    bn_eps: float = 1e-5
    ln_eps: float = 1e-5
    final_se: bool = True
    image_mean: tuple = (0.0, 0.0, 0.0)
    image_std: tuple = (1.0, 1.0, 1.0)

    @property
    def final_features(self) -> int:
        return int(self.dims[-1] * self.cls_ratio)

    @property
    def stride(self) -> int:
        return 4 * 2 ** sum(1 for d in self.downsamples if d)

    def to_dict(self) -> dict:
        return asdict(self)

    @staticmethod
    def from_dict(d: dict) -> "FastViTConfig":
        kw = {k: (tuple(v) if isinstance(v, list) else v) for k, v in d.items() if k in FastViTConfig.__dataclass_fields__}
        return FastViTConfig(**kw)


def _mci(layers, dims, mlp=3.0, se=(False, False, True, True), **kw):
    n = len(layers)
    return FastViTConfig(layers=tuple(layers), dims=tuple(dims), mlp_ratios=(mlp,) * n,
                         downsamples=(False,) + (True,) * (n - 1), se_downsamples=tuple(se),
                         pos_embs=kw.pop("pos_embs", (False,) * (n - 1) + (True,)),
                         token_mixers=kw.pop("token_mixers", ("repmixer",) * (n - 1) + ("attention",)), **kw)


_FIVE = dict(mlp=4.0, se=(False,) * 5, pos_embs=(False, False, False, True, True),
             token_mixers=("repmixer", "repmixer", "repmixer", "attention", "attention"), attn_norm="ln",
             stem_scale_branch=False)

FASTVIT_PRESETS = {
    "mci0": _mci((2, 6, 10, 2), (64, 128, 256, 512)),
    "mci1": _mci((4, 12, 20, 4), (64, 128, 256, 512)),
    "mci2": _mci((4, 12, 24, 4), (80, 160, 320, 640)),
    "mci3": _mci((2, 12, 24, 4, 2), (96, 192, 384, 768, 1536), **_FIVE),
    "mci4": _mci((2, 12, 24, 4, 2), (128, 256, 512, 1024, 2048), **_FIVE),
    # FastVLM vision tower: FastViTHD, 1024 px -> 16 x 16 x 3072 (conv_exp) features
    "fastvithd": _mci((2, 12, 24, 4, 2), (96, 192, 384, 768, 1536), image_size=1024, **_FIVE),
    # CPU-test geometry: every block type, both attention norms exercised across presets
    "tiny": _mci((1, 1, 1), (32, 64, 64), mlp=2.0, se=(False, True, False), image_size=64,
                 pos_embs=(False, True, True), token_mixers=("repmixer", "repmixer", "attention")),
    "tiny-ln": _mci((1, 1, 1), (32, 64, 64), mlp=2.0, se=(False, False, True), image_size=64, attn_norm="ln",
                    stem_scale_branch=False, pos_embs=(False, False, True),
                    token_mixers=("repmixer", "attention", "attention")),
}


# ----------------------------------------------------------------------------------------------
# reparameterisation (training-form timm / ml-fastvlm names -> fused conv weights)
# ----------------------------------------------------------------------------------------------
def _bn_fuse(w: torch.Tensor, sd: dict, p: str, eps: float):
    """conv weight [O, I/g, k, k] + BN ``p.*`` -> fused (w, b)."""
    g = sd[p + ".weight"].float()
    beta = sd[p + ".bias"].float()
    std = torch.sqrt(sd[p + ".running_var"].float() + eps)
    t = g / std
    return w.float() * t.view(-1, 1, 1, 1), beta - sd[p + ".running_mean"].float() * t


def _identity_kernel(c: int, in_per_group: int, k: int) -> torch.Tensor:
    w = torch.zeros(c, in_per_group, k, k)
    for i in range(c):
        w[i, i % in_per_group, k // 2, k // 2] = 1.0
    return w


def _pad_to(w: torch.Tensor, k: int) -> torch.Tensor:
    p = (k - w.shape[-1]) // 2
    return F.pad(w, (p, p, p, p)) if p > 0 else w


def mobileone_fused(sd: dict, p: str, k: int, cin: int, cout: int, groups: int, eps: float):
    """MobileOneBlock ``p`` -> (w [cout, cin/g, k, k], b [cout])."""
    if p + ".reparam_conv.weight" in sd:
        w = sd[p + ".reparam_conv.weight"].float()
        b = sd.get(p + ".reparam_conv.bias")
        return w, (b.float() if b is not None else torch.zeros(cout))
    ipg = cin // groups
    w = torch.zeros(cout, ipg, k, k)
    b = torch.zeros(cout)
    i = 0
    while p + f".rbr_conv.{i}.conv.weight" in sd:
        wi, bi = _bn_fuse(sd[p + f".rbr_conv.{i}.conv.weight"], sd, p + f".rbr_conv.{i}.bn", eps)
        w, b = w + wi, b + bi
        i += 1
    if p + ".rbr_scale.conv.weight" in sd:
        ws, bs = _bn_fuse(sd[p + ".rbr_scale.conv.weight"], sd, p + ".rbr_scale.bn", eps)
        w, b = w + _pad_to(ws, k), b + bs
    if p + ".rbr_skip.running_mean" in sd:
        wi, bi = _bn_fuse(_identity_kernel(cout, ipg, k), sd, p + ".rbr_skip", eps)
        w, b = w + wi, b + bi
    return w, b


def large_kernel_fused(sd: dict, p: str, k: int, cout: int, eps: float):
    """ReparamLargeKernelConv ``p`` (large k x k + small 3 x 3 branch) -> (w, b)."""
    if p + ".reparam_conv.weight" in sd:
        return sd[p + ".reparam_conv.weight"].float(), sd[p + ".reparam_conv.bias"].float()
    w, b = _bn_fuse(sd[p + ".large_conv.conv.weight"], sd, p + ".large_conv.bn", eps)
    if p + ".small_conv.conv.weight" in sd:
        ws, bs = _bn_fuse(sd[p + ".small_conv.conv.weight"], sd, p + ".small_conv.bn", eps)
        w, b = w + _pad_to(ws, k), b + bs
    return w, b


def repmixer_fused(sd: dict, p: str, dim: int, k: int, eps: float):
    """RepMixer ``p``: x + gamma * (mixer(x) - norm(x)) -> one depthwise conv (w, b)."""
    if p + ".reparam_conv.weight" in sd:
        return sd[p + ".reparam_conv.weight"].float(), sd[p + ".reparam_conv.bias"].float()
    wm, bm = mobileone_fused(sd, p + ".mixer", k, dim, dim, dim, eps)
    wn, bn = mobileone_fused(sd, p + ".norm", k, dim, dim, dim, eps)
    gamma = sd[p + ".layer_scale.gamma"].float().reshape(-1) if p + ".layer_scale.gamma" in sd \
        else sd[p + ".layer_scale"].float().reshape(-1)
    w = _identity_kernel(dim, 1, k) + gamma.view(-1, 1, 1, 1) * (wm - wn)
    return w, gamma * (bm - bn)


def cpe_fused(sd: dict, p: str, dim: int, k: int):
    """RepConditionalPosEnc ``p``: x + dwconv(x) -> one depthwise conv."""
    if p + ".reparam_conv.weight" in sd:
        return sd[p + ".reparam_conv.weight"].float(), sd[p + ".reparam_conv.bias"].float()
    w = sd[p + ".pos_enc.weight"].float()
    return w + _identity_kernel(dim, w.shape[1], k), sd[p + ".pos_enc.bias"].float()


def _gamma(sd: dict, p: str) -> torch.Tensor:
    for key in (p + ".gamma", p):
        if key in sd:
            return sd[key].float().reshape(-1)
    raise KeyError(p)


# ----------------------------------------------------------------------------------------------
# inference modules (NHWC)
# ----------------------------------------------------------------------------------------------
class DWConv(nn.Module):
    """Depthwise (channel multiplier ``mult``) k x k conv with bias (+act), NHWC."""

    def __init__(self, cin: int, k: int, stride: int = 1, mult: int = 1, act=None, dtype=torch.bfloat16):
        super().__init__()
        self.cin, self.k, self.stride, self.mult, self.act = cin, k, stride, mult, act
        self.w = nn.Parameter(torch.zeros(k, k, cin * mult, dtype=dtype), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(cin * mult, dtype=torch.float32), requires_grad=False)

    def load(self, w: torch.Tensor, b: torch.Tensor):
        """w: torch grouped layout [cin*mult, 1, k, k] (groups = cin)."""
        self.w.data.copy_(w.float().reshape(self.cin * self.mult, self.k, self.k).permute(1, 2, 0).to(self.w.dtype))
        self.b.data.copy_(b.float())

    def export(self):
        return self.w.float().permute(2, 0, 1).unsqueeze(1).contiguous(), self.b.float().clone()

    def forward(self, x, act=None):
        if self.mult > 1:   # grouped conv, groups = cin: output channel o reads input o // mult
            x = x.repeat_interleave(self.mult, dim=-1)
        return cnn.conv2d_dw(x, self.w, self.b, self.stride, self.k // 2, 1, act=act if act is not None else self.act)


class SE(nn.Module):
    """Squeeze-excite (timm SqueezeExcite: mean -> 1x1 reduce + ReLU -> 1x1 expand -> sigmoid)."""

    def __init__(self, c: int, rd: int, dtype=torch.bfloat16):
        super().__init__()
        self.fc1 = Linear(c, rd, act="relu", dtype=dtype)
        self.fc2 = Linear(rd, c, act="sigmoid", dtype=dtype)

    def forward(self, x):
        s = cnn.global_avgpool(x).to(self.fc1.w.dtype)
        s = self.fc2(self.fc1(s), out_dtype=torch.float32)
        return cnn.channel_scale_(x, s)


def _gelu_(x: torch.Tensor, ones: torch.Tensor, zeros: torch.Tensor) -> torch.Tensor:
    return cnn.channel_affine(x, ones, zeros, act="gelu", out=x)


class _Mlp(nn.Module):
    """ConvMlp: depthwise 7x7 (+BN) -> 1x1 + GELU -> 1x1 (x gamma) -> + residual."""

    def __init__(self, dim: int, hidden: int, k: int, dtype):
        super().__init__()
        self.dw = DWConv(dim, k, dtype=dtype)
        self.fc1 = ConvBN(dim, hidden, 1, act="gelu", dtype=dtype)
        self.fc2 = ConvBN(hidden, dim, 1, dtype=dtype)

    def forward(self, x):
        return self.fc2(self.fc1(self.dw(x)), residual=x, out=x)


class _Attention(nn.Module):
    def __init__(self, dim: int, head_dim: int, norm: str, mlp_hidden: int, k: int, eps: float, dtype):
        super().__init__()
        self.dim, self.heads, self.norm, self.eps = dim, dim // head_dim, norm, eps
        self.ln_w = nn.Parameter(torch.ones(dim, dtype=dtype), requires_grad=False) if norm == "ln" else None
        self.ln_b = nn.Parameter(torch.zeros(dim, dtype=dtype), requires_grad=False) if norm == "ln" else None
        self.qkv_w = nn.Parameter(torch.zeros(3 * dim, dim, dtype=dtype), requires_grad=False)
        self.qkv_b = nn.Parameter(torch.zeros(3 * dim, dtype=torch.float32), requires_grad=False)
        self.proj_w = nn.Parameter(torch.zeros(dim, dim, dtype=dtype), requires_grad=False)
        self.proj_b = nn.Parameter(torch.zeros(dim, dtype=torch.float32), requires_grad=False)
        self.mlp = _Mlp(dim, mlp_hidden, k, dtype)

    def forward(self, x):
        N, H, W, C = x.shape
        T = N * H * W
        t = x.view(T, C)                      # NHWC rows are the attention tokens
        h = ops.layer_norm(t, self.ln_w, self.ln_b, self.eps) if self.norm == "ln" else t
        qkv = ops.linear(h, self.qkv_w, self.qkv_b).view(N, H * W, 3, self.heads, C // self.heads)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
        ops.linear(o.view(T, C), self.proj_w, self.proj_b, residual=t, out=t)
        return self.mlp(x)


class _RepMixerBlock(nn.Module):
    def __init__(self, dim: int, k: int, mlp_hidden: int, mk: int, dtype):
        super().__init__()
        self.mixer = DWConv(dim, k, dtype=dtype)
        self.mlp = _Mlp(dim, mlp_hidden, mk, dtype)

    def forward(self, x):
        return self.mlp(self.mixer(x))


class FastViTTower(nn.Module):
    """Reparameterised FastViT trunk + (optional) pooled linear head, NHWC bf16."""

    def __init__(self, cfg: FastViTConfig, embed_dim: Optional[int] = None, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.embed_dim = embed_dim
        d0 = cfg.dims[0]
        self.stem0 = ConvBN(3, d0, 3, stride=2, act="gelu", dtype=dtype)
        self.stem1 = DWConv(d0, 3, stride=2, act="gelu", dtype=dtype)
        self.stem2 = ConvBN(d0, d0, 1, act="gelu", dtype=dtype)
        self.stages = nn.ModuleList()
        prev = d0
        for i, (n, dim) in enumerate(zip(cfg.layers, cfg.dims)):
            st = nn.Module()
            st.down = None
            if cfg.downsamples[i]:
                st.down = nn.Module()
                st.down.lk = DWConv(prev, cfg.down_kernel, stride=2, mult=dim // prev, dtype=dtype)
                st.down.se = SE(dim, max(1, int(dim * 0.0625)), dtype) if cfg.se_downsamples[i] else None
                st.down.pw = ConvBN(dim, dim, 1, act="gelu", dtype=dtype)
            st.cpe = DWConv(dim, cfg.cpe_kernel, dtype=dtype) if cfg.pos_embs[i] else None
            hid = int(dim * cfg.mlp_ratios[i])
            st.blocks = nn.ModuleList([
                _Attention(dim, cfg.head_dim, cfg.attn_norm, hid, cfg.mlp_kernel, cfg.ln_eps, dtype)
                if cfg.token_mixers[i] == "attention" else _RepMixerBlock(dim, cfg.mixer_kernel, hid, cfg.mlp_kernel, dtype)
                for _ in range(n)])
            self.stages.append(st)
            prev = dim
        ff = cfg.final_features
        self.final = DWConv(prev, 3, mult=ff // prev, dtype=dtype)
        self.final_se = SE(ff, max(1, int(ff * 0.0625)), dtype) if cfg.final_se else None
        self.head = Linear(ff, embed_dim, dtype=dtype) if embed_dim else None
        self.register_buffer("_ones", torch.ones(max(ff, max(cfg.dims))), persistent=False)
        self.register_buffer("_zeros", torch.zeros(max(ff, max(cfg.dims))), persistent=False)
        if device is not None:
            self.to(device)

    # ---------------------------------------------------------------- forward
    def _act(self, x):
        c = x.shape[-1]
        return _gelu_(x, self._ones[:c], self._zeros[:c])

    @torch.no_grad()
    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        """NHWC8 normalised image [N, S, S, 8] -> conv_exp feature map [N, S/stride, S/stride, final]."""
        x = self.stem2(self.stem1(self.stem0(x)))
        for st in self.stages:
            if st.down is not None:
                d = st.down
                x = d.lk(x, act=None if d.se is not None or not self.cfg.lkc_use_act else "gelu")
                if d.se is not None:
                    d.se(x)
                    if self.cfg.lkc_use_act:
                        self._act(x)
                x = d.pw(x)
            if st.cpe is not None:
                x = st.cpe(x)
            for blk in st.blocks:
                x = blk(x)
        x = self.final(x, act=None if self.final_se is not None else "gelu")
        if self.final_se is not None:
            self.final_se(x)
            self._act(x)
        return x

    @torch.no_grad()
    def forward_embed(self, x: torch.Tensor) -> torch.Tensor:
        """-> L2-normalised fp32 [N, embed_dim] (global average pool + linear head)."""
        f = self.forward_features(x)
        pooled = cnn.global_avgpool(f).to(self.head.w.dtype)
        emb = self.head(pooled, out_dtype=torch.float32)
        return ops.l2_normalize_(emb.contiguous())

    def preprocess(self, images, mean, std, filter: str = "pil_bicubic", center_crop: bool = False) -> torch.Tensor:
        s = self.cfg.image_size
        return ops.image_prep(images, (s, s), mean=mean, std=std, filter=filter, layout="nhwc8",
                              out_dtype=self.stem0.w.dtype, device=self.stem0.w.device, center_crop=center_crop)

    # ---------------------------------------------------------------- weights
    def load_timm(self, sd: dict, prefix: str = "") -> None:
        """timm ``FastVit`` / ml-fastvlm ``mci`` state dict (training or reparameterised form)."""
        c, e = self.cfg, self.cfg.bn_eps
        P = prefix
        d0 = c.dims[0]
        w, b = mobileone_fused(sd, P + "stem.0", 3, 3, d0, 1, e)
        self.stem0.load_torch(w, b)
        w, b = mobileone_fused(sd, P + "stem.1", 3, d0, d0, d0, e)
        self.stem1.load(w, b)
        w, b = mobileone_fused(sd, P + "stem.2", 1, d0, d0, 1, e)
        self.stem2.load_torch(w, b)
        prev = d0
        for i, st in enumerate(self.stages):
            dim = c.dims[i]
            sp = f"{P}stages.{i}"
            if st.down is not None:
                w, b = large_kernel_fused(sd, sp + ".downsample.proj.0", c.down_kernel, dim, e)
                st.down.lk.load(w, b)
                if st.down.se is not None:
                    _load_se(st.down.se, sd, sp + ".downsample.proj.0.se")
                w, b = mobileone_fused(sd, sp + ".downsample.proj.1", 1, dim, dim, 1, e)
                st.down.pw.load_torch(w, b)
            if st.cpe is not None:
                w, b = cpe_fused(sd, sp + ".pos_emb", dim, c.cpe_kernel)
                st.cpe.load(w, b)
            for j, blk in enumerate(st.blocks):
                bp = f"{sp}.blocks.{j}"
                if isinstance(blk, _RepMixerBlock):
                    w, b = repmixer_fused(sd, bp + ".token_mixer", dim, c.mixer_kernel, e)
                    blk.mixer.load(w, b)
                    _load_mlp(blk.mlp, sd, bp + ".mlp", _gamma(sd, bp + ".layer_scale"), e)
                else:
                    _load_attn(blk, sd, bp, e)
            prev = dim
        w, b = mobileone_fused(sd, P + "final_conv", 3, prev, c.final_features, prev, e)
        self.final.load(w, b)
        if self.final_se is not None:
            _load_se(self.final_se, sd, P + "final_conv.se")
        if self.head is not None:
            self.head.load_torch(sd[P + "head.fc.weight"], sd.get(P + "head.fc.bias"))

    def export_timm(self, prefix: str = "") -> dict:
        """Reparameterised timm naming (``reparam_conv``; ConvMlp conv + identity BN)."""
        c, P = self.cfg, prefix
        sd = {}

        def conv(p, m: ConvBN):
            sd[p + ".reparam_conv.weight"] = m.w[: m.cout, :, :, : m.cin].float().permute(0, 3, 1, 2).contiguous()
            sd[p + ".reparam_conv.bias"] = m.b[: m.cout].float().clone()

        def dw(p, m: DWConv):
            sd[p + ".weight"], sd[p + ".bias"] = m.export()

        def se(p, m: SE):
            sd[p + ".fc1.weight"] = m.fc1.w[: m.fc1.cout, : m.fc1.cin].float().reshape(m.fc1.cout, m.fc1.cin, 1, 1)
            sd[p + ".fc1.bias"] = m.fc1.b[: m.fc1.cout].float().clone()
            sd[p + ".fc2.weight"] = m.fc2.w[: m.fc2.cout, : m.fc2.cin].float().reshape(m.fc2.cout, m.fc2.cin, 1, 1)
            sd[p + ".fc2.bias"] = m.fc2.b[: m.fc2.cout].float().clone()

        def mlp(p, m: _Mlp, dim):
            w, b = m.dw.export()
            sd[p + ".conv.conv.weight"] = w
            sd[p + ".conv.bn.weight"], sd[p + ".conv.bn.bias"] = torch.ones(dim), b
            sd[p + ".conv.bn.running_mean"] = torch.zeros(dim)
            sd[p + ".conv.bn.running_var"] = torch.full((dim,), 1.0 - c.bn_eps)
            for n, f in (("fc1", m.fc1), ("fc2", m.fc2)):
                sd[p + f".{n}.weight"] = f.w[: f.cout, :, :, : f.cin].float().permute(0, 3, 1, 2).contiguous()
                sd[p + f".{n}.bias"] = f.b[: f.cout].float().clone()

        conv(P + "stem.0", self.stem0)
        dw(P + "stem.1.reparam_conv", self.stem1)
        conv(P + "stem.2", self.stem2)
        for i, st in enumerate(self.stages):
            dim, sp = c.dims[i], f"{P}stages.{i}"
            if st.down is not None:
                dw(sp + ".downsample.proj.0.reparam_conv", st.down.lk)
                if st.down.se is not None:
                    se(sp + ".downsample.proj.0.se", st.down.se)
                conv(sp + ".downsample.proj.1", st.down.pw)
            if st.cpe is not None:
                dw(sp + ".pos_emb.reparam_conv", st.cpe)
            for j, blk in enumerate(st.blocks):
                bp = f"{sp}.blocks.{j}"
                if isinstance(blk, _RepMixerBlock):
                    dw(bp + ".token_mixer.reparam_conv", blk.mixer)
                    mlp(bp + ".mlp", blk.mlp, dim)
                    sd[bp + ".layer_scale.gamma"] = torch.ones(dim, 1, 1)
                else:
                    if blk.norm == "ln":
                        sd[bp + ".norm.weight"], sd[bp + ".norm.bias"] = blk.ln_w.float().clone(), blk.ln_b.float().clone()
                    else:
                        sd[bp + ".norm.weight"], sd[bp + ".norm.bias"] = torch.ones(dim), torch.zeros(dim)
                        sd[bp + ".norm.running_mean"] = torch.zeros(dim)
                        sd[bp + ".norm.running_var"] = torch.full((dim,), 1.0 - c.bn_eps)
                    sd[bp + ".token_mixer.qkv.weight"] = blk.qkv_w.float().clone()
                    sd[bp + ".token_mixer.qkv.bias"] = blk.qkv_b.float().clone()
                    sd[bp + ".token_mixer.proj.weight"] = blk.proj_w.float().clone()
                    sd[bp + ".token_mixer.proj.bias"] = blk.proj_b.float().clone()
                    sd[bp + ".layer_scale_1.gamma"] = torch.ones(dim, 1, 1)
                    sd[bp + ".layer_scale_2.gamma"] = torch.ones(dim, 1, 1)
                    mlp(bp + ".mlp", blk.mlp, dim)
        dw(P + "final_conv.reparam_conv", self.final)
        if self.final_se is not None:
            se(P + "final_conv.se", self.final_se)
        if self.head is not None:
            sd[P + "head.fc.weight"] = self.head.w[: self.head.cout, : self.head.cin].float().clone()
            sd[P + "head.fc.bias"] = self.head.b[: self.head.cout].float().clone()
        return {k: v.detach().contiguous().cpu() for k, v in sd.items()}

    def random_init(self, g: torch.Generator) -> None:
        """Random weights of the right scale (synthetic model directories, tests)."""
        for m in self.modules():
            if isinstance(m, ConvBN):
                m.random_init(g, gain=0.5)
            elif isinstance(m, DWConv):
                w = torch.randn(m.k, m.k, m.cin * m.mult, generator=g) * (0.5 / m.k)
                w[m.k // 2, m.k // 2] += 1.0          # near-identity: keeps activations O(1) through deep stacks
                m.w.data.copy_(w.to(m.w.dtype))
                m.b.data.copy_(torch.randn(m.b.shape, generator=g) * 0.01)
            elif isinstance(m, Linear):
                m.random_init(g)
            elif isinstance(m, _Attention):
                d = m.dim
                m.qkv_w.data.copy_((torch.randn(3 * d, d, generator=g) * d ** -0.5).to(m.qkv_w.dtype))
                m.proj_w.data.copy_((torch.randn(d, d, generator=g) * 0.1 * d ** -0.5).to(m.proj_w.dtype))
        for st in self.stages:
            for blk in st.blocks:
                blk.mlp.fc2.w.data.mul_(0.1)         # small residual branches (LayerScale-like)


def _load_se(m: SE, sd: dict, p: str) -> None:
    m.fc1.load_torch(sd[p + ".fc1.weight"].reshape(m.fc1.cout, m.fc1.cin), sd[p + ".fc1.bias"])
    m.fc2.load_torch(sd[p + ".fc2.weight"].reshape(m.fc2.cout, m.fc2.cin), sd[p + ".fc2.bias"])


def _load_mlp(m: _Mlp, sd: dict, p: str, gamma: torch.Tensor, eps: float) -> None:
    w, b = _bn_fuse(sd[p + ".conv.conv.weight"], sd, p + ".conv.bn", eps)
    m.dw.load(w, b)
    m.fc1.load_torch(sd[p + ".fc1.weight"], sd[p + ".fc1.bias"])
    m.fc2.load_torch(sd[p + ".fc2.weight"].float() * gamma.view(-1, 1, 1, 1), sd[p + ".fc2.bias"].float() * gamma)


def _load_attn(blk: _Attention, sd: dict, bp: str, eps: float) -> None:
    qkv_w = sd[bp + ".token_mixer.qkv.weight"].float()
    qkv_b = sd.get(bp + ".token_mixer.qkv.bias")
    qkv_b = qkv_b.float() if qkv_b is not None else torch.zeros(qkv_w.shape[0])
    if blk.norm == "ln":
        blk.ln_w.data.copy_(sd[bp + ".norm.weight"].float().reshape(-1).to(blk.ln_w.dtype))
        blk.ln_b.data.copy_(sd[bp + ".norm.bias"].float().reshape(-1).to(blk.ln_b.dtype))
    else:   # BatchNorm before attention: fold y = s*x + t into the QKV projection
        s = sd[bp + ".norm.weight"].float() / torch.sqrt(sd[bp + ".norm.running_var"].float() + eps)
        t = sd[bp + ".norm.bias"].float() - sd[bp + ".norm.running_mean"].float() * s
        qkv_b = qkv_b + qkv_w @ t
        qkv_w = qkv_w * s.view(1, -1)
    blk.qkv_w.data.copy_(qkv_w.to(blk.qkv_w.dtype))
    blk.qkv_b.data.copy_(qkv_b)
    g1 = _gamma(sd, bp + ".layer_scale_1")
    blk.proj_w.data.copy_((sd[bp + ".token_mixer.proj.weight"].float() * g1.view(-1, 1)).to(blk.proj_w.dtype))
    blk.proj_b.data.copy_(sd[bp + ".token_mixer.proj.bias"].float() * g1)
    _load_mlp(blk.mlp, sd, bp + ".mlp", _gamma(sd, bp + ".layer_scale_2"), eps)
