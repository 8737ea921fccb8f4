"""FastViT / MobileCLIP MCi towers: the reparameterised NHWC inference path must reproduce
a training-form (multi-branch, un-fused BatchNorm, LayerScale) forward written directly
from the timm ``FastVit`` module structure (fp32, CPU).  Parity against released MobileCLIP2
weights is unpinned (no checkpoints offline); this pins the reparameterisation math and the
block wiring.  The GPU kernels are checked against this CPU path in test_fastvit_gpu.py."""
import math

import pytest
import torch
import torch.nn.functional as F

from lumen_amd.models.fastvit import FASTVIT_PRESETS, FastViTConfig, FastViTTower


def _bn(sd, p, c, g):
    sd[p + ".weight"] = 1.0 + 0.2 * torch.randn(c, generator=g)
    sd[p + ".bias"] = 0.1 * torch.randn(c, generator=g)
    sd[p + ".running_mean"] = 0.1 * torch.randn(c, generator=g)
    sd[p + ".running_var"] = 0.5 + torch.rand(c, generator=g)


def _conv_bn(sd, p, cout, ipg, k, g):
    sd[p + ".conv.weight"] = torch.randn(cout, ipg, k, k, generator=g) * (0.5 / math.sqrt(ipg * k * k))
    _bn(sd, p + ".bn", cout, g)


def _mobileone(sd, p, cin, cout, k, groups, stride, g, scale=True, branches=1, skip_ok=True):
    for i in range(branches):
        _conv_bn(sd, p + f".rbr_conv.{i}", cout, cin // groups, k, g)
    if k > 1 and scale:
        _conv_bn(sd, p + ".rbr_scale", cout, cin // groups, 1, g)
    if skip_ok and cin == cout and stride == 1:
        _bn(sd, p + ".rbr_skip", cout, g)


def _se(sd, p, c, g):
    rd = max(1, int(c * 0.0625))
    sd[p + ".fc1.weight"] = torch.randn(rd, c, 1, 1, generator=g) * c ** -0.5
    sd[p + ".fc1.bias"] = 0.1 * torch.randn(rd, generator=g)
    sd[p + ".fc2.weight"] = torch.randn(c, rd, 1, 1, generator=g) * rd ** -0.5
    sd[p + ".fc2.bias"] = 0.1 * torch.randn(c, generator=g)


def _mlp(sd, p, dim, hid, k, g):
    _conv_bn(sd, p + ".conv", dim, 1, k, g)
    sd[p + ".fc1.weight"] = torch.randn(hid, dim, 1, 1, generator=g) * dim ** -0.5
    sd[p + ".fc1.bias"] = 0.1 * torch.randn(hid, generator=g)
    sd[p + ".fc2.weight"] = torch.randn(dim, hid, 1, 1, generator=g) * hid ** -0.5
    sd[p + ".fc2.bias"] = 0.1 * torch.randn(dim, generator=g)


def training_state_dict(c: FastViTConfig, embed: int, seed: int = 0) -> dict:
    """Random training-form timm FastVit state dict (what an un-reparameterised checkpoint holds)."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    d0 = c.dims[0]
    _mobileone(sd, "stem.0", 3, d0, 3, 1, 2, g, scale=c.stem_scale_branch)
    _mobileone(sd, "stem.1", d0, d0, 3, d0, 2, g, scale=c.stem_scale_branch)
    _mobileone(sd, "stem.2", d0, d0, 1, 1, 1, g)
    prev = d0
    for i, (n, dim) in enumerate(zip(c.layers, c.dims)):
        sp = f"stages.{i}"
        if c.downsamples[i]:
            _conv_bn(sd, sp + ".downsample.proj.0.large_conv", dim, 1, c.down_kernel, g)
            _conv_bn(sd, sp + ".downsample.proj.0.small_conv", dim, 1, 3, g)
            if c.se_downsamples[i]:
                _se(sd, sp + ".downsample.proj.0.se", dim, g)
            _mobileone(sd, sp + ".downsample.proj.1", dim, dim, 1, 1, 1, g)
        if c.pos_embs[i]:
            sd[sp + ".pos_emb.pos_enc.weight"] = 0.1 * torch.randn(dim, 1, c.cpe_kernel, c.cpe_kernel, generator=g)
            sd[sp + ".pos_emb.pos_enc.bias"] = 0.1 * torch.randn(dim, generator=g)
        hid = int(dim * c.mlp_ratios[i])
        for j in range(n):
            bp = f"{sp}.blocks.{j}"
            if c.token_mixers[i] == "repmixer":
                _mobileone(sd, bp + ".token_mixer.norm", dim, dim, c.mixer_kernel, dim, 1, g, scale=False, branches=0)
                _mobileone(sd, bp + ".token_mixer.mixer", dim, dim, c.mixer_kernel, dim, 1, g)
                sd[bp + ".token_mixer.layer_scale.gamma"] = 0.5 + torch.rand(dim, 1, 1, generator=g)
                sd[bp + ".layer_scale.gamma"] = 0.5 + torch.rand(dim, 1, 1, generator=g)
            else:
                if c.attn_norm == "ln":
                    sd[bp + ".norm.weight"] = 1.0 + 0.2 * torch.randn(dim, generator=g)
                    sd[bp + ".norm.bias"] = 0.1 * torch.randn(dim, generator=g)
                else:
                    _bn(sd, bp + ".norm", dim, g)
                sd[bp + ".token_mixer.qkv.weight"] = torch.randn(3 * dim, dim, generator=g) * dim ** -0.5
                sd[bp + ".token_mixer.proj.weight"] = torch.randn(dim, dim, generator=g) * dim ** -0.5
                sd[bp + ".token_mixer.proj.bias"] = 0.1 * torch.randn(dim, generator=g)
                sd[bp + ".layer_scale_1.gamma"] = 0.5 + torch.rand(dim, 1, 1, generator=g)
                sd[bp + ".layer_scale_2.gamma"] = 0.5 + torch.rand(dim, 1, 1, generator=g)
            _mlp(sd, bp + ".mlp", dim, hid, c.mlp_kernel, g)
        prev = dim
    ff = c.final_features
    _mobileone(sd, "final_conv", prev, ff, 3, prev, 1, g)
    _se(sd, "final_conv.se", ff, g)
    sd["head.fc.weight"] = torch.randn(embed, ff, generator=g) * ff ** -0.5
    sd["head.fc.bias"] = 0.1 * torch.randn(embed, generator=g)
    return sd


# ------------------------------------------------------------------ training-form reference forward (NCHW)
def _bn_eval(x, sd, p, eps=1e-5):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, eps)


def _cbn(x, sd, p, stride, groups):
    w = sd[p + ".conv.weight"]
    return _bn_eval(F.conv2d(x, w, None, stride, w.shape[-1] // 2, 1, groups), sd, p + ".bn")


def _ref_se(x, sd, p):
    s = x.mean((2, 3), keepdim=True)
    s = F.relu(F.conv2d(s, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"]))
    return x * torch.sigmoid(F.conv2d(s, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"]))


def _ref_mobileone(x, sd, p, stride, groups, act=True, se=False):
    out = 0
    i = 0
    while p + f".rbr_conv.{i}.conv.weight" in sd:
        out = out + _cbn(x, sd, p + f".rbr_conv.{i}", stride, groups)
        i += 1
    if p + ".rbr_scale.conv.weight" in sd:
        out = out + _cbn(x, sd, p + ".rbr_scale", stride, groups)
    if p + ".rbr_skip.running_mean" in sd:
        out = out + _bn_eval(x, sd, p + ".rbr_skip")
    if se:
        out = _ref_se(out, sd, p + ".se")
    return F.gelu(out) if act else out


def _ref_mlp(x, sd, p):
    y = _cbn(x, sd, p + ".conv", 1, x.shape[1])
    y = F.gelu(F.conv2d(y, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"]))
    return F.conv2d(y, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"])


def ref_forward(sd: dict, c: FastViTConfig, x: torch.Tensor) -> torch.Tensor:
    x = _ref_mobileone(x, sd, "stem.0", 2, 1)
    x = _ref_mobileone(x, sd, "stem.1", 2, x.shape[1])
    x = _ref_mobileone(x, sd, "stem.2", 1, 1)
    for i, (n, dim) in enumerate(zip(c.layers, c.dims)):
        sp = f"stages.{i}"
        if c.downsamples[i]:
            q = sp + ".downsample.proj.0"
            cin = x.shape[1]
            y = _cbn(x, sd, q + ".large_conv", 2, cin) + _cbn(x, sd, q + ".small_conv", 2, cin)
            if c.se_downsamples[i]:
                y = _ref_se(y, sd, q + ".se")
            x = F.gelu(y) if c.lkc_use_act else y
            x = _ref_mobileone(x, sd, sp + ".downsample.proj.1", 1, 1)
        if c.pos_embs[i]:
            w = sd[sp + ".pos_emb.pos_enc.weight"]
            x = x + F.conv2d(x, w, sd[sp + ".pos_emb.pos_enc.bias"], 1, w.shape[-1] // 2, 1, dim)
        for j in range(n):
            bp = f"{sp}.blocks.{j}"
            if c.token_mixers[i] == "repmixer":
                tm = bp + ".token_mixer"
                mix = _ref_mobileone(x, sd, tm + ".mixer", 1, dim, act=False)
                nrm = _ref_mobileone(x, sd, tm + ".norm", 1, dim, act=False)
                x = x + sd[tm + ".layer_scale.gamma"] * (mix - nrm)
                x = x + sd[bp + ".layer_scale.gamma"] * _ref_mlp(x, sd, bp + ".mlp")
            else:
                if c.attn_norm == "ln":
                    y = F.layer_norm(x.permute(0, 2, 3, 1), (dim,), sd[bp + ".norm.weight"], sd[bp + ".norm.bias"],
                                     c.ln_eps).permute(0, 3, 1, 2)
                else:
                    y = _bn_eval(x, sd, bp + ".norm")
                B, C, H, W = y.shape
                t = y.flatten(2).transpose(1, 2)
                heads = C // c.head_dim
                qkv = (t @ sd[bp + ".token_mixer.qkv.weight"].t()).reshape(B, H * W, 3, heads, c.head_dim)
                q, k, v = qkv.permute(2, 0, 3, 1, 4)
                a = torch.softmax((q @ k.transpose(-1, -2)) * c.head_dim ** -0.5, dim=-1) @ v
                a = a.transpose(1, 2).reshape(B, H * W, C)
                a = a @ sd[bp + ".token_mixer.proj.weight"].t() + sd[bp + ".token_mixer.proj.bias"]
                x = x + sd[bp + ".layer_scale_1.gamma"] * a.transpose(1, 2).reshape(B, C, H, W)
                x = x + sd[bp + ".layer_scale_2.gamma"] * _ref_mlp(x, sd, bp + ".mlp")
    x = _ref_mobileone(x, sd, "final_conv", 1, x.shape[1], se=True)
    e = x.mean((2, 3)) @ sd["head.fc.weight"].t() + sd["head.fc.bias"]
    return e / e.norm(dim=-1, keepdim=True)


def _nhwc8(x):
    return F.pad(x.permute(0, 2, 3, 1), (0, 5)).contiguous()


@pytest.mark.parametrize("preset", ["tiny", "tiny-ln"])
def test_reparameterised_matches_training_form(preset):
    c = FASTVIT_PRESETS[preset]
    sd = training_state_dict(c, embed=48, seed=1)
    m = FastViTTower(c, embed_dim=48, dtype=torch.float32)
    m.load_timm({"visual.trunk." + k: v for k, v in sd.items()}, prefix="visual.trunk.")
    x = torch.randn(2, 3, c.image_size, c.image_size, generator=torch.Generator().manual_seed(2))
    ref = ref_forward(sd, c, x)
    got = m.forward_embed(_nhwc8(x))
    assert got.shape == (2, 48)
    assert torch.allclose(got, ref, atol=2e-4), (got - ref).abs().max()


def test_export_roundtrip_and_feature_geometry():
    c = FASTVIT_PRESETS["tiny"]
    a = FastViTTower(c, embed_dim=32, dtype=torch.float32)
    a.random_init(torch.Generator().manual_seed(0))
    b = FastViTTower(c, embed_dim=32, dtype=torch.float32)
    b.load_timm(a.export_timm())
    x = _nhwc8(torch.randn(1, 3, c.image_size, c.image_size))
    assert torch.allclose(a.forward_embed(x), b.forward_embed(x), atol=1e-5)
    f = a.forward_features(x)
    s = c.image_size // c.stride
    assert f.shape == (1, s, s, c.final_features)
    assert FastViTConfig.from_dict(c.to_dict()) == c


def test_presets_geometry():
    assert FASTVIT_PRESETS["mci2"].final_features == 1280 and FASTVIT_PRESETS["mci2"].stride == 32
    hd = FASTVIT_PRESETS["fastvithd"]
    assert hd.final_features == 3072 and (hd.image_size // hd.stride) ** 2 == 256   # FastVLM: 256 image tokens


def test_mobileclip_backend_end_to_end(tmp_path):
    """Synthetic MobileCLIP2 directory (open_clip layout: visual.trunk.* FastViT + text
    transformer) through resources -> CLIP backend; config detection from open_clip_config
    (timm_model_name fastvit_*) alone."""
    import numpy as np

    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.resources.synthetic import write_clip_model
    from lumen_amd.services.clip.backend import MI355XClipBackend
    from lumen_amd.services.clip.resources import ResourceLoader
    from lumen_amd.utils.image import encode_jpeg

    name = "MobileCLIP2-S2-tiny"
    root = write_clip_model(tmp_path / "models" / name, name, dataset="ImageNet_1k", n_labels=10)
    (root / "lumen_clip_config.json").unlink()
    res = ResourceLoader.load_model_resources(tmp_path, ModelConfig(model=name, runtime=Runtime.torch,
                                                                    dataset="ImageNet_1k"))
    cfg = res.clip_config()
    assert cfg.vision_arch == "fastvit" and cfg.fastvit == FASTVIT_PRESETS["tiny"]
    assert tuple(cfg.image_std) == (1.0, 1.0, 1.0)
    be = MI355XClipBackend(res, device="cpu")
    be.initialize()
    try:
        img = encode_jpeg(np.random.default_rng(0).integers(0, 255, (50, 70, 3), dtype=np.uint8))
        v = be.image_to_vector(img)
        assert v.shape == (cfg.embed_dim,) and abs(float(np.linalg.norm(v)) - 1) < 1e-4
        t = be.text_batch_to_vectors(["a photo of a cat", "a dog"])
        assert t.shape == (2, cfg.embed_dim)
    finally:
        be.close()


def test_fastvlm_vision_path_and_pack_roundtrip():
    """FastVLM-style VLM: FastViT conv_exp map rows are the image tokens -> projector."""
    from lumen_amd.models.vlm import VLM, VLM_PRESETS, VLMConfig

    cfg = VLM_PRESETS["tiny-fastvit"]
    assert cfg.num_image_tokens == 16 and cfg.vision_width == cfg.fastvit.final_features
    m = VLM(cfg, dtype=torch.float32, device="cpu")
    m.random_init(0)
    imgs = [torch.randint(0, 256, (40, 70, 3), dtype=torch.uint8), torch.randint(0, 256, (64, 64, 3), dtype=torch.uint8)]
    e = m.encode_images(imgs)
    assert e.shape == (2 * 16, cfg.llm.hidden_size) and torch.isfinite(e).all()
    m2 = VLM(VLMConfig.from_dict(cfg.to_dict()), dtype=torch.float32, device="cpu")
    m2.load_pack_state_dict(m.export_state_dict())
    assert torch.allclose(m2.encode_images(imgs), e, atol=1e-5)
