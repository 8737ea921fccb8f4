"""CPU reference path of lumen_amd.ops vs independent PyTorch / PIL implementations."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from PIL import Image

from lumen_amd import ops
from lumen_amd.models.clip import CLIPModel


def test_linear_epilogue_order():
    x = torch.randn(10, 64)
    w = torch.randn(32, 64)
    b = torch.randn(32)
    r = torch.randn(10, 32)
    y = ops.linear(x, w, b, act="gelu", residual=r, alpha=0.5)
    ref = F.gelu(0.5 * (x @ w.t()) + b) + r
    assert torch.allclose(y, ref, atol=1e-4)


def test_linear_row_scatter():
    B, P, S = 2, 4, 5
    x = torch.randn(B * P, 64)
    w = torch.randn(16, 64)
    pos = torch.randn(S, 16)
    out = torch.zeros(B * S, 16)
    ops.linear(x, w, table=pos, table_period=P, table_offset=1, out=out, out_group=P, out_group_stride=S,
               out_row_offset=1)
    y = (x @ w.t()).view(B, P, 16) + pos[1:]
    assert torch.allclose(out.view(B, S, 16)[:, 1:], y, atol=1e-5)
    assert out.view(B, S, 16)[:, 0].abs().sum() == 0


def test_norms():
    x = torch.randn(7, 96)
    w, b = torch.randn(96), torch.randn(96)
    assert torch.allclose(ops.layer_norm(x, w, b), F.layer_norm(x, (96,), w, b), atol=1e-5)
    ref = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * w
    assert torch.allclose(ops.rms_norm(x, w), ref, atol=1e-5)
    a = torch.randn(7, 96)
    ro = torch.empty(7, 96)
    y = ops.rms_norm(x, w, add=a, resid_out=ro)
    assert torch.allclose(ro, x + a) and torch.allclose(y, ops.rms_norm(x + a, w), atol=1e-5)


@pytest.mark.parametrize("causal", [False, True])
def test_attention_ref(causal):
    B, S, H, D = 2, 9, 4, 16
    q, k, v = (torch.randn(B, S, H, D) for _ in range(3))
    o = ops.attention(q, k, v, causal=causal)
    ref = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                         is_causal=causal).transpose(1, 2)
    assert torch.allclose(o, ref, atol=1e-5)


def test_attention_gqa_kvlen():
    B, S, H, Hkv, D = 2, 6, 4, 2, 8
    q = torch.randn(B, S, H, D)
    k, v = torch.randn(B, S, Hkv, D), torch.randn(B, S, Hkv, D)
    kl = torch.tensor([6, 3])
    o = ops.attention(q, k, v, kv_len=kl)
    kr, vr = k.repeat_interleave(2, 2), v.repeat_interleave(2, 2)
    mask = torch.arange(S).view(1, 1, 1, S) < kl.view(B, 1, 1, 1)
    ref = F.scaled_dot_product_attention(q.transpose(1, 2), kr.transpose(1, 2), vr.transpose(1, 2),
                                         attn_mask=mask).transpose(1, 2)
    assert torch.allclose(o, ref, atol=1e-5)


@pytest.mark.parametrize("size,resample,name", [((32, 32), Image.BICUBIC, "pil_bicubic"),
                                                ((50, 40), Image.BILINEAR, "pil_bilinear"),
                                                ((224, 224), Image.BICUBIC, "pil_bicubic")])
def test_image_prep_matches_pil(size, resample, name):
    rng = np.random.default_rng(0)
    im = rng.integers(0, 256, (67, 83, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(im).resize(size, resample)).astype(np.float32)
    got = ops.image_prep([torch.from_numpy(im)], (size[1], size[0]), filter=name, scale=1.0, layout="nhwc")[0]
    # PIL uses 8-bit fixed-point coefficients: allow 1 LSB
    assert np.abs(got.numpy() - ref).max() <= 1.0


def test_image_prep_letterbox_and_pad_square():
    im = torch.randint(0, 256, (20, 40, 3), dtype=torch.uint8)
    g = ops.ImageGeom.letterbox(20, 40, 0, 64, 64, 32, 64)
    out = ops.image_prep([im], (64, 64), filter="cv2_linear", scale=1.0, layout="nhwc", geoms=[g])[0]
    assert out[32:].abs().sum() == 0 and out[:32].abs().sum() > 0
    g = ops.ImageGeom.pad_square(20, 40, 0, 40)
    out = ops.image_prep([im], (40, 40), filter="pil_bicubic", scale=1.0, layout="nhwc", geoms=[g])[0]
    assert out[:8].abs().max() < 1 and out[-8:].abs().max() < 1  # black bars top/bottom
    assert torch.allclose(out[10:30], im.float(), atol=1)


def _naive_vision(m, imgs):
    v = m.visual
    cfg = m.cfg.vision
    W, p, s = cfg.width, cfg.patch_size, cfg.image_size
    B = imgs.shape[0]
    pix = np.stack([np.asarray(Image.fromarray(im.numpy()).resize((s, s), Image.BICUBIC)) for im in imgs])
    pix = torch.from_numpy(pix).float() / 255
    pix = ((pix - torch.tensor(m.cfg.image_mean)) / torch.tensor(m.cfg.image_std)).permute(0, 3, 1, 2)
    conv = v.patch_w[:, : v.kdim].float().reshape(W, 3, p, p)
    x = F.conv2d(pix, conv, stride=p).flatten(2).transpose(1, 2)
    x = torch.cat([v.class_emb.float().expand(B, 1, W), x], 1) + v.pos_emb.float()
    x = F.layer_norm(x, (W,), v.ln_pre_w.float(), v.ln_pre_b.float())
    H = cfg.heads
    S = x.shape[1]
    for b in v.blocks:
        h = F.layer_norm(x, (W,), b.ln1_w.float(), b.ln1_b.float())
        qkv = h @ b.qkv_w.float().t() + b.qkv_b.float()
        q, k, vv = qkv.view(B, S, 3, H, W // H).unbind(2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), vv.transpose(1, 2))
        x = x + a.transpose(1, 2).reshape(B, S, W) @ b.out_w.float().t() + b.out_b.float()
        h = F.layer_norm(x, (W,), b.ln2_w.float(), b.ln2_b.float())
        f = h @ b.fc1_w.float().t() + b.fc1_b.float()
        f = f * torch.sigmoid(1.702 * f)
        x = x + f @ b.fc2_w.float().t() + b.fc2_b.float()
    e = F.layer_norm(x[:, 0], (W,), v.ln_post_w.float(), v.ln_post_b.float()) @ v.proj_w.float().t()
    return e / e.norm(dim=-1, keepdim=True)


def test_clip_tiny_matches_naive():
    m = CLIPModel.random("tiny", seed=1, dtype=torch.float32)
    imgs = torch.randint(0, 256, (3, 40, 48, 3), dtype=torch.uint8)
    e = m.encode_image_uint8(imgs)
    ref = _naive_vision(m, imgs)
    assert torch.allclose(e.norm(dim=-1), torch.ones(3), atol=1e-5)
    assert (e * ref).sum(-1).min() > 0.9999


def test_clip_text_eot_pooling_causal():
    m = CLIPModel.random("tiny", seed=2, dtype=torch.float32)
    ids = torch.randint(1, 400, (2, 16))
    ids[:, 6] = 511
    e1 = m.encode_text_ids(ids)
    ids2 = ids.clone()
    ids2[:, 7:] = torch.randint(1, 400, (2, 9))  # tokens after EOT cannot change a causal EOT pool
    e2 = m.encode_text_ids(ids2)
    assert torch.allclose(e1, e2, atol=1e-5)


def test_hf_weight_mapping_roundtrip():
    m = CLIPModel.random("tiny", seed=4, dtype=torch.float32)
    v = m.visual
    cfg = m.cfg
    sd = {
        "vision_model.embeddings.patch_embedding.weight": v.patch_w[:, : v.kdim].reshape(-1, 3, 8, 8).clone(),
        "vision_model.embeddings.class_embedding": v.class_emb.clone(),
        "vision_model.embeddings.position_embedding.weight": v.pos_emb.clone(),
        "vision_model.pre_layrnorm.weight": v.ln_pre_w.clone(), "vision_model.pre_layrnorm.bias": v.ln_pre_b.clone(),
        "vision_model.post_layernorm.weight": v.ln_post_w.clone(),
        "vision_model.post_layernorm.bias": v.ln_post_b.clone(),
        "visual_projection.weight": v.proj_w.clone(),
    }
    for i, b in enumerate(v.blocks):
        p = f"vision_model.encoder.layers.{i}."
        W = cfg.vision.width
        for j, x in enumerate("qkv"):
            sd[p + f"self_attn.{x}_proj.weight"] = b.qkv_w[j * W:(j + 1) * W].clone()
            sd[p + f"self_attn.{x}_proj.bias"] = b.qkv_b[j * W:(j + 1) * W].clone()
        sd[p + "self_attn.out_proj.weight"] = b.out_w.clone(); sd[p + "self_attn.out_proj.bias"] = b.out_b.clone()
        sd[p + "layer_norm1.weight"] = b.ln1_w.clone(); sd[p + "layer_norm1.bias"] = b.ln1_b.clone()
        sd[p + "layer_norm2.weight"] = b.ln2_w.clone(); sd[p + "layer_norm2.bias"] = b.ln2_b.clone()
        sd[p + "mlp.fc1.weight"] = b.fc1_w.clone(); sd[p + "mlp.fc1.bias"] = b.fc1_b.clone()
        sd[p + "mlp.fc2.weight"] = b.fc2_w.clone(); sd[p + "mlp.fc2.bias"] = b.fc2_b.clone()
    m2 = CLIPModel(cfg, dtype=torch.float32, with_text=False)
    m2.load_state_dict_any(sd)
    imgs = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    assert torch.allclose(m.encode_image_uint8(imgs), m2.encode_image_uint8(imgs), atol=1e-6)


@pytest.mark.parametrize("hw", [(67, 83), (120, 90), (50, 50), (31, 97)])
def test_center_crop_matches_open_clip_transform(hw):
    """shortest-side PIL bicubic resize + centre crop (open_clip / torchvision Resize(224) +
    CenterCrop(224), the reference torch runtime, torch_backend.py:201-204,568-576), re-derived
    with PIL: torchvision sizes the long side int(size * long / short) and crops at
    int(round(d / 2))."""
    S = 40
    rng = np.random.default_rng(hw[0])
    im = rng.integers(0, 256, (hw[0], hw[1], 3), dtype=np.uint8)
    h, w = hw
    if w <= h:
        nw, nh = S, int(S * h / w)
    else:
        nh, nw = S, int(S * w / h)
    r = np.asarray(Image.fromarray(im).resize((nw, nh), Image.BICUBIC)).astype(np.float32)
    top, left = int(round((nh - S) / 2.0)), int(round((nw - S) / 2.0))
    ref = r[top:top + S, left:left + S]
    got = ops.image_prep([torch.from_numpy(im)], (S, S), filter="pil_bicubic", scale=1.0, layout="nhwc",
                         center_crop=True)[0]
    assert got.shape == (S, S, 3)
    assert np.abs(got.numpy() - ref).max() <= 1.0                # PIL 8-bit coefficients: 1 LSB


def test_layernorm_folded_into_linear_matches_unfused():
    """ln_row_stats + linear_lnf (LayerNorm folded into the projection, the GPU block form)
    equals layer_norm followed by linear, on rows with a large common offset."""
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(37, 96, generator=g) * 3 + 5).bfloat16()
    gam, bet = torch.rand(96, generator=g) + 0.5, torch.randn(96, generator=g)
    w, b = torch.randn(48, 96, generator=g) * 0.1, torch.randn(48, generator=g)
    ref = ops.linear(ops.layer_norm(x.float(), gam, bet, 1e-5), w, b, act="gelu")
    wf, ca = ops.ln_fold_weights(w, b, gam, bet)
    st = ops.ln_row_stats(x, 1e-5)
    got = ops.linear_lnf(x.float(), wf, ca, st, act="gelu", out=torch.empty(37, 48))
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4)
