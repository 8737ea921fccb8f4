"""Face models on the CPU reference path.

* IResNet: an insightface-layout PyTorch NCHW iresnet (written here from the
  published architecture) with random weights + random BN statistics is loaded
  through ``IResNet.load_insightface_state_dict``; embeddings must match.
* SCRFD: shapes of the fused head maps, synthetic model pack round trip.
"""
import json

import torch
import torch.nn.functional as F
from torch import nn

from lumen_amd.models.face import IRESNET_PRESETS, SCRFD, SCRFD_PRESETS, IResNet, write_face_model


class _RefBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.prelu = nn.PReLU(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, stride, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.downsample = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
                           if stride != 1 or cin != cout else None)

    def forward(self, x):
        idt = self.downsample(x) if self.downsample is not None else x
        h = self.bn3(self.conv2(self.prelu(self.bn2(self.conv1(self.bn1(x))))))
        return h + idt


class _RefIResNet(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        w0 = cfg.widths[0]
        self.conv1 = nn.Conv2d(3, w0, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(w0)
        self.prelu = nn.PReLU(w0)
        cin = w0
        for li, (n, w) in enumerate(zip(cfg.layers, cfg.widths)):
            blocks = []
            for i in range(n):
                blocks.append(_RefBlock(cin, w, 2 if i == 0 else 1))
                cin = w
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self.nlayers = len(cfg.layers)
        self.bn2 = nn.BatchNorm2d(cin)
        hw = cfg.input_size // 16
        self.fc = nn.Linear(cin * hw * hw, cfg.embedding)
        self.features = nn.BatchNorm1d(cfg.embedding)

    def forward(self, x):
        h = self.prelu(self.bn1(self.conv1(x)))
        for li in range(self.nlayers):
            h = getattr(self, f"layer{li + 1}")(h)
        h = self.bn2(h).flatten(1)
        return self.features(self.fc(h))


def _randomise(m, g):
    for mod in m.modules():
        if isinstance(mod, (nn.BatchNorm2d, nn.BatchNorm1d)):
            mod.weight.data = 1 + 0.1 * torch.randn(mod.weight.shape, generator=g)
            mod.bias.data = 0.1 * torch.randn(mod.bias.shape, generator=g)
            mod.running_mean.data = 0.1 * torch.randn(mod.running_mean.shape, generator=g)
            mod.running_var.data = 1 + 0.2 * torch.rand(mod.running_var.shape, generator=g)
        elif isinstance(mod, nn.PReLU):
            mod.weight.data = 0.25 + 0.05 * torch.randn(mod.weight.shape, generator=g)


def test_iresnet_matches_insightface_layout():
    g = torch.Generator().manual_seed(0)
    cfg = IRESNET_PRESETS["tiny"]
    ref = _RefIResNet(cfg)
    _randomise(ref, g)
    ref.eval()
    ours = IResNet(cfg)
    ours.load_insightface_state_dict(ref.state_dict())
    x = torch.randn(3, 3, 112, 112, generator=g)
    want = F.normalize(ref(x).float(), dim=-1)
    xn = F.pad(x.permute(0, 2, 3, 1), (0, 5))  # NHWC8
    got = ours(xn)
    cos = (got * want).sum(-1)
    assert got.shape == (3, cfg.embedding)
    assert cos.min() > 0.99, cos


def test_scrfd_heads_and_pack(tmp_path):
    cfg = SCRFD_PRESETS["tiny"]
    det = SCRFD(cfg)
    det.random_init(torch.Generator().manual_seed(1))
    outs = det(torch.randn(1, cfg.input_size, cfg.input_size, 8))
    assert [o.shape[1] for o in outs] == [cfg.input_size // s for s in cfg.strides]
    assert all(o.shape[-1] >= cfg.anchors * 15 and o.dtype == torch.float32 for o in outs)
    root = write_face_model(tmp_path / "buffalo_tiny", "buffalo_tiny")
    info = json.loads((root / "model_info.json").read_text())
    assert info["model_type"] == "face" and (root / "detection.safetensors").exists()
