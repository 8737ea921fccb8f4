"""ONNX graph executor on the MI355X kernels (the counterpart of the reference's ONNX
Runtime sessions for its face / OCR model packs: packages/lumen-face/src/lumen_face/backends/
onnxrt_backend.py, packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py).

``OnnxGraph(path_or_model, device)`` parses the graph with :mod:`lumen_amd.utils.onnx_lite`
(no code from the file runs), then plans it once:

* Conv -> BatchNormalization is folded into the conv weights, and a following
  Relu / LeakyRelu / Sigmoid / HardSwish / Clip(0, 6) / PRelu is fused into the conv
  epilogue, as is a residual ``Add`` of an NHWC tensor of the same shape (ResNet / IResNet);
* conv weights are re-laid out once to the implicit-GEMM ``[Cout, KH, KW, Cin8]`` /
  depthwise ``[KH, KW, C]`` layouts, channel counts padded to the kernels' multiples.

At run time 4-D activations stay NHWC on the GPU (channels padded to a multiple of 8/16
and sliced back only when an NCHW-semantic op needs them).  On the GPU every compute node is
a HIP kernel: Conv (dense incl. asymmetric padding, depthwise, grouped = one dense launch per
group on channel slices), ConvTranspose with kernel == stride (1x1 GEMM + pixel shuffle, BN /
activation folded), pooling, GlobalAveragePool, nearest / bilinear Resize, Concat on channels,
LayerNormalization (and the ReduceMean-Sub-Pow-ReduceMean-Add-Sqrt-Div-Mul-Add subgraph
exporters emit for it), Softmax, activation x activation MatMul (strided batched GEMM),
elementwise unary / broadcast binary ops (csrc/onnx_ops.hip).  Shape arithmetic (Shape,
integer Gather / Concat / Mul, Reshape targets) stays on the host; Reshape / Transpose /
Slice are views or copies.  Unsupported ops are reported when the graph is LOADED.  On the
CPU every node runs the fp32 NCHW reference (the numerics oracle for the GPU path).

Compute nodes that no HIP path covers run on a torch fp32 tier on the GPU (a conv whose
weight is computed, a ConvTranspose with kernel != stride, AveragePool, GlobalMaxPool, a
ReduceMean outside the LayerNorm pattern, unusual Resize modes, ...).  They are never silent:
the load-time scan logs every node that can only take that tier (``fallback_nodes``;
``strict=True`` refuses such a graph), and every execution on it is counted per op type in
``fallback_counts`` with a warning the first time a node takes it.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass
from pathlib import Path
from typing import Optional, Sequence, Union

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..ops import cnn
from ..utils import onnx_lite as ox

log = logging.getLogger("lumen.onnx")

_ACTS = {"Relu": "relu", "Sigmoid": "sigmoid", "HardSwish": "hardswish", "LeakyRelu": "leaky"}

SUPPORTED_OPS = frozenset({
    "Conv", "ConvTranspose", "BatchNormalization", "Relu", "Sigmoid", "Tanh", "Exp", "Log", "Sqrt", "Neg", "Abs",
    "Reciprocal", "Floor", "Ceil", "Erf", "LeakyRelu", "HardSigmoid", "HardSwish", "PRelu", "Clip", "Add", "Sub", "Mul",
    "Div", "Pow", "Max", "Min", "Equal", "Greater", "Less", "MaxPool", "AveragePool", "GlobalAveragePool",
    "GlobalMaxPool", "Resize", "Upsample", "Concat", "Flatten", "Reshape", "Transpose", "Squeeze", "Unsqueeze",
    "Shape", "Gather", "Slice", "Cast", "Softmax", "Gemm", "MatMul", "Constant", "ReduceMean", "ArgMax",
    "Identity", "Dropout", "LayerNormalization"})
_UNARY = {"Relu": 0, "Sigmoid": 1, "Tanh": 2, "Exp": 3, "Log": 4, "Sqrt": 5, "Neg": 6, "Abs": 7, "Reciprocal": 8,
          "HardSwish": 9, "HardSigmoid": 10, "LeakyRelu": 11, "Clip": 12, "Floor": 13, "Ceil": 14, "Erf": 15}
_BINARY = {"Add": 0, "Sub": 1, "Mul": 2, "Div": 3, "Pow": 4, "Max": 5, "Min": 6}
_RESIZE_MODES = {"half_pixel": 0, "align_corners": 1, "asymmetric": 2, "pytorch_half_pixel": 3}
# ops whose generic path is data movement / host shape arithmetic (not a compute fallback)
_DATA_OPS = frozenset({"Flatten", "Reshape", "Transpose", "Squeeze", "Unsqueeze", "Shape", "Gather", "Slice", "Cast",
                       "Constant", "Identity", "Dropout", "Concat", "ArgMax"})
# planned "node" steps of these ops have no HIP path on the GPU (known at load time)
_TORCH_ONLY = frozenset({"Conv", "ConvTranspose", "AveragePool", "GlobalMaxPool", "ReduceMean"})


def _pad_to(c: int, m: int) -> int:
    return (c + m - 1) // m * m


@dataclass
class _V:
    """A value: torch tensor, NHWC-with-padded-channels flag, logical channel count."""
    t: torch.Tensor
    nhwc: bool = False
    c: int = 0

    def nchw(self) -> torch.Tensor:
        if not self.nhwc:
            return self.t
        return self.t[..., : self.c].permute(0, 3, 1, 2)


class OnnxGraph:
    def __init__(self, src: Union[str, Path, bytes, ox.Model], device: Union[str, torch.device] = "cpu",
                 dtype: Optional[torch.dtype] = None, strict: bool = False):
        self.model = src if isinstance(src, ox.Model) else ox.load_model(src)
        g = self.model.graph
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.dtype = dtype or (torch.bfloat16 if self.gpu else torch.float32)
        bad = sorted({n.op_type for n in g.nodes} - SUPPORTED_OPS)
        if bad:     # fail at load time, not on the first request
            raise NotImplementedError(f"ONNX ops not supported by the MI355X graph executor: {', '.join(bad)}")
        self.init = {k: torch.from_numpy(np.array(v)) for k, v in g.initializers.items()}
        self.consumers: dict[str, list] = {}
        for n in g.nodes:
            for x in n.inputs:
                self.consumers.setdefault(x, []).append(n)
        self._dev_init: dict = {}
        self.plan = self._plan(g)
        self.fallback_counts: dict[str, int] = {}
        self._fallback_seen: set = set()
        self.fallback_nodes = self._scan_fallbacks() if self.gpu else []
        if self.fallback_nodes:
            ops_ = sorted({op for op, _ in self.fallback_nodes})
            msg = (f"ONNX graph: {len(self.fallback_nodes)} compute node(s) have no HIP path and run on the "
                   f"torch fp32 tier on {self.device}: {', '.join(ops_)} "
                   f"({', '.join(nm for _, nm in self.fallback_nodes[:8])}{' ...' if len(self.fallback_nodes) > 8 else ''})")
            if strict:
                raise NotImplementedError(msg)
            log.warning(msg)

    def _scan_fallbacks(self) -> list[tuple[str, str]]:
        """(op, node name) of the planned generic steps that can only take the torch tier."""
        out = []
        for kind, step in self.plan:
            if kind == "conv" and step.get("mode") == "ref":
                out.append(("Conv", step.get("name", step["out"])))
            elif kind == "node":
                op, a = step.op_type, step.attrs
                bad = op in _TORCH_ONLY
                if op == "MaxPool":
                    p = a.get("pads", [0, 0, 0, 0])
                    bad = p[:2] != p[2:] or bool(a.get("ceil_mode", 0))
                if op in ("Resize", "Upsample"):
                    mode = a.get("mode", "nearest")
                    bad = mode not in ("nearest", "linear") or (
                        mode == "linear" and a.get("coordinate_transformation_mode", "half_pixel") not in _RESIZE_MODES)
                if bad:
                    out.append((op, step.name or (step.outputs[0] if step.outputs else op)))
        return out

    def _note_fallback(self, n) -> None:
        self.fallback_counts[n.op_type] = self.fallback_counts.get(n.op_type, 0) + 1
        key = id(n)
        if key not in self._fallback_seen:
            self._fallback_seen.add(key)
            log.warning("ONNX node %s (%s) ran on the torch fp32 tier on %s (no HIP path for its inputs)",
                        n.name or n.outputs[0], n.op_type, self.device)

    # ------------------------------------------------------------------ planning
    def _single_consumer(self, name: str, op: str):
        cs = self.consumers.get(name, [])
        if len(cs) == 1 and cs[0].op_type == op and name not in self.model.graph.outputs:
            return cs[0]
        return None

    def _plan(self, g: ox.Graph) -> list:
        plan, skip = [], set()
        for n in g.nodes:
            if id(n) in skip:
                continue
            if n.op_type == "Conv" and n.inputs[1] in self.init:
                step = self._plan_conv(n, skip)
                plan.append(step)
            elif n.op_type == "ConvTranspose" and self.gpu and self._convt_ok(n):
                plan.append(self._plan_convt(n, skip))
            elif n.op_type == "ReduceMean" and self.gpu and (ln := self._match_layernorm(n)) is not None:
                skip.update(ln.pop("nodes"))
                plan.append(("ln", ln))
            else:
                plan.append(("node", n))
        return plan

    # ---- ConvTranspose with kernel == stride (DBNet heads): 1x1 GEMM to f*f*Cout + pixel shuffle
    def _convt_ok(self, n) -> bool:
        a = n.attrs
        if n.inputs[1] not in self.init or int(a.get("group", 1)) != 1:
            return False
        w = self.init[n.inputs[1]]
        k = tuple(a.get("kernel_shape", w.shape[2:]))
        s = tuple(a.get("strides", [1, 1]))
        return (w.dim() == 4 and k[0] == k[1] == s[0] == s[1] and not any(a.get("pads", [0, 0, 0, 0]))
                and not any(a.get("output_padding", [0, 0])) and tuple(a.get("dilations", [1, 1])) == (1, 1))

    def _plan_convt(self, n, skip):
        w = self.init[n.inputs[1]].float()                       # [Cin, Cout, f, f]
        cin, cout, f, _ = w.shape
        b = self.init[n.inputs[2]].float() if len(n.inputs) > 2 and n.inputs[2] else torch.zeros(cout)
        out = n.outputs[0]
        bn = self._single_consumer(out, "BatchNormalization")
        if bn is not None and all(x in self.init for x in bn.inputs[1:5]):
            sc, bi, mu, var = (self.init[x].float() for x in bn.inputs[1:5])
            s = sc / torch.sqrt(var + float(bn.attrs.get("epsilon", 1e-5)))
            w = w * s.view(1, -1, 1, 1)
            b = (b - mu) * s + bi
            skip.add(id(bn))
            out = bn.outputs[0]
        act = None
        nxt = self.consumers.get(out, [])
        if len(nxt) == 1 and out not in self.model.graph.outputs and nxt[0].op_type in ("Relu", "Sigmoid"):
            act = _ACTS[nxt[0].op_type]
            skip.add(id(nxt[0]))
            out = nxt[0].outputs[0]
        cin_p, cout_p = _pad_to(cin, 8), _pad_to(cout, 8)
        while (f * f * cout_p) % 16:
            cout_p += 8
        w1 = torch.zeros(f, f, cout_p, cin_p)                     # rows (dy, dx, co) = pixel-shuffle order
        w1[:, :, :cout, :cin] = w.permute(2, 3, 1, 0)
        b1 = torch.zeros(f, f, cout_p)
        b1[:, :, :cout] = b
        st = {"x": n.inputs[0], "out": out, "f": f, "cin_p": cin_p, "cout": cout, "cout_p": cout_p, "act": act,
              "gw": w1.reshape(f * f * cout_p, 1, 1, cin_p).to(self.device, self.dtype).contiguous(),
              "gb": b1.reshape(-1).to(self.device).contiguous()}
        return ("convt", st)

    # ---- LayerNorm subgraph: m = ReduceMean(x); d = Sub(x, m); v = ReduceMean(Pow(d, 2));
    #      y = Div(d, Sqrt(Add(v, eps))) [* gamma] [+ beta], all over the last axis
    def _match_layernorm(self, rm):
        def one(name, op):
            c = self.consumers.get(name, [])
            return c[0] if len(c) == 1 and c[0].op_type == op else None

        def const(name):
            return float(self.init[name].reshape(-1)[0]) if name in self.init and self.init[name].numel() == 1 else None

        if rm.attrs.get("axes") not in ([-1],) or not rm.attrs.get("keepdims", 1):
            return None
        x = rm.inputs[0]
        subs = [c for c in self.consumers.get(rm.outputs[0], []) if c.op_type == "Sub" and c.inputs[0] == x]
        if len(subs) != 1:
            return None
        sub = subs[0]
        d = sub.outputs[0]
        dc = self.consumers.get(d, [])
        pw = next((c for c in dc if c.op_type == "Pow"), None)
        dv = next((c for c in dc if c.op_type == "Div" and c.inputs[0] == d), None)
        if pw is None or dv is None or len(dc) != 2 or const(pw.inputs[1]) != 2.0:
            return None
        rm2 = one(pw.outputs[0], "ReduceMean")
        if rm2 is None or rm2.attrs.get("axes") not in ([-1],):
            return None
        ad = one(rm2.outputs[0], "Add")
        if ad is None:
            return None
        eps = const(ad.inputs[1] if ad.inputs[0] == rm2.outputs[0] else ad.inputs[0])
        sq = one(ad.outputs[0], "Sqrt")
        if eps is None or sq is None or dv.inputs[1] != sq.outputs[0]:
            return None
        nodes = [rm, sub, pw, rm2, ad, sq, dv]
        out, gamma, beta = dv.outputs[0], None, None
        mul = one(out, "Mul")
        if mul is not None:
            g = mul.inputs[1] if mul.inputs[0] == out else mul.inputs[0]
            if g in self.init:
                gamma, out = g, mul.outputs[0]
                nodes.append(mul)
                add = one(out, "Add")
                if add is not None:
                    bb = add.inputs[1] if add.inputs[0] == out else add.inputs[0]
                    if bb in self.init:
                        beta, out = bb, add.outputs[0]
                        nodes.append(add)
        return {"x": x, "out": out, "eps": eps, "gamma": gamma, "beta": beta, "nodes": {id(q) for q in nodes}}

    def _plan_conv(self, n: ox.Node, skip: set):
        w = self.init[n.inputs[1]].float()
        b = self.init[n.inputs[2]].float() if len(n.inputs) > 2 and n.inputs[2] else torch.zeros(w.shape[0])
        out = n.outputs[0]
        bn = self._single_consumer(out, "BatchNormalization")
        if bn is not None and all(x in self.init for x in bn.inputs[1:5]):
            sc, bi, mu, var = (self.init[x].float() for x in bn.inputs[1:5])
            s = sc / torch.sqrt(var + float(bn.attrs.get("epsilon", 1e-5)))
            w = w * s.view(-1, 1, 1, 1)
            b = (b - mu) * s + bi
            skip.add(id(bn))
            out = bn.outputs[0]
        act, prelu, res = None, None, None
        nxt = self.consumers.get(out, [])
        if len(nxt) == 1 and out not in self.model.graph.outputs:
            a = nxt[0]
            if a.op_type in ("Relu", "Sigmoid", "HardSwish") or \
                    (a.op_type == "LeakyRelu" and abs(float(a.attrs.get("alpha", 0.01)) - 0.1) < 1e-6):
                act = _ACTS[a.op_type]
            elif a.op_type == "Clip" and self._clip_is_relu6(a):
                act = "relu6"
            elif a.op_type == "PRelu" and a.inputs[1] in self.init:
                prelu = self.init[a.inputs[1]].float().reshape(-1)
            elif a.op_type == "Add" and len(a.inputs) == 2:
                other = a.inputs[1] if a.inputs[0] == out else a.inputs[0]
                if other not in self.init:
                    res = other
            if act or prelu is not None or res is not None:
                skip.add(id(a))
                out = a.outputs[0]
        at = n.attrs
        k = tuple(at.get("kernel_shape", w.shape[2:]))
        pads = at.get("pads", [0, 0, 0, 0])
        if at.get("auto_pad", "NOTSET") not in ("NOTSET", "VALID"):
            pads = [k[0] // 2, k[1] // 2, k[0] // 2, k[1] // 2]
        step = {"kind": "conv", "x": n.inputs[0], "out": out, "w": w, "b": b, "groups": int(at.get("group", 1)),
                "stride": tuple(at.get("strides", [1, 1])), "dil": tuple(at.get("dilations", [1, 1])),
                "pads": tuple(pads), "act": act, "prelu": prelu, "res": res}
        if self.gpu:
            self._prep_conv_gpu(step)
        return ("conv", step)

    def _clip_is_relu6(self, a) -> bool:
        lo = a.attrs.get("min")
        hi = a.attrs.get("max")
        if len(a.inputs) >= 3 and a.inputs[1] in self.init and a.inputs[2] in self.init:
            lo, hi = float(self.init[a.inputs[1]]), float(self.init[a.inputs[2]])
        return lo is not None and hi is not None and float(lo) == 0.0 and float(hi) == 6.0

    def _prep_conv_gpu(self, s: dict):
        w, G = s["w"], s["groups"]
        cout, ipg, kh, kw = w.shape
        cin = ipg * G
        dev, dt = self.device, self.dtype
        s["cin"], s["cout"] = cin, cout
        if G == 1:
            cin_p, cout_p = _pad_to(cin, 8), _pad_to(cout, 16)
            wt = torch.zeros(cout_p, kh, kw, cin_p)
            wt[:cout, :, :, :cin] = w.permute(0, 2, 3, 1)
            s["gw"] = wt.to(dev, dt).contiguous()
            bb = torch.zeros(cout_p)
            bb[:cout] = s["b"]
            s["gb"] = bb.to(dev).contiguous()
            if s["prelu"] is not None:
                pp = torch.zeros(cout_p)
                pp[:cout] = s["prelu"] if s["prelu"].numel() > 1 else s["prelu"].expand(cout)
                s["gprelu"] = pp.to(dev, dt).contiguous()
            s["mode"] = "dense"
        elif G == cin and cout % cin == 0 and s["dil"] == (1, 1):
            mult = cout // cin
            cp = _pad_to(cout, 8)
            wt = torch.zeros(kh, kw, cp)
            wt[:, :, :cout] = w.reshape(cout, kh, kw).permute(1, 2, 0)
            s["gw"] = wt.to(dev, dt).contiguous()
            bb = torch.zeros(cp)
            bb[:cout] = s["b"]
            s["gb"] = bb.to(dev).contiguous()
            s["mode"] = "dw"
            s["mult"] = mult
        elif cin % G == 0 and (cin // G) % 8 == 0 and (cout // G) % 16 == 0:
            # grouped: one dense conv per group over channel slices (ipg % 8: 16-byte slice starts)
            ipg, opg = cin // G, cout // G
            s["gws"] = [w[gi * opg:(gi + 1) * opg].permute(0, 2, 3, 1).to(dev, dt).contiguous() for gi in range(G)]
            s["gb"] = s["b"].to(dev).contiguous()
            if s["prelu"] is not None:
                pr = s["prelu"] if s["prelu"].numel() > 1 else s["prelu"].expand(cout)
                s["gprelu"] = pr.to(dev, dt).contiguous()
            s.update(mode="grouped", ipg=ipg, opg=opg, kh=kh, kw=kw)
        else:
            s["mode"] = "ref"     # grouped conv with unaligned group widths: NCHW torch on the device

    # ------------------------------------------------------------------ execution
    @torch.no_grad()
    def run(self, feeds: dict) -> list[torch.Tensor]:
        vals: dict[str, _V] = {}
        for k, v in feeds.items():
            vals[k] = _V(torch.as_tensor(v).to(self.device))
        for kind, step in self.plan:
            if kind == "conv":
                vals[step["out"]] = self._conv(step, vals)
            elif kind == "convt":
                vals[step["out"]] = self._convt(step, vals)
            elif kind == "ln":
                vals[step["out"]] = self._layernorm(vals, step["x"], step["gamma"], step["beta"], step["eps"])
            else:
                for name, v in zip(step.outputs, self._node(step, vals)):
                    vals[name] = v
        outs = []
        for name in self.model.graph.outputs:
            v = vals[name]
            outs.append(v.nchw().contiguous() if v.nhwc else v.t)
        return outs

    def _get(self, vals, name) -> _V:
        if name in vals:
            return vals[name]
        if name in self.init:
            t = self.init[name]
            if not t.is_floating_point():       # shape / index data: host-side
                return _V(t)
            if name not in self._dev_init:
                self._dev_init[name] = t.to(self.device)
            return _V(self._dev_init[name])
        raise KeyError(f"onnx value {name} not computed")

    def _convt(self, s: dict, vals) -> _V:
        x = self._nhwc(self._get(vals, s["x"]), s["cin_p"])
        y = cnn.conv2d(x, s["gw"], s["gb"], 1, 0, 1, act=s["act"])
        return _V(cnn.pixel_shuffle_up(y, s["cout_p"], s["f"]), True, s["cout"])

    def _layernorm(self, vals, x_name, gamma, beta, eps) -> _V:
        v = self._get(vals, x_name)
        x = v.nchw() if v.nhwc else v.t
        D = x.shape[-1]
        g = self._get(vals, gamma).t.to(self.dtype) if gamma else torch.ones(D, device=self.device, dtype=self.dtype)
        b = self._get(vals, beta).t.to(self.dtype) if beta else torch.zeros(D, device=self.device, dtype=self.dtype)
        x2 = x.reshape(-1, D).to(self.dtype).contiguous()
        y = ops.layer_norm(x2, g.reshape(-1).contiguous(), b.reshape(-1).contiguous(), eps)
        return _V(y.reshape(x.shape))

    def _nhwc(self, v: _V, cp: int) -> torch.Tensor:
        """value as a contiguous NHWC tensor with ``cp`` (padded) channels, compute dtype."""
        if v.nhwc and v.t.shape[-1] == cp:
            return v.t
        x = v.nchw() if v.nhwc else v.t
        N, C, H, W = x.shape
        out = torch.zeros((N, H, W, cp), device=self.device, dtype=self.dtype)
        out[..., :C] = x.permute(0, 2, 3, 1).to(self.dtype)
        return out

    def _conv(self, s: dict, vals) -> _V:
        x = self._get(vals, s["x"])
        if self.gpu and s.get("mode") == "ref":
            self.fallback_counts["Conv"] = self.fallback_counts.get("Conv", 0) + 1
        if not self.gpu or s.get("mode") == "ref":
            xt = x.nchw().float() if self.gpu else x.nchw()
            pt, pl, pb, pr = s["pads"][0], s["pads"][1], s["pads"][2], s["pads"][3]
            if (pt, pl) != (pb, pr):
                xt = F.pad(xt, (pl, pr, pt, pb))
                pad = 0
            else:
                pad = (pt, pl)
            w = s["w"].to(xt.device, xt.dtype)
            y = F.conv2d(xt, w, s["b"].to(xt.device, xt.dtype), s["stride"], pad, s["dil"], s["groups"])
            if s["act"] == "relu6":
                y = y.clamp(0, 6)
            elif s["act"]:
                y = ops._act_ref(y, ops.act_id(s["act"]))
            if s["prelu"] is not None:
                p = s["prelu"].to(y.device, y.dtype).view(1, -1, 1, 1)
                y = torch.where(y > 0, y, y * p)
            if s["res"] is not None:
                y = y + self._get(vals, s["res"]).nchw().to(y.dtype)
            return _V(y.to(self.dtype) if self.gpu else y)
        pt, pl, pb, pr = s["pads"]
        pads = (pt, pl, pb, pr)                  # asymmetric: the kernels pad top / left, Ho / Wo do the rest
        act = s["act"]
        relu6 = act == "relu6"
        if s["mode"] == "dense":
            cin_p = s["gw"].shape[-1]
            xt = self._nhwc(x, cin_p)
            res = None
            if s["res"] is not None:
                res = self._nhwc(self._get(vals, s["res"]), s["gw"].shape[0])
            y = cnn.conv2d(xt, s["gw"], s["gb"], s["stride"], pads, s["dil"], act=None if relu6 else act,
                           residual=res, prelu=s.get("gprelu"))
            if relu6:
                y = self._unary(y, 12, 0.0, 6.0)
            return _V(y, True, s["cout"])
        if s["mode"] == "grouped":               # one dense launch per group on channel slices
            G, ipg, opg = s["groups"], s["ipg"], s["opg"]
            xt = self._nhwc(x, s["cin"])
            N, H, W, _ = xt.shape
            Ho, Wo = cnn.conv_out_hw(H, W, s["kh"], s["kw"], s["stride"], pads, s["dil"])
            y = torch.empty((N, Ho, Wo, s["cout"]), device=self.device, dtype=self.dtype)
            res = self._nhwc(self._get(vals, s["res"]), s["cout"]) if s["res"] is not None else None
            for gi in range(G):
                cs, os_ = slice(gi * ipg, (gi + 1) * ipg), slice(gi * opg, (gi + 1) * opg)
                cnn.conv2d(xt[..., cs], s["gws"][gi], s["gb"][os_], s["stride"], pads, s["dil"],
                           act=None if relu6 else act, residual=res[..., os_] if res is not None else None,
                           prelu=s["gprelu"][os_] if s.get("gprelu") is not None else None, out=y[..., os_])
            if relu6:
                y = self._unary(y, 12, 0.0, 6.0)
            return _V(y, True, s["cout"])
        # depthwise (channel multiplier m): duplicate input channels, one dw pass
        cp = s["gw"].shape[-1]
        if s["mult"] > 1:
            xt = self._nhwc(x, _pad_to(s["cin"], 8))[..., : s["cin"]].repeat_interleave(s["mult"], dim=-1)
            if xt.shape[-1] != cp:
                xt = F.pad(xt, (0, cp - xt.shape[-1]))
            xt = xt.contiguous()
        else:
            xt = self._nhwc(x, cp)
        N, H, W, _ = xt.shape
        Ho, Wo = cnn.conv_out_hw(H, W, s["gw"].shape[0], s["gw"].shape[1], s["stride"], pads, s["dil"])
        y = torch.empty((N, Ho, Wo, cp), device=self.device, dtype=self.dtype)
        y = cnn.conv2d_dw(xt, s["gw"], s["gb"], s["stride"], pads, s["dil"], act=None if relu6 else act, out=y)
        if relu6:
            y = self._unary(y, 12, 0.0, 6.0)
        if s["prelu"] is not None:          # per-channel PReLU = max(x,0) + a*min(x,0) via the binary kernel
            p = s["prelu"].to(self.device, torch.float32)
            p = (p if p.numel() > 1 else p.expand(s["cout"])).contiguous()
            pp = torch.zeros(cp, device=self.device)
            pp[: s["cout"]] = p
            neg = self._binary(y, torch.zeros((), device=self.device), 6)        # min(x, 0)
            pos = self._binary(y, torch.zeros((), device=self.device), 5)        # max(x, 0)
            y = self._binary(pos, self._binary(neg, pp, 2, f32=True), 0)
        if s["res"] is not None:
            r = self._nhwc(self._get(vals, s["res"]), cp)
            y = self._binary(y, r, 0)
        return _V(y, True, s["cout"])

    # ---- elementwise HIP kernels (csrc/onnx_ops.hip)
    def _unary(self, x: torch.Tensor, op: int, p0: float = 0.0, p1: float = 0.0) -> torch.Tensor:
        x = x.contiguous()
        out = torch.empty(x.shape, device=self.device, dtype=self.dtype)
        ops.hip_ops().ew_unary(x, out, int(op), float(p0), float(p1))
        return out

    def _binary(self, a: torch.Tensor, b: torch.Tensor, op: int, f32: bool = False) -> torch.Tensor:
        shape = torch.broadcast_shapes(a.shape, b.shape)
        if not a.is_floating_point():
            a = a.float()
        if not b.is_floating_point():
            b = b.float()
        if a.dtype not in (torch.float32, torch.bfloat16):
            a = a.float()
        if b.dtype not in (torch.float32, torch.bfloat16):
            b = b.float()
        out = torch.empty(shape, device=self.device, dtype=torch.float32 if f32 else self.dtype)
        ops.hip_ops().ew_binary(a.to(self.device), b.to(self.device), out, int(op))
        return out

    # ------------------------------------------------------------------ generic nodes
    def _node(self, n: ox.Node, vals) -> list[_V]:
        op, a = n.op_type, n.attrs
        ins = [self._get(vals, x) if x else None for x in n.inputs]
        if self.gpu:
            fast = self._node_nhwc(n, ins)
            if fast is None:
                fast = self._node_gpu(n, ins)
            if fast is not None:
                return fast
        t = [i.nchw() if i is not None else None for i in ins]
        if self.gpu:
            t = [x.float() if x is not None and x.is_floating_point() else x for x in t]
            if op not in _DATA_OPS and any(x is not None and x.is_floating_point() for x in t):
                self._note_fallback(n)

        def out(*ys):
            return [_V(y.to(self.dtype) if self.gpu and y.is_floating_point() else y) for y in ys]

        if op == "Identity" or op == "Dropout":
            return out(t[0])
        if op in ("Relu", "Sigmoid", "Tanh", "Exp", "Log", "Sqrt", "Neg", "Abs", "Reciprocal", "Floor", "Ceil"):
            f = {"Relu": F.relu, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh, "Exp": torch.exp, "Log": torch.log,
                 "Sqrt": torch.sqrt, "Neg": torch.neg, "Abs": torch.abs, "Reciprocal": torch.reciprocal,
                 "Floor": torch.floor, "Ceil": torch.ceil}[op]
            return out(f(t[0]))
        if op == "LeakyRelu":
            return out(F.leaky_relu(t[0], float(a.get("alpha", 0.01))))
        if op == "HardSigmoid":
            return out(torch.clamp(t[0] * float(a.get("alpha", 0.2)) + float(a.get("beta", 0.5)), 0, 1))
        if op == "HardSwish":
            return out(F.hardswish(t[0]))
        if op == "PRelu":
            s = t[1]
            if s.dim() == 1 and t[0].dim() == 4:
                s = s.view(1, -1, 1, 1)
            return out(torch.where(t[0] > 0, t[0], t[0] * s))
        if op == "Clip":
            lo = float(t[1]) if len(t) > 1 and t[1] is not None else a.get("min", None)
            hi = float(t[2]) if len(t) > 2 and t[2] is not None else a.get("max", None)
            return out(torch.clamp(t[0], lo, hi))
        if op in ("Add", "Sub", "Mul", "Div", "Pow", "Max", "Min", "Equal", "Greater", "Less"):
            f = {"Add": torch.add, "Sub": torch.sub, "Mul": torch.mul, "Div": torch.div, "Pow": torch.pow,
                 "Max": torch.maximum, "Min": torch.minimum, "Equal": torch.eq, "Greater": torch.gt,
                 "Less": torch.lt}[op]
            x, y = t[0], t[1]
            if x.is_floating_point() != y.is_floating_point():
                y = y.to(x.dtype) if x.is_floating_point() else y
                x = x.to(y.dtype)
            return out(f(x, y))
        if op == "BatchNormalization":
            sc, bi, mu, var = (x.view(1, -1, 1, 1) if t[0].dim() == 4 else x for x in t[1:5])
            return out((t[0] - mu) / torch.sqrt(var + float(a.get("epsilon", 1e-5))) * sc + bi)
        if op == "Conv":   # conv with a computed (non-initializer) weight
            p = a.get("pads", [0, 0, 0, 0])
            return out(F.conv2d(t[0], t[1], t[2] if len(t) > 2 else None, tuple(a.get("strides", [1, 1])),
                                (p[0], p[1]), tuple(a.get("dilations", [1, 1])), int(a.get("group", 1))))
        if op == "ConvTranspose":
            p = a.get("pads", [0, 0, 0, 0])
            return out(F.conv_transpose2d(t[0], t[1], t[2] if len(t) > 2 else None, tuple(a.get("strides", [1, 1])),
                                          (p[0], p[1]), tuple(a.get("output_padding", [0, 0])),
                                          int(a.get("group", 1))))
        if op in ("MaxPool", "AveragePool"):
            k = tuple(a["kernel_shape"])
            p = a.get("pads", [0, 0, 0, 0])
            s = tuple(a.get("strides", k))
            x = t[0]
            if (p[0], p[1]) != (p[2], p[3]):
                x = F.pad(x, (p[1], p[3], p[0], p[2]), value=-math.inf if op == "MaxPool" else 0.0)
                pp = (0, 0)
            else:
                pp = (p[0], p[1])
            if op == "MaxPool":
                return out(F.max_pool2d(x, k, s, pp, ceil_mode=bool(a.get("ceil_mode", 0))))
            return out(F.avg_pool2d(x, k, s, pp, ceil_mode=bool(a.get("ceil_mode", 0)),
                                    count_include_pad=bool(a.get("count_include_pad", 0))))
        if op == "GlobalAveragePool":
            return out(t[0].mean(dim=(2, 3), keepdim=True))
        if op == "GlobalMaxPool":
            return out(t[0].amax(dim=(2, 3), keepdim=True))
        if op in ("Resize", "Upsample"):
            return out(self._resize(n, t))
        if op == "Concat":
            return out(torch.cat([x for x in t], dim=int(a.get("axis", 1))))
        if op == "Flatten":
            ax = int(a.get("axis", 1))
            x = t[0]
            return out(x.reshape(int(np.prod(x.shape[:ax])) if ax else 1, -1))
        if op == "Reshape":
            shape = [int(s) for s in t[1].tolist()]
            shape = [t[0].shape[i] if s == 0 and not a.get("allowzero", 0) else s for i, s in enumerate(shape)]
            return out(t[0].reshape(shape))
        if op == "Transpose":
            perm = a.get("perm", list(range(t[0].dim()))[::-1])
            return out(t[0].permute(*perm).contiguous())
        if op == "Squeeze":
            axes = a.get("axes") if "axes" in a else (t[1].tolist() if len(t) > 1 and t[1] is not None else None)
            x = t[0]
            if axes is None:
                return out(x.squeeze())
            for ax in sorted((int(q) % x.dim() for q in axes), reverse=True):
                x = x.squeeze(ax)
            return out(x)
        if op == "Unsqueeze":
            axes = a.get("axes") if "axes" in a else t[1].tolist()
            x = t[0]
            for ax in sorted(int(q) for q in axes):
                x = x.unsqueeze(ax if ax >= 0 else x.dim() + 1 + ax)
            return out(x)
        if op == "Shape":        # host-side: shape arithmetic never launches device kernels
            return out(torch.tensor(list(t[0].shape), dtype=torch.int64))
        if op == "Gather":
            ax = int(a.get("axis", 0))
            idx = t[1].long()
            r = torch.index_select(t[0], ax, idx.reshape(-1)).reshape(
                *t[0].shape[:ax], *idx.shape, *t[0].shape[ax + 1:])
            return out(r)
        if op == "Slice":
            x = t[0]
            starts, ends = t[1].tolist(), t[2].tolist()
            axes = t[3].tolist() if len(t) > 3 and t[3] is not None else list(range(len(starts)))
            steps = t[4].tolist() if len(t) > 4 and t[4] is not None else [1] * len(starts)
            sl = [slice(None)] * x.dim()
            for s0, e0, ax, st in zip(starts, ends, axes, steps):
                dimn = x.shape[ax]
                s0 = max(0, min(dimn, s0 + dimn if s0 < 0 else s0))
                e0 = max(0, min(dimn, e0 + dimn if e0 < 0 else e0))
                sl[ax] = slice(s0, e0, st)
            return out(x[tuple(sl)])
        if op == "Cast":
            to = ox.DTYPES.get(int(a["to"]), np.float32)
            return out(t[0].to(torch.from_numpy(np.zeros(0, to)).dtype))
        if op == "Softmax":
            return out(torch.softmax(t[0], dim=int(a.get("axis", -1))))
        if op in ("Gemm", "MatMul"):
            return out(self._matmul(n, t))
        if op == "Constant":
            c = torch.as_tensor(np.array(a["value"]))
            return out(c.to(self.device) if c.is_floating_point() else c)
        if op == "ReduceMean":
            axes = a.get("axes", None)
            return out(t[0].mean(dim=tuple(axes), keepdim=bool(a.get("keepdims", 1))) if axes else t[0].mean())
        if op == "LayerNormalization":
            ax = int(a.get("axis", -1)) % t[0].dim()
            shape = t[0].shape[ax:]
            w = t[1] if len(t) > 1 and t[1] is not None else None
            b = t[2] if len(t) > 2 and t[2] is not None else None
            return out(F.layer_norm(t[0], shape, w.reshape(shape) if w is not None else None,
                                    b.reshape(shape) if b is not None else None, float(a.get("epsilon", 1e-5))))
        if op == "Erf":
            return out(torch.erf(t[0]))
        if op == "ArgMax":
            return out(t[0].argmax(dim=int(a.get("axis", 0)), keepdim=bool(a.get("keepdims", 1))))
        raise NotImplementedError(f"ONNX op {op} is not supported by the MI355X graph executor")

    def _node_gpu(self, n: ox.Node, ins) -> Optional[list]:
        """HIP kernels for the NCHW-semantic compute nodes; None -> the generic path (host-side
        shape arithmetic, views / copies)."""
        op, a = n.op_type, n.attrs
        t = [i.nchw() if i is not None else None for i in ins]
        fp = [x is not None and x.is_floating_point() for x in t]
        if op in _UNARY and t and fp[0]:
            p0, p1 = 0.0, 0.0
            if op == "HardSigmoid":
                p0, p1 = float(a.get("alpha", 0.2)), float(a.get("beta", 0.5))
            elif op == "LeakyRelu":
                p0 = float(a.get("alpha", 0.01))
            elif op == "Clip":
                lo = float(t[1]) if len(t) > 1 and t[1] is not None else a.get("min", None)
                hi = float(t[2]) if len(t) > 2 and t[2] is not None else a.get("max", None)
                p0 = float(lo) if lo is not None else -math.inf
                p1 = float(hi) if hi is not None else math.inf
            return [_V(self._unary(t[0], _UNARY[op], p0, p1))]
        if op in _BINARY and len(t) == 2 and (fp[0] or fp[1]):
            return [_V(self._binary(t[0], t[1], _BINARY[op]))]
        if op == "PRelu" and fp[0]:
            sl = t[1]
            if sl.dim() == 1 and t[0].dim() == 4:
                sl = sl.view(1, -1, 1, 1)
            z = torch.zeros((), device=self.device)
            return [_V(self._binary(self._binary(t[0], z, 5), self._binary(self._binary(t[0], z, 6), sl, 2), 0))]
        if op == "BatchNormalization" and fp[0]:
            sc, bi, mu, var = (x.float() for x in t[1:5])
            scale = sc / torch.sqrt(var + float(a.get("epsilon", 1e-5)))
            shift = bi - mu * scale
            if t[0].dim() == 4:
                scale, shift = scale.view(1, -1, 1, 1), shift.view(1, -1, 1, 1)
            return [_V(self._binary(self._binary(t[0], scale, 2, f32=True), shift, 0))]
        if op == "Softmax" and fp[0]:
            x = t[0]
            ax = int(a.get("axis", -1)) % x.dim()
            xm = x.movedim(ax, -1).contiguous()
            y = torch.empty(xm.shape, device=self.device, dtype=self.dtype)
            ops.hip_ops().softmax_rows(xm, y)
            return [_V(y.movedim(-1, ax))]
        if op == "LayerNormalization" and fp[0] and int(a.get("axis", -1)) in (-1, t[0].dim() - 1):
            return [self._layernorm({n.inputs[0]: ins[0]}, n.inputs[0], n.inputs[1] if len(n.inputs) > 1 else None,
                                    n.inputs[2] if len(n.inputs) > 2 else None, float(a.get("epsilon", 1e-5)))]
        if op == "MatMul" and fp[0] and fp[1] and not (n.inputs[1] in self.init and t[1].dim() == 2):
            x, w = t[0], t[1]
            if x.dim() >= 2 and w.dim() >= 2:
                lead = torch.broadcast_shapes(x.shape[:-2], w.shape[:-2])
                M, K, N = x.shape[-2], x.shape[-1], w.shape[-1]
                xb = x.expand(*lead, M, K).reshape(-1, M, K)
                wb = w.expand(*lead, K, N).reshape(-1, K, N)
                y = torch.empty((xb.shape[0], M, N), device=self.device, dtype=torch.float32)
                ops.hip_ops().bmm(xb, wb, y)
                return [_V(y.reshape(*lead, M, N).to(self.dtype))]
        if op in ("Resize", "Upsample") and fp[0] and t[0].dim() == 4 and a.get("mode", "nearest") == "linear":
            x = ins[0]
            cp = _pad_to(x.c if x.nhwc else t[0].shape[1], 8)
            xt = self._nhwc(x, cp)
            N, H, W, _ = xt.shape
            scales = sizes = None
            if op == "Upsample":
                scales = t[1].tolist()
            else:
                if len(t) > 2 and t[2] is not None and t[2].numel():
                    scales = t[2].tolist()
                if len(t) > 3 and t[3] is not None and t[3].numel():
                    sizes = [int(q) for q in t[3].tolist()]
            Ho, Wo = (sizes[2], sizes[3]) if sizes else (int(H * scales[2]), int(W * scales[3]))
            mode = _RESIZE_MODES.get(a.get("coordinate_transformation_mode", "half_pixel"))
            if mode is None:
                return None
            y = torch.empty((N, Ho, Wo, cp), device=self.device, dtype=self.dtype)
            ops.hip_ops().resize_bilinear_nhwc(xt.contiguous(), y, int(mode))
            return [_V(y, True, x.c if x.nhwc else t[0].shape[1])]
        return None

    def _resize(self, n, t):
        a = n.attrs
        x = t[0]
        scales = None
        sizes = None
        if n.op_type == "Upsample":
            scales = t[1].tolist()
        else:
            if len(t) > 2 and t[2] is not None and t[2].numel():
                scales = t[2].tolist()
            if len(t) > 3 and t[3] is not None and t[3].numel():
                sizes = [int(s) for s in t[3].tolist()]
        mode = a.get("mode", "nearest")
        size = tuple(sizes[2:]) if sizes else (int(x.shape[2] * scales[2]), int(x.shape[3] * scales[3]))
        if mode == "nearest":
            return F.interpolate(x, size=size, mode="nearest")
        align = a.get("coordinate_transformation_mode", "half_pixel") == "align_corners"
        return F.interpolate(x, size=size, mode="bilinear", align_corners=align)

    def _matmul(self, n, t):
        a = n.attrs
        x, w = t[0], t[1]
        if n.op_type == "Gemm":
            if a.get("transA", 0):
                x = x.t()
            w_nk = w if a.get("transB", 0) else w.t()      # -> [N, K]
            alpha, beta = float(a.get("alpha", 1.0)), float(a.get("beta", 1.0))
            bias = t[2] * beta if len(t) > 2 and t[2] is not None else None
        else:
            if w.dim() != 2:
                return torch.matmul(x, w)
            w_nk, alpha, bias = w.t(), 1.0, None
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        K, N = x2.shape[1], w_nk.shape[0]
        if self.gpu and K % 64 == 0 and N % 16 == 0:
            y = ops.linear(x2.to(self.dtype).contiguous(), w_nk.to(self.dtype).contiguous(),
                           bias.float().contiguous() if bias is not None else None, alpha=alpha,
                           out_dtype=torch.float32)
        else:
            y = (x2.float() @ w_nk.float().t()) * alpha
            if bias is not None:
                y = y + bias.float()
        return y.reshape(*lead, N)

    def _node_nhwc(self, n: ox.Node, ins) -> Optional[list]:
        """HIP-kernel fast paths for NHWC activations; None -> generic NCHW fallback."""
        op, a = n.op_type, n.attrs
        x = ins[0] if ins else None
        if x is None or not x.nhwc:
            return None
        if op == "GlobalAveragePool":
            y = cnn.global_avgpool(x.t)[:, : x.c]
            return [_V(y.to(self.dtype).view(y.shape[0], x.c, 1, 1))]
        if op == "MaxPool" and a.get("pads", [0, 0, 0, 0])[:2] == a.get("pads", [0, 0, 0, 0])[2:] \
                and not a.get("ceil_mode", 0):
            k = tuple(a["kernel_shape"])
            p = a.get("pads", [0, 0, 0, 0])
            return [_V(cnn.pool2d(x.t, k, tuple(a.get("strides", k)), (p[0], p[1]), True), True, x.c)]
        if op in ("Relu", "Sigmoid", "HardSwish"):
            c = x.t.shape[-1]
            y = cnn.channel_affine(x.t, torch.ones(c, device=self.device), torch.zeros(c, device=self.device),
                                   act=_ACTS[op])
            return [_V(y, True, x.c)]
        if op == "Concat" and int(a.get("axis", 1)) == 1 and all(i is not None and i.nhwc and i.t.dim() == 4
                                                                  for i in ins):
            parts = [i.t[..., : i.c] for i in ins]
            y = torch.cat(parts, dim=-1)
            c = y.shape[-1]
            if c % 8:
                y = F.pad(y, (0, _pad_to(c, 8) - c))
            return [_V(y.contiguous(), True, c)]
        if op in ("Resize", "Upsample"):
            mode = a.get("mode", "nearest")
            sc = None
            if op == "Upsample" and ins[1] is not None:
                sc = ins[1].t.tolist()
            elif len(ins) > 2 and ins[2] is not None and ins[2].t.numel():
                sc = ins[2].t.tolist()
            if mode == "nearest" and sc and float(sc[2]) == float(sc[3]) and float(sc[2]).is_integer() and \
                    float(sc[0]) == 1.0:
                return [_V(cnn.upsample_add(x.t, None, int(sc[2])), True, x.c)]
            return None
        if op == "Add" and len(ins) == 2 and ins[1] is not None and ins[1].nhwc and \
                ins[0].t.shape == ins[1].t.shape:
            return [_V((ins[0].t.float() + ins[1].t.float()).to(self.dtype), True, x.c)]
        return None


def load_graph(path, device="cpu") -> OnnxGraph:
    return OnnxGraph(path, device)
