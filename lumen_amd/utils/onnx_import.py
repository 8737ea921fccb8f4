"""Import the weights of exported ONNX graphs onto the native MI355X models.

The reference's default runtime is ONNX Runtime over per-component graphs:
CLIP ``onnx/vision[.fp16].onnx`` + ``onnx/text[.fp16].onnx``
(packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:140-289) and FastVLM
``onnx/vision|embed|decoder[.fp16].onnx`` (packages/lumen-vlm/src/lumen_vlm/backends/
onnxrt_backend.py:55-160, 538-659).  Here those graphs are not executed: their
initializers are read (utils/onnx_lite.py, nothing in the file runs) and mapped back to
the parameter names of the PyTorch module they were exported from, then loaded into the
native CLIP / LLM / FastViTHD models (the same kernels as the safetensors path).

``torch.onnx.export`` keeps parameter names for tensors used as-is (conv weights,
embeddings, norms, biases) but constant-folds the transpose of every ``nn.Linear``
weight feeding a ``MatMul`` into a generated ``onnx::MatMul_<n>`` initializer.  Those
names are recovered, in order of reliability, from:

1. the bias the product feeds: ``MatMul(x, W^T) -> Add(b, .)`` with ``b`` named
   ``<module>.bias`` (``in_proj_bias`` -> ``in_proj_weight``) gives ``<module>.weight``;
2. the node's scope name: ``/model/layers.0/self_attn/o_proj/MatMul`` ->
   ``model.layers.0.self_attn.o_proj.weight``;
3. for a graph's single remaining un-named projection, the caller's fallback (CLIP
   ``visual.proj`` / ``text_projection``).
``Gemm`` weights honour ``transB``; fp16 graphs are widened to fp32 (the models cast to
their compute dtype on load).

Quantised packs (the reference selects ``vision.{precision}.onnx`` for precision ``int8`` /
``q4fp16``, packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:245-289) are
dequantised first (:func:`dequantize_model`): ``DequantizeLinear`` of an initializer (QDQ,
per-tensor or per-axis), ``MatMulInteger`` with an int8 / uint8 weight and its
``<w>_scale`` / ``<w>_zero_point`` initializers (dynamic quantisation), and ``MatMulNBits``
(com.microsoft, 4-bit blockwise, fp16 / fp32 scales, optional packed zero points) become
plain float ``MatMul`` operands under the original weight name, so the name recovery above
applies unchanged.  The native models then run the dequantised weights in their own compute
dtype (bf16 / fp8 on the GPU) -- the int8 / 4-bit ONNX runtime kernels are not emulated.
"""
from __future__ import annotations

import logging
import re
from pathlib import Path
from typing import Optional, Sequence, Union

import numpy as np

from . import onnx_lite

log = logging.getLogger("lumen.onnx_import")

# exporter-made names: "onnx::MatMul_123", "/scope/Constant_output_0", "val_12", "_v_3", "1234"
_GENERATED = re.compile(r"^(onnx::|/)|::|^(val|_v|initializer)_\d+$|^[\d_]+$")


def _is_generated(name: str) -> bool:
    return bool(_GENERATED.search(name))


def _scope_to_param(node_name: str, suffix: str = "weight") -> Optional[str]:
    """``/model/layers.0/self_attn/q_proj/MatMul`` -> ``model.layers.0.self_attn.q_proj.weight``."""
    parts = [p for p in node_name.split("/") if p]
    if len(parts) < 2:
        return None
    mods = parts[:-1]
    out: list[str] = []
    for p in mods:                       # scopes repeat the parent list name: "mm_projector/mm_projector.0"
        if out and p.startswith(out[-1] + "."):
            out[-1] = p
        else:
            out.append(p)
    return ".".join(out) + "." + suffix


# ---------------------------------------------------------------------------- quantised packs
def _strip(name: str, suffixes: Sequence[str]) -> str:
    for suf in suffixes:
        if name.endswith(suf):
            return name[: -len(suf)]
    return name


def dequantize_linear(q: np.ndarray, scale: np.ndarray, zp: Optional[np.ndarray], axis: int = 1) -> np.ndarray:
    """ONNX DequantizeLinear: (q - zero_point) * scale, per tensor or along ``axis``."""
    x = q.astype(np.float32)
    sc = np.asarray(scale, np.float32)
    z = np.zeros_like(sc) if zp is None else np.asarray(zp).astype(np.float32)
    if sc.ndim == 1 and sc.size > 1:
        shape = [1] * x.ndim
        shape[axis % x.ndim] = sc.size
        sc, z = sc.reshape(shape), z.reshape(shape)
    return (x - z) * sc


def dequantize_nbits(b: np.ndarray, scales: np.ndarray, zero_points: Optional[np.ndarray], K: int, N: int,
                     bits: int = 4, block_size: int = 32) -> np.ndarray:
    """com.microsoft MatMulNBits weight -> float [N, K] (the nn.Linear layout).  ``b``: uint8
    [N, n_blocks, block_size * bits / 8], values packed low nibble first; ``scales`` [N * n_blocks];
    ``zero_points``: uint8 packed like b (or float, one per block), default 2^(bits-1)."""
    if bits != 4:
        raise ValueError(f"MatMulNBits with {bits} bits is not supported (4-bit packs only)")
    nb = -(-K // block_size)
    raw = np.asarray(b, np.uint8).reshape(N, nb, block_size // 2)
    q = np.empty((N, nb, block_size), np.float32)
    q[..., 0::2] = raw & 0x0F
    q[..., 1::2] = raw >> 4
    sc = np.asarray(scales).astype(np.float32).reshape(N, nb)
    if zero_points is None:
        zp = np.full((N, nb), 8.0, np.float32)
    elif np.asarray(zero_points).dtype == np.uint8:
        zr = np.asarray(zero_points, np.uint8).reshape(N, -1)
        zz = np.empty((N, zr.shape[1] * 2), np.float32)
        zz[:, 0::2] = zr & 0x0F
        zz[:, 1::2] = zr >> 4
        zp = zz[:, :nb]
    else:
        zp = np.asarray(zero_points).astype(np.float32).reshape(N, nb)
    w = (q - zp[..., None]) * sc[..., None]
    return w.reshape(N, nb * block_size)[:, :K]


def dequantize_model(m: onnx_lite.Model) -> onnx_lite.Model:
    """Replace quantised weight patterns by float initializers + plain MatMul (see module doc)."""
    g = m.graph
    inits = dict(g.initializers)
    rename: dict[str, str] = {}
    nodes: list = []
    spent: set = set()          # quantised tensors folded into a float initializer
    for n in g.nodes:
        op = n.op_type
        if op == "DequantizeLinear" and n.inputs and n.inputs[0] in inits:
            q = inits[n.inputs[0]]
            sc = inits[n.inputs[1]]
            zp = inits.get(n.inputs[2]) if len(n.inputs) > 2 and n.inputs[2] else None
            base = _strip(n.inputs[0], ("_quantized", "_q", "_int8"))
            name = base if base != n.inputs[0] else n.outputs[0]
            inits[name] = dequantize_linear(q, sc, zp, int(n.attrs.get("axis", 1)))
            rename[n.outputs[0]] = name
            spent.update(x for x in n.inputs if x)
            continue
        if op == "MatMulInteger" and len(n.inputs) > 1 and n.inputs[1] in inits:
            wq = n.inputs[1]
            base = _strip(wq, ("_quantized", "_q", "_int8"))
            sc = inits.get(base + "_scale")
            if sc is None:
                raise ValueError(f"MatMulInteger {n.name or n.outputs[0]}: no {base}_scale initializer")
            zp = inits.get(n.inputs[3]) if len(n.inputs) > 3 and n.inputs[3] else inits.get(base + "_zero_point")
            inits[base] = dequantize_linear(inits[wq], sc, zp, 1)      # B [K, N]: per-column scales
            spent.update({wq, base + "_scale", base + "_zero_point"} | ({n.inputs[3]} if len(n.inputs) > 3 else set()))
            nodes.append(onnx_lite.Node("MatMul", [n.inputs[0], base], list(n.outputs), name=n.name))
            continue
        if op == "MatMulNBits" and len(n.inputs) > 2 and n.inputs[1] in inits:
            a = n.attrs
            K, N = int(a["K"]), int(a["N"])
            zp = inits.get(n.inputs[3]) if len(n.inputs) > 3 and n.inputs[3] else None
            w = dequantize_nbits(inits[n.inputs[1]], inits[n.inputs[2]], zp, K, N, int(a.get("bits", 4)),
                                 int(a.get("block_size", 32)))
            base = _strip(n.inputs[1], ("_Q4", "_Q8", "_q4", "_quantized"))
            inits[base] = w.T                                            # MatMul B operand [K, N]
            spent.update(x for x in n.inputs[1:4] if x)
            out = n.outputs[0]
            if len(n.inputs) > 5 and n.inputs[5]:                        # fused bias input
                nodes.append(onnx_lite.Node("MatMul", [n.inputs[0], base], [out + "__mm"], name=n.name))
                nodes.append(onnx_lite.Node("Add", [n.inputs[5], out + "__mm"], [out], name=n.name + "_bias"))
            else:
                nodes.append(onnx_lite.Node("MatMul", [n.inputs[0], base], [out], name=n.name))
            continue
        nodes.append(n)
    if not spent:
        return m
    for n in nodes:
        n.inputs = [rename.get(x, x) for x in n.inputs]
    used = {x for n in nodes for x in n.inputs}
    keep = {k: v for k, v in inits.items() if k in used or k not in spent}
    g2 = onnx_lite.Graph(nodes=nodes, initializers=keep, inputs=list(g.inputs),
                         outputs=[rename.get(x, x) for x in g.outputs], name=g.name)
    return onnx_lite.Model(graph=g2, opset=m.opset, ir_version=m.ir_version)


def recover_state_dict(src: Union[str, Path, bytes, onnx_lite.Model]) -> tuple[dict, list]:
    """(name -> np.float32 array in PyTorch layout, [unresolved (node, array)]) of one graph
    (quantised weights are dequantised first, :func:`dequantize_model`)."""
    m = src if isinstance(src, onnx_lite.Model) else onnx_lite.load_model(src)
    m = dequantize_model(m)
    g = m.graph
    inits = g.initializers
    consumers: dict[str, list] = {}
    for n in g.nodes:
        for i, x in enumerate(n.inputs):
            consumers.setdefault(x, []).append((n, i))

    def f32(a):
        a = np.asarray(a)
        return a.astype(np.float32) if a.dtype in (np.float16, np.float64) or a.dtype.kind == "f" else a

    out: dict = {}
    unresolved: list = []
    for name, arr in inits.items():
        if not _is_generated(name):
            out[name] = f32(arr)
            continue
        placed = False
        for node, idx in consumers.get(name, []):
            if node.op_type == "MatMul" and idx == 1 and np.ndim(arr) == 2:
                w = f32(arr).T
                pname = None
                for nxt, _ in _downstream(consumers, node.outputs[0]):
                    if nxt.op_type == "Add":
                        other = [x for x in nxt.inputs if x != node.outputs[0]]
                        if other and other[0] in inits and not _is_generated(other[0]):
                            b = other[0]
                            if b.endswith("in_proj_bias"):
                                pname = b[: -len("in_proj_bias")] + "in_proj_weight"
                            elif b.endswith("bias"):
                                pname = b[: -len("bias")] + "weight"
                if pname is None and node.name:
                    pname = _scope_to_param(node.name)
                if pname is None:
                    unresolved.append((node, w))
                else:
                    out[pname] = w
                placed = True
                break
            if node.op_type == "Gemm" and idx == 1 and np.ndim(arr) == 2:
                w = f32(arr) if node.attrs.get("transB", 0) else f32(arr).T
                pname = None
                if len(node.inputs) > 2 and node.inputs[2] in inits and not _is_generated(node.inputs[2]):
                    pname = node.inputs[2][: -len("bias")] + "weight" if node.inputs[2].endswith("bias") else None
                pname = pname or (_scope_to_param(node.name) if node.name else None)
                if pname is None:
                    unresolved.append((node, w))
                else:
                    out[pname] = w
                placed = True
                break
            if node.op_type in ("Conv", "ConvTranspose", "Gather") and node.name:
                suffix = "weight" if idx == (1 if node.op_type != "Gather" else 0) else "bias"
                pname = _scope_to_param(node.name, suffix)
                if pname is not None:
                    out[pname] = f32(arr)
                    placed = True
                    break
        if not placed:
            out.setdefault(name, f32(arr))
    return out, unresolved


def _downstream(consumers: dict, name: str, hops: int = 3) -> list:
    """Consumers of ``name``, looking through the Cast / Mul of a dequantised product
    (MatMulInteger -> Cast -> Mul(scales) -> Add(bias))."""
    out, frontier = [], [name]
    for _ in range(hops):
        nxt = []
        for v in frontier:
            for node, i in consumers.get(v, []):
                out.append((node, i))
                if node.op_type in ("Cast", "Mul"):
                    nxt.append(node.outputs[0])
        frontier = nxt
        if not frontier:
            break
    return out


def pick_file(root: Path, component: str, precision: Optional[str] = None) -> Optional[Path]:
    """``<component>.<precision>.onnx`` -> ``<component>.onnx`` -> ``.fp32`` -> ``.fp16`` / ``_fp16``
    (the reference's precedence, onnxrt_backend.py:_select_model_file)."""
    cands = []
    if precision:
        cands.append(root / f"{component}.{precision}.onnx")
    cands += [root / f"{component}.onnx", root / f"{component}.fp32.onnx", root / f"{component}.fp16.onnx",
              root / f"{component}_fp16.onnx"]
    return next((p for p in cands if p.exists()), None)


# ---------------------------------------------------------------------------- CLIP
def clip_state_dict(vision: Union[str, Path], text: Optional[Union[str, Path]] = None) -> dict:
    """torch state dict (OpenCLIP or HF ``CLIPModel`` naming, whichever the graphs were exported
    from) for :meth:`lumen_amd.models.clip.CLIPModel.load_state_dict_any`."""
    import torch

    sd: dict = {}
    for path, kind in ((vision, "vision"), (text, "text")):
        if path is None:
            continue
        part, unresolved = recover_state_dict(path)
        hf = any(k.startswith(("vision_model.", "text_model.")) for k in part)
        if unresolved:
            if len(unresolved) > 1:
                raise ValueError(f"{path}: {len(unresolved)} projection weights without a recoverable name")
            w = unresolved[0][1]          # [out, in] (transposed back from the MatMul operand)
            if kind == "vision":
                key, val = ("visual_projection.weight", w) if hf else ("visual.proj", w.T)
            else:
                key, val = ("text_projection.weight", w) if hf else ("text_projection", w.T)
            part[key] = val
        sd.update(part)
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items() if isinstance(v, np.ndarray)}


# ---------------------------------------------------------------------------- FastVLM
def vlm_state_dicts(vision: Union[str, Path], embed: Union[str, Path], decoder: Union[str, Path]) -> tuple[dict, dict]:
    """(vision-side dict, decoder dict in HF Qwen2 naming ``model.*``) from the three graphs."""
    import torch

    def tt(d):
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in d.items() if isinstance(v, np.ndarray)}

    dec, un = recover_state_dict(decoder)
    if un:
        # an untied lm_head is the only projection without a scope after the last norm
        if len(un) == 1:
            dec["lm_head.weight"] = un[0][1]
        else:
            raise ValueError(f"{decoder}: {len(un)} unresolved decoder weights")
    emb, _ = recover_state_dict(embed)
    if "model.embed_tokens.weight" not in dec:
        tables = [v for v in emb.values() if np.ndim(v) == 2]
        if len(tables) != 1:
            raise ValueError(f"{embed}: expected one embedding table, found {len(tables)}")
        dec["model.embed_tokens.weight"] = tables[0]
    vis, vun = recover_state_dict(vision)
    for node, w in vun:                    # projector Linears exported without scope names
        log.warning("vision graph: unnamed MatMul weight %s at node %s", w.shape, node.name)
    return tt(vis), tt(dec)


def load_vlm(model, vision: Union[str, Path], embed: Union[str, Path], decoder: Union[str, Path]) -> None:
    """Load a FastVLM ONNX pack into a :class:`lumen_amd.models.vlm.VLM` (FastViTHD tower)."""
    import torch

    vis, dec = vlm_state_dicts(vision, embed, decoder)
    if model.cfg.vision_arch != "fastvit":
        raise ValueError("ONNX VLM import supports the FastViTHD (FastVLM) vision tower")
    key = next((k for k in vis if ".stem.0." in "." + k or k.startswith("stem.0.")), None)
    if key is None:
        raise ValueError(f"{vision}: no FastViT stem found among {len(vis)} initializers")
    prefix = key[: ("." + key).index(".stem.0.")]          # "" or "<path>." (keeps its trailing dot)
    model.vision.load_timm(vis, prefix=prefix)
    proj = {}
    for k, v in vis.items():
        mm = re.search(r"mm_projector\.(\d+)\.(weight|bias)$", k)
        if mm:
            proj[(int(mm.group(1)), mm.group(2))] = v
    if len(proj) < 4:
        raise ValueError(f"{vision}: mm_projector weights not found ({sorted(proj)})")
    idx = sorted({i for i, _ in proj})
    with torch.no_grad():
        for dst, (li, kind) in ((model.proj1_w, (idx[0], "weight")), (model.proj1_b, (idx[0], "bias")),
                                (model.proj2_w, (idx[-1], "weight")), (model.proj2_b, (idx[-1], "bias"))):
            dst.copy_(proj[(li, kind)].to(dst.dtype))
    model.llm.load_hf_state_dict(dec)


def find_vlm_pack(root: Path, precision: Optional[str] = None) -> Optional[tuple[Path, Path, Path]]:
    d = root / "onnx" if (root / "onnx").is_dir() else root
    files = tuple(pick_file(d, c, precision) for c in ("vision", "embed", "decoder"))
    return files if all(files) else None  # type: ignore[return-value]


# ---------------------------------------------------------------------------- writers (tests, tools)
def fold_linear(name_w: str, w: np.ndarray, bias_name: Optional[str], x_in: str, scope: str, k: int,
                nodes: list, inits: dict, keep_scope: bool = True) -> str:
    """Emit MatMul(x, onnx::MatMul_k = W^T) [-> Add(bias)] like torch.onnx.export; returns the output."""
    wn = f"onnx::MatMul_{k}"
    inits[wn] = np.ascontiguousarray(w.T)
    mm = f"{scope}/MatMul_output_0"
    nodes.append(onnx_lite.Node("MatMul", [x_in, wn], [mm], name=f"{scope}/MatMul" if keep_scope else ""))
    if bias_name is None:
        return mm
    out = f"{scope}/Add_output_0"
    nodes.append(onnx_lite.Node("Add", [bias_name, mm], [out], name=f"{scope}/Add"))
    return out


def export_like_torch(sd: dict, linear_keys: Sequence[str], path: Union[str, Path], input_name: str = "input",
                      keep_scope: bool = True, drop_scope_for: Sequence[str] = (), fp16: bool = False) -> None:
    """Write an ONNX file whose initializers look like a ``torch.onnx.export`` of a model with
    state dict ``sd``: Linear weights in ``linear_keys`` folded to ``onnx::MatMul_<n>`` (scope
    from the parameter path, ``drop_scope_for`` without), everything else kept by name.  The
    graph is structural (weights + consumer nodes), for importer tests and tooling."""
    nodes: list = []
    inits: dict = {}
    x = input_name
    k = 0
    for key, t in sd.items():
        a = t.detach().float().cpu().numpy() if hasattr(t, "detach") else np.asarray(t, np.float32)
        if fp16:
            a = a.astype(np.float16)
        if key in linear_keys:
            mod = key[: -len("in_proj_weight")] + "in_proj" if key.endswith("in_proj_weight") else key[: -len(".weight")]
            bias = (mod[: -len("in_proj")] + "in_proj_bias") if key.endswith("in_proj_weight") else mod + ".bias"
            scope = "/" + mod.replace(".", "/")
            keep = keep_scope and key not in drop_scope_for
            x = fold_linear(key, a, bias if bias in sd else None, x, scope, k, nodes, inits, keep)
            k += 1
        else:
            inits[key] = a
            nodes.append(onnx_lite.Node("Identity", [key], [f"{key}__use"], name=""))
    g = onnx_lite.Graph(nodes=nodes, initializers=inits, inputs=[input_name], outputs=[x], name="lumen_export")
    Path(path).write_bytes(onnx_lite.write_model(g, opset=17))
