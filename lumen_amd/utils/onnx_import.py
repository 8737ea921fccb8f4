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


def recover_state_dict(src: Union[str, Path, bytes, onnx_lite.Model]) -> tuple[dict, list]:
    """(name -> np.float32 array in PyTorch layout, [unresolved (node, array)]) of one graph."""
    m = src if isinstance(src, onnx_lite.Model) else onnx_lite.load_model(src)
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
                for nxt, _ in consumers.get(node.outputs[0], []):
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
