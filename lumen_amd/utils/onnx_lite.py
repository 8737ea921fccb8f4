"""Minimal ONNX (protobuf wire format) reader / writer — no ``onnx`` package needed.

The reference ships its face / OCR / VLM models as ONNX graphs run by ONNX Runtime
(packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py, lumen-ocr/.../onnxrt_backend.py,
lumen-vlm/.../onnxrt_backend.py).  This module parses exactly the subset of ``onnx.proto3``
that a graph executor needs — ModelProto.graph / opset_import, GraphProto.{node, initializer,
input, output}, NodeProto, AttributeProto, TensorProto (raw or typed data, external data
files), ValueInfoProto names — by decoding the protobuf wire format directly, so loading a
model executes nothing from the file.  ``write_model`` is the inverse for the same subset
(used to build test graphs).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Optional, Union

import numpy as np

# TensorProto.DataType -> numpy
DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_,
          10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}
BF16 = 16
NP2ONNX = {np.dtype(v): k for k, v in DTYPES.items()}


@dataclass
class Tensor:
    name: str
    array: np.ndarray


@dataclass
class Node:
    op_type: str
    inputs: list
    outputs: list
    name: str = ""
    attrs: dict = field(default_factory=dict)
    domain: str = ""


@dataclass
class Graph:
    nodes: list
    initializers: dict                      # name -> np.ndarray
    inputs: list                            # graph input names (initializers excluded)
    outputs: list
    name: str = ""


@dataclass
class Model:
    graph: Graph
    opset: int = 13
    ir_version: int = 8
    producer: str = ""


# ------------------------------------------------------------------------------ wire format
def _varint(b: memoryview, i: int) -> tuple[int, int]:
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, i
        s += 7


def _fields(b: memoryview):
    """yield (field_number, wire_type, value) — value is int or memoryview."""
    i, n = 0, len(b)
    while i < n:
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _packed_varints(v) -> list[int]:
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def _signed64(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


def _read_external(base_dir: Path, name: str, external: dict) -> bytes:
    """Read an external-data initializer, confined to the model directory.

    A downloaded pack is untrusted: an absolute ``location`` or one with ``..`` that
    resolves outside ``base_dir`` is refused (it could pull any host file into a
    weight tensor), and offset/length are checked against the file size before
    reading (no unbounded reads of devices such as /dev/zero)."""
    loc = external.get("location", "")
    if not loc or Path(loc).is_absolute():
        raise ValueError(f"tensor {name}: external data location {loc!r} must be a relative path")
    root = base_dir.resolve()
    p = (root / loc).resolve()
    if root != p and root not in p.parents:
        raise ValueError(f"tensor {name}: external data {loc!r} escapes the model directory")
    if not p.is_file():
        raise ValueError(f"tensor {name}: external data file {loc!r} not found")
    size = p.stat().st_size
    off = int(external.get("offset", 0))
    ln = int(external["length"]) if external.get("length") else size - off
    if off < 0 or ln < 0 or off + ln > size:
        raise ValueError(f"tensor {name}: external data range [{off}, {off + ln}) outside {loc!r} ({size} B)")
    with open(p, "rb") as fh:
        fh.seek(off)
        return fh.read(ln)


def _parse_tensor(b: memoryview, base_dir: Optional[Path]) -> Tensor:
    dims, dtype, name, raw = [], 1, "", None
    floats, int32s, int64s, doubles = [], [], [], []
    external: dict = {}
    location = 0
    for f, wt, v in _fields(b):
        if f == 1:
            dims.extend(_signed64(x) for x in (_packed_varints(v) if wt == 2 else [v]))
        elif f == 2:
            dtype = v
        elif f == 4:
            floats.extend(np.frombuffer(bytes(v), "<f4") if wt == 2 else [struct.unpack("<f", bytes(v))[0]])
        elif f == 5:
            int32s.extend(_packed_varints(v) if wt == 2 else [v])
        elif f == 7:
            int64s.extend(_signed64(x) for x in (_packed_varints(v) if wt == 2 else [v]))
        elif f == 8:
            name = bytes(v).decode()
        elif f == 9:
            raw = bytes(v)
        elif f == 10:
            doubles.extend(np.frombuffer(bytes(v), "<f8") if wt == 2 else [struct.unpack("<d", bytes(v))[0]])
        elif f == 13:
            k = val = ""
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    k = bytes(v2).decode()
                elif f2 == 2:
                    val = bytes(v2).decode()
            external[k] = val
        elif f == 14:
            location = v
    shape = tuple(dims)
    if location == 1:                          # external data
        if base_dir is None:
            raise ValueError(f"tensor {name}: external data without a model path")
        raw = _read_external(Path(base_dir), name, external)
    if dtype == BF16:
        u16 = np.frombuffer(raw, "<u2") if raw is not None else np.asarray(int32s, np.uint16)
        arr = (u16.astype(np.uint32) << 16).view(np.float32)
    elif raw is not None:
        arr = np.frombuffer(raw, dtype=np.dtype(DTYPES[dtype]).newbyteorder("<")).astype(DTYPES[dtype])
    elif dtype in (1,):
        arr = np.asarray(floats, np.float32)
    elif dtype == 11:
        arr = np.asarray(doubles, np.float64)
    elif dtype == 7:
        arr = np.asarray(int64s, np.int64)
    elif dtype == 10:
        arr = np.asarray(int32s, np.uint16).view(np.float16)
    else:
        arr = np.asarray(int32s, DTYPES[dtype])
    return Tensor(name, arr.reshape(shape) if shape else arr.reshape(()))


def _parse_attr(b: memoryview, base_dir) -> tuple[str, Any]:
    name, f_, i_, s_, t_ = "", None, None, None, None
    fl, il, sl = [], [], []
    for f, wt, v in _fields(b):
        if f == 1:
            name = bytes(v).decode()
        elif f == 2:
            f_ = struct.unpack("<f", bytes(v))[0]
        elif f == 3:
            i_ = _signed64(v)
        elif f == 4:
            s_ = bytes(v)
        elif f == 5:
            t_ = _parse_tensor(v, base_dir).array
        elif f == 7:
            fl.extend(np.frombuffer(bytes(v), "<f4").tolist() if wt == 2 else [struct.unpack("<f", bytes(v))[0]])
        elif f == 8:
            il.extend(_signed64(x) for x in (_packed_varints(v) if wt == 2 else [v]))
        elif f == 9:
            sl.append(bytes(v))
    for val in (f_, i_, s_, t_):
        if val is not None:
            return name, (val.decode() if isinstance(val, bytes) else val)
    if fl:
        return name, fl
    if il:
        return name, il
    if sl:
        return name, [x.decode() for x in sl]
    return name, []


def _parse_node(b: memoryview, base_dir) -> Node:
    n = Node("", [], [])
    for f, _, v in _fields(b):
        if f == 1:
            n.inputs.append(bytes(v).decode())
        elif f == 2:
            n.outputs.append(bytes(v).decode())
        elif f == 3:
            n.name = bytes(v).decode()
        elif f == 4:
            n.op_type = bytes(v).decode()
        elif f == 5:
            k, val = _parse_attr(v, base_dir)
            n.attrs[k] = val
        elif f == 7:
            n.domain = bytes(v).decode()
    return n


def _value_name(b: memoryview) -> str:
    for f, _, v in _fields(b):
        if f == 1:
            return bytes(v).decode()
    return ""


def _parse_graph(b: memoryview, base_dir) -> Graph:
    g = Graph([], {}, [], [])
    ins = []
    for f, _, v in _fields(b):
        if f == 1:
            g.nodes.append(_parse_node(v, base_dir))
        elif f == 2:
            g.name = bytes(v).decode()
        elif f == 5:
            t = _parse_tensor(v, base_dir)
            g.initializers[t.name] = t.array
        elif f == 11:
            ins.append(_value_name(v))
        elif f == 12:
            g.outputs.append(_value_name(v))
    g.inputs = [x for x in ins if x not in g.initializers]
    return g


def load_model(src: Union[str, Path, bytes]) -> Model:
    """Parse an ONNX file (or bytes).  Nothing in the file is executed."""
    base_dir = None
    if isinstance(src, (str, Path)):
        base_dir = Path(src).parent
        data = Path(src).read_bytes()
    else:
        data = bytes(src)
    m = Model(graph=Graph([], {}, [], []))
    for f, _, v in _fields(memoryview(data)):
        if f == 1:
            m.ir_version = v
        elif f == 2:
            m.producer = bytes(v).decode()
        elif f == 7:
            m.graph = _parse_graph(v, base_dir)
        elif f == 8:
            dom, ver = "", 0
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    dom = bytes(v2).decode()
                elif f2 == 2:
                    ver = v2
            if dom in ("", "ai.onnx"):
                m.opset = ver
    return m


def load_initializers(src) -> dict:
    """name -> np.ndarray of every graph initializer (ONNX-initializer weight extraction)."""
    return load_model(src).graph.initializers


# ------------------------------------------------------------------------------ writer
def _enc_varint(x: int) -> bytes:
    if x < 0:
        x += 1 << 64
    out = bytearray()
    while True:
        c = x & 0x7F
        x >>= 7
        if x:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _key(f: int, wt: int) -> bytes:
    return _enc_varint((f << 3) | wt)


def _ld(f: int, payload: bytes) -> bytes:
    return _key(f, 2) + _enc_varint(len(payload)) + payload


def _vi(f: int, x: int) -> bytes:
    return _key(f, 0) + _enc_varint(x)


def _tensor_bytes(name: str, a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a)
    out = b"".join(_vi(1, d) for d in a.shape)
    out += _vi(2, NP2ONNX[a.dtype])
    out += _ld(8, name.encode())
    out += _ld(9, a.astype(a.dtype.newbyteorder("<")).tobytes())
    return out


def _attr_bytes(name: str, v) -> bytes:
    out = _ld(1, name.encode())
    if isinstance(v, float):
        return out + _key(2, 5) + struct.pack("<f", v) + _vi(20, 1)
    if isinstance(v, (bool, int, np.integer)):
        return out + _vi(3, int(v)) + _vi(20, 2)
    if isinstance(v, str):
        return out + _ld(4, v.encode()) + _vi(20, 3)
    if isinstance(v, np.ndarray):
        return out + _ld(5, _tensor_bytes("", v)) + _vi(20, 4)
    if isinstance(v, (list, tuple)):
        if v and all(isinstance(x, float) for x in v):
            return out + b"".join(_key(7, 5) + struct.pack("<f", x) for x in v) + _vi(20, 6)
        return out + b"".join(_vi(8, int(x)) for x in v) + _vi(20, 7)
    raise TypeError(f"attribute {name}: {type(v)}")


def write_model(graph: Graph, opset: int = 13) -> bytes:
    g = b""
    for n in graph.nodes:
        nb = b"".join(_ld(1, x.encode()) for x in n.inputs) + b"".join(_ld(2, x.encode()) for x in n.outputs)
        nb += _ld(3, (n.name or n.outputs[0]).encode()) + _ld(4, n.op_type.encode())
        nb += b"".join(_ld(5, _attr_bytes(k, v)) for k, v in n.attrs.items())
        g += _ld(1, nb)
    g += _ld(2, (graph.name or "g").encode())
    for k, a in graph.initializers.items():
        g += _ld(5, _tensor_bytes(k, a))
    for x in graph.inputs:
        g += _ld(11, _ld(1, x.encode()))
    for x in graph.outputs:
        g += _ld(12, _ld(1, x.encode()))
    return _vi(1, 8) + _ld(2, b"lumen_amd") + _ld(7, g) + _ld(8, _ld(1, b"") + _vi(2, opset))
