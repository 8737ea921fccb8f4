"""A small JSON-Schema (Draft-7 subset) validator — the ``jsonschema`` wheel is not part of
this image, and config validation must work without it.

Supports the keywords the Lumen schemas use (reference
packages/lumen-resources/src/lumen_resources/schemas/config-schema.yaml and
model_info-schema.json): ``type`` (incl. lists and ``integer``), ``enum``, ``const``,
``properties``, ``required``, ``additionalProperties`` (bool or schema),
``patternProperties``, ``propertyNames``, ``minProperties``, ``items`` (schema),
``minItems`` / ``maxItems`` / ``uniqueItems``, ``minLength`` / ``maxLength`` / ``pattern``,
``minimum`` / ``maximum`` / ``exclusiveMinimum`` / ``exclusiveMaximum``, ``allOf`` /
``anyOf`` / ``oneOf`` / ``not``, ``if`` / ``then`` / ``else``, ``$ref`` to
``#/definitions/...`` (and ``$defs``).  Errors carry a JSON path (``$.server.port``).
"""
from __future__ import annotations

import json
import re
from pathlib import Path
from typing import Any, Union

_TYPES = {
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
    "string": lambda v: isinstance(v, str),
    "boolean": lambda v: isinstance(v, bool),
    "null": lambda v: v is None,
    "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
}


class SchemaValidator:
    def __init__(self, schema: dict):
        self.schema = schema

    @classmethod
    def from_file(cls, path: Union[str, Path]) -> "SchemaValidator":
        p = Path(path)
        text = p.read_text(encoding="utf-8")
        if p.suffix in (".yaml", ".yml"):
            import yaml

            return cls(yaml.safe_load(text))
        return cls(json.loads(text))

    # ---- public
    def errors(self, data: Any) -> list[str]:
        out: list[str] = []
        self._check(data, self.schema, "$", out)
        return out

    def is_valid(self, data: Any) -> bool:
        return not self.errors(data)

    # ---- internals
    def _resolve(self, ref: str) -> dict:
        if not ref.startswith("#/"):
            raise ValueError(f"only local $ref supported: {ref}")
        node: Any = self.schema
        for part in ref[2:].split("/"):
            node = node[part.replace("~1", "/").replace("~0", "~")]
        return node

    def _check(self, v: Any, s: Any, path: str, out: list[str]) -> None:
        if s is True or s is None:
            return
        if s is False:
            out.append(f"{path}: no value allowed here")
            return
        if "$ref" in s:
            self._check(v, self._resolve(s["$ref"]), path, out)
        t = s.get("type")
        if t is not None:
            ts = t if isinstance(t, list) else [t]
            if not any(_TYPES[x](v) for x in ts):
                out.append(f"{path}: expected {' or '.join(ts)}, got {type(v).__name__}")
                return
        if "enum" in s and v not in s["enum"]:
            out.append(f"{path}: {v!r} is not one of {s['enum']}")
        if "const" in s and v != s["const"]:
            out.append(f"{path}: must be {s['const']!r}")
        if isinstance(v, str):
            if "minLength" in s and len(v) < s["minLength"]:
                out.append(f"{path}: shorter than {s['minLength']}")
            if "maxLength" in s and len(v) > s["maxLength"]:
                out.append(f"{path}: longer than {s['maxLength']}")
            if "pattern" in s and re.search(s["pattern"], v) is None:
                out.append(f"{path}: {v!r} does not match {s['pattern']!r}")
        if _TYPES["number"](v):
            if "minimum" in s and v < s["minimum"]:
                out.append(f"{path}: {v} < minimum {s['minimum']}")
            if "maximum" in s and v > s["maximum"]:
                out.append(f"{path}: {v} > maximum {s['maximum']}")
            if "exclusiveMinimum" in s and v <= s["exclusiveMinimum"]:
                out.append(f"{path}: {v} <= exclusiveMinimum {s['exclusiveMinimum']}")
            if "exclusiveMaximum" in s and v >= s["exclusiveMaximum"]:
                out.append(f"{path}: {v} >= exclusiveMaximum {s['exclusiveMaximum']}")
        if isinstance(v, list):
            if "minItems" in s and len(v) < s["minItems"]:
                out.append(f"{path}: fewer than {s['minItems']} items")
            if "maxItems" in s and len(v) > s["maxItems"]:
                out.append(f"{path}: more than {s['maxItems']} items")
            if s.get("uniqueItems") and len({json.dumps(x, sort_keys=True) for x in v}) != len(v):
                out.append(f"{path}: items are not unique")
            if "items" in s:
                it = s["items"]
                if isinstance(it, list):
                    for i, (x, si) in enumerate(zip(v, it)):
                        self._check(x, si, f"{path}[{i}]", out)
                else:
                    for i, x in enumerate(v):
                        self._check(x, it, f"{path}[{i}]", out)
        if isinstance(v, dict):
            props = s.get("properties", {})
            for k in s.get("required", []):
                if k not in v:
                    out.append(f"{path}: missing required property '{k}'")
            if "minProperties" in s and len(v) < s["minProperties"]:
                out.append(f"{path}: fewer than {s['minProperties']} properties")
            pats = s.get("patternProperties", {})
            addl = s.get("additionalProperties", True)
            for k, x in v.items():
                sub = f"{path}.{k}"
                if "propertyNames" in s:
                    self._check(k, s["propertyNames"], f"{path}[key {k!r}]", out)
                matched = False
                if k in props:
                    self._check(x, props[k], sub, out)
                    matched = True
                for pat, ps in pats.items():
                    if re.search(pat, k):
                        self._check(x, ps, sub, out)
                        matched = True
                if not matched:
                    if addl is False:
                        out.append(f"{path}: unexpected property '{k}'")
                    elif isinstance(addl, dict):
                        self._check(x, addl, sub, out)
        for sub in s.get("allOf", []):
            self._check(v, sub, path, out)
        if "anyOf" in s and not any(not self._sub(v, x, path) for x in s["anyOf"]):
            out.append(f"{path}: does not match any allowed form ({self._why(v, s['anyOf'], path)})")
        if "oneOf" in s:
            ok = [x for x in s["oneOf"] if not self._sub(v, x, path)]
            if len(ok) != 1:
                what = "none" if not ok else f"{len(ok)}"
                out.append(f"{path}: must match exactly one form, matched {what} ({self._why(v, s['oneOf'], path)})")
        if "not" in s and not self._sub(v, s["not"], path):
            out.append(f"{path}: matches a forbidden form")
        if "if" in s:
            if not self._sub(v, s["if"], path):
                if "then" in s:
                    self._check(v, s["then"], path, out)
            elif "else" in s:
                self._check(v, s["else"], path, out)

    def _sub(self, v, s, path) -> list[str]:
        o: list[str] = []
        self._check(v, s, path, o)
        return o

    def _why(self, v, alts, path) -> str:
        best = min((self._sub(v, x, path) for x in alts), key=len)
        return "; ".join(best[:2]) if best else "ambiguous"
