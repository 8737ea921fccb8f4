"""JSON-schema config / manifest validation (reference lumen_config_validator.py:19-270,
schemas/config-schema.yaml, model_info_validator.py).  ``jsonschema`` is not installed, so
``jsonschema_lite`` is tested directly, then against the Lumen schemas and — where the
reference tree is present — against the reference's own schema file and example configs."""
import copy
import glob
import json
import os
from pathlib import Path

import pytest
import yaml

from lumen_amd.resources.config import LumenConfig
from lumen_amd.resources.jsonschema_lite import SchemaValidator
from lumen_amd.resources.model_info import ModelInfo, model_info_schema_errors
from lumen_amd.resources.validator import ConfigValidator, schema_errors

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
EXAMPLES = sorted(glob.glob(str(ROOT / "examples/config/*.yaml")))


def test_lite_keywords():
    s = SchemaValidator({
        "definitions": {"pos": {"type": "integer", "minimum": 1}},
        "type": "object",
        "properties": {
            "a": {"$ref": "#/definitions/pos"},
            "b": {"oneOf": [{"type": "string"}, {"type": "integer"}]},
            "c": {"anyOf": [{"const": 1}, {"const": 2}]},
            "d": {"type": "array", "items": {"enum": ["x", "y"]}, "minItems": 1, "uniqueItems": True},
            "e": {"type": "object", "if": {"properties": {"on": {"const": True}}, "required": ["on"]},
                  "then": {"required": ["name"]}},
        },
        "required": ["a"],
        "additionalProperties": False,
    })
    assert s.errors({"a": 3, "b": "s", "c": 2, "d": ["x"], "e": {"on": False}}) == []
    errs = s.errors({"a": 0, "b": 1.5, "c": 3, "d": ["x", "x", "z"], "e": {"on": True}, "zz": 1})
    joined = "\n".join(errs)
    for frag in ("$.a: 0 < minimum 1", "$.b: must match exactly one form", "$.c: does not match any",
                 "$.d: items are not unique", "$.d[2]", "$.e: missing required property 'name'",
                 "unexpected property 'zz'"):
        assert frag in joined, (frag, errs)
    assert s.errors({"b": True}) and "missing required property 'a'" in s.errors({})[0]


@pytest.mark.parametrize("path", EXAMPLES)
def test_examples_valid(path):
    data = yaml.safe_load(open(path))
    assert schema_errors(data) == []
    ok, errs = ConfigValidator().validate_file(path, strict=True)
    assert ok, errs


def _base():
    return yaml.safe_load(open(ROOT / "examples/config/hub.example.yaml"))


@pytest.mark.parametrize("mutate,frag", [
    (lambda d: d["server"].__setitem__("port", 80), "$.server.port: 80 < minimum 1024"),
    (lambda d: d["server"].__setitem__("mdns", {"enabled": True}), "missing required property 'service_name'"),
    (lambda d: d.__setitem__("extra", 1), "unexpected property 'extra'"),
    (lambda d: d["metadata"].__setitem__("version", "1.0"), "$.metadata.version"),
    (lambda d: d["metadata"].__setitem__("region", "eu"), "$.metadata.region"),
    (lambda d: d.__setitem__("deployment", {"mode": "single"}), "$.deployment: must match exactly one form"),
    (lambda d: next(iter(d["services"].values()))["backend_settings"].__setitem__("dp", 8),
     "unexpected property 'dp'"),
    (lambda d: next(iter(next(iter(d["services"].values()))["models"].values())).__setitem__("runtime", "rknn"),
     "missing required property 'rknn_device'"),
    (lambda d: next(iter(d["services"].values()))["import_info"].__setitem__("registry_class", "Bad"),
     "registry_class"),
])
def test_invalid_configs_named(mutate, frag):
    d = _base()
    mutate(d)
    errs = schema_errors(d)
    assert any(frag in e for e in errs), errs


def test_strict_cross_references():
    from lumen_amd.resources.validator import semantic_errors, structural_errors

    d = _base()
    d["deployment"]["services"] = ["nosuch"]
    assert schema_errors(d) == []
    assert any("hub service 'nosuch' is not defined" in e for e in semantic_errors(d) + structural_errors(d))


def test_schema_agrees_with_pydantic():
    """Random single-field corruptions: the schema must reject whatever pydantic rejects
    (same contract whichever validation mode a user picks)."""
    import random

    rng = random.Random(0)
    base = _base()
    leaves = []

    def walk(node, path):
        if isinstance(node, dict):
            for k, v in node.items():
                walk(v, path + [k])
        elif isinstance(node, list):
            for i, v in enumerate(node):
                walk(v, path + [i])
        else:
            leaves.append(path)

    walk(base, [])
    bad_values = [None, -1, 0, 70000, "", "UPPER", 1.5, True, [], {}]
    n_checked = 0
    for _ in range(300):
        d = copy.deepcopy(base)
        p = rng.choice(leaves)
        node = d
        for k in p[:-1]:
            node = node[k]
        node[p[-1]] = rng.choice(bad_values)
        try:
            LumenConfig.model_validate(d)
            py_ok = True
        except Exception:
            py_ok = False
        if not py_ok:
            assert schema_errors(d), (p, node[p[-1]])
            n_checked += 1
    assert n_checked > 50


@pytest.mark.skipif(not (REF / "packages/lumen-resources/src/lumen_resources/schemas/config-schema.yaml").exists(),
                    reason="reference tree not present")
def test_reference_schema_and_examples():
    """The reference's own Draft-7 schema, run by jsonschema_lite, accepts the reference's
    example configs and ours, and agrees with our schema on them."""
    ref_schema = SchemaValidator.from_file(REF / "packages/lumen-resources/src/lumen_resources/schemas/config-schema.yaml")
    ref_examples = sorted(glob.glob(str(REF / "packages/*/examples/config/*.yaml")))
    assert ref_examples
    for p in ref_examples + EXAMPLES:
        data = yaml.safe_load(open(p))
        assert ref_schema.errors(data) == [], (p, ref_schema.errors(data))
        assert schema_errors(data) == [], (p, schema_errors(data))
    bad = _base()
    bad["server"]["port"] = 5
    assert ref_schema.errors(bad) and schema_errors(bad)


def test_model_info_schema(tmp_path):
    good = {"name": "m", "version": "1.0.0", "description": "d", "model_type": "clip", "embedding_dim": 512,
            "source": {"format": "custom", "repo_id": "x/y"},
            "runtimes": {"onnx": {"available": True, "files": ["onnx/vision.fp32.onnx"]},
                         "rknn": {"available": False, "files": {"rk3588": ["a.rknn"]}}},
            "datasets": {"ImageNet_1k": {"labels": "l.json", "embeddings": "e.npy"}}}
    assert model_info_schema_errors(good) == []
    ModelInfo.model_validate(good)
    for mut, frag in [(lambda d: d.pop("source"), "missing required property 'source'"),
                      (lambda d: d.__setitem__("version", "v1"), "$.version"),
                      (lambda d: d["source"].__setitem__("format", "zip"), "$.source.format"),
                      (lambda d: d["runtimes"]["onnx"].__setitem__("files", 3), "$.runtimes.onnx.files"),
                      (lambda d: d.__setitem__("embedding_dim", 0), "$.embedding_dim")]:
        d = copy.deepcopy(good)
        mut(d)
        assert any(frag in e for e in model_info_schema_errors(d)), (frag, model_info_schema_errors(d))
    ref_mi = REF / "packages/lumen-resources/docs/examples/model_info_template.json"
    if ref_mi.exists():
        data = json.loads(ref_mi.read_text())
        # the template is a documentation skeleton; it must at least parse with our schema's structure
        assert isinstance(model_info_schema_errors(data), list)


def test_cli_schema_only(tmp_path, capsys):
    from lumen_amd.resources.cli import main

    cfg = tmp_path / "c.yaml"
    d = _base()
    cfg.write_text(yaml.safe_dump(d))
    assert main(["validate", str(cfg), "--schema-only"]) == 0
    d["server"]["port"] = 1
    cfg.write_text(yaml.safe_dump(d))
    assert main(["validate", str(cfg), "--schema-only"]) == 1
    assert "minimum 1024" in capsys.readouterr().out
