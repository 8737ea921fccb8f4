"""Config validation: strict (JSON schema + pydantic) and schema-only (JSON schema) modes.

Mirrors packages/lumen-resources/src/lumen_resources/lumen_config_validator.py:19-270
(``load_and_validate_config``, ``ConfigValidator.validate_and_load``, ``--schema-only``).
The Draft-7 schema ``schemas/config-schema.json`` (checked by :mod:`jsonschema_lite`)
carries the conditional rules of the reference's config-schema.yaml — ``oneOf`` single |
hub deployment, mdns.service_name required when mDNS is enabled, rknn_device required
for runtime=rknn — and :func:`semantic_errors` the cross-references a schema cannot
express (deployment.service / every hub service must be configured).
"""
from __future__ import annotations

import re
from pathlib import Path
from typing import Any, Union

import yaml

from .config import LumenConfig
from .exceptions import ConfigError
from .jsonschema_lite import SchemaValidator

SCHEMA_DIR = Path(__file__).resolve().parent / "schemas"
_CONFIG_SCHEMA: "SchemaValidator | None" = None


def config_schema() -> SchemaValidator:
    global _CONFIG_SCHEMA
    if _CONFIG_SCHEMA is None:
        _CONFIG_SCHEMA = SchemaValidator.from_file(SCHEMA_DIR / "config-schema.json")
    return _CONFIG_SCHEMA


def schema_errors(data: dict) -> list[str]:
    """JSON-schema validation only (``--schema-only``; like the reference, cross-references
    between nodes are checked in strict mode only — a reference example config names a
    service key that does not exist and still passes its schema)."""
    return config_schema().errors(data)


def semantic_errors(data: dict) -> list[str]:
    """Rules that need more than one node of the document."""
    errs: list[str] = []
    dep = data.get("deployment") if isinstance(data, dict) else None
    services = data.get("services") if isinstance(data, dict) else None
    if not isinstance(dep, dict) or not isinstance(services, dict):
        return errs
    if dep.get("mode") == "single" and isinstance(dep.get("service"), str) and dep["service"] not in services:
        errs.append(f"deployment.service '{dep['service']}' is not defined under services")
    if dep.get("mode") == "hub":
        for s in dep.get("services") or []:
            if isinstance(s, str) and s not in services:
                errs.append(f"hub service '{s}' is not defined under services")
    return errs


def _load_yaml(path: Union[str, Path]) -> dict:
    p = Path(path).expanduser()
    if not p.exists():
        raise ConfigError(f"config file not found: {p}")
    try:
        data = yaml.safe_load(p.read_text(encoding="utf-8"))
    except yaml.YAMLError as e:
        raise ConfigError(f"invalid YAML in {p}: {e}") from e
    if not isinstance(data, dict):
        raise ConfigError(f"config root must be a mapping: {p}")
    return data


def structural_errors(data: dict) -> list[str]:
    """Schema-level checks that do not need pydantic (``--schema-only``)."""
    errs: list[str] = []
    for key in ("metadata", "deployment", "server", "services"):
        if key not in data:
            errs.append(f"missing required key '{key}'")
    extra = set(data) - {"metadata", "deployment", "server", "services"}
    if extra:
        errs.append(f"unexpected top-level keys: {sorted(extra)}")
    md = data.get("metadata") or {}
    if not re.match(r"^\d+\.\d+\.\d+$", str(md.get("version", ""))):
        errs.append("metadata.version must be semantic x.y.z")
    if md.get("region") not in ("cn", "other"):
        errs.append("metadata.region must be 'cn' or 'other'")
    if not md.get("cache_dir"):
        errs.append("metadata.cache_dir is required")
    dep = data.get("deployment") or {}
    mode = dep.get("mode")
    services = data.get("services") or {}
    if mode == "single":
        if not dep.get("service"):
            errs.append("deployment.service is required when mode=single")
        elif dep["service"] not in services:
            errs.append(f"deployment.service '{dep['service']}' is not defined under services")
    elif mode == "hub":
        svcs = dep.get("services") or []
        if not svcs:
            errs.append("deployment.services must list at least one service when mode=hub")
        for s in svcs:
            if s not in services:
                errs.append(f"hub service '{s}' is not defined under services")
    else:
        errs.append("deployment.mode must be 'single' or 'hub'")
    srv = data.get("server") or {}
    port = srv.get("port")
    if not isinstance(port, int) or not (1024 <= port <= 65535):
        errs.append("server.port must be an integer in [1024, 65535]")
    mdns = srv.get("mdns") or {}
    if mdns.get("enabled") and not mdns.get("service_name"):
        errs.append("server.mdns.service_name is required when mdns.enabled is true")
    for name, svc in services.items():
        if not isinstance(svc, dict):
            errs.append(f"services.{name} must be a mapping")
            continue
        bs = svc.get("backend_settings") or {}
        extra = set(bs) - {"device", "batch_size", "onnx_providers"}
        if extra:
            errs.append(f"services.{name}.backend_settings has unknown keys {sorted(extra)}")
        for alias, m in (svc.get("models") or {}).items():
            if m.get("runtime") not in ("torch", "onnx", "rknn"):
                errs.append(f"services.{name}.models.{alias}.runtime must be torch|onnx|rknn")
            if m.get("runtime") == "rknn" and not m.get("rknn_device"):
                errs.append(f"services.{name}.models.{alias}.rknn_device is required for runtime=rknn")
    return errs


class ConfigValidator:
    def validate_file(self, path, strict: bool = True) -> tuple[bool, list[str]]:
        """strict: JSON schema + hand rules + pydantic; schema-only: JSON schema + cross-refs."""
        try:
            data = _load_yaml(path)
        except ConfigError as e:
            return False, [str(e)]
        errs = schema_errors(data)
        if strict and not errs:
            errs = structural_errors(data)
        if strict and not errs:
            try:
                LumenConfig.model_validate(data)
            except Exception as e:
                errs.append(str(e))
        return not errs, errs

    def validate_and_load(self, path) -> LumenConfig:
        data = _load_yaml(path)
        errs = schema_errors(data) or structural_errors(data)
        if errs:
            raise ConfigError("configuration invalid:\n  - " + "\n  - ".join(errs))
        try:
            return LumenConfig.model_validate(data)
        except Exception as e:
            raise ConfigError(f"configuration invalid: {e}") from e


def load_and_validate_config(path: Union[str, Path]) -> LumenConfig:
    """Load a LumenConfig YAML file and validate it (raises ConfigError)."""
    return ConfigValidator().validate_and_load(path)


def config_from_dict(data: dict[str, Any]) -> LumenConfig:
    errs = schema_errors(data) or structural_errors(data)
    if errs:
        raise ConfigError("configuration invalid:\n  - " + "\n  - ".join(errs))
    return LumenConfig.model_validate(data)
