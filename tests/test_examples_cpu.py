"""Example configurations (examples/config/*.example.yaml, the counterparts of the reference's
per-package examples/config and lumen-resources docs/examples) validate against the config
schema and every registry_class resolves to an MI355X service class."""
from pathlib import Path

import pytest

from lumen_amd.hub.loader import resolve_path
from lumen_amd.resources.validator import load_and_validate_config

EXAMPLES = sorted((Path(__file__).resolve().parents[1] / "examples" / "config").glob("*.example.yaml"))


def test_examples_present():
    names = {p.name.split(".")[0] for p in EXAMPLES}
    assert {"clip_cn", "bioclip", "unified", "face", "ocr", "vlm", "hub"} <= names


@pytest.mark.parametrize("path", EXAMPLES, ids=lambda p: p.name)
def test_example_validates_and_resolves(path):
    import importlib

    cfg = load_and_validate_config(path)
    enabled = cfg.enabled_services()
    assert enabled
    if cfg.deployment.mode.value == "single" if hasattr(cfg.deployment.mode, "value") else cfg.deployment.mode == "single":
        assert cfg.deployment.service in enabled
    for name, sc in enabled.items():
        target = resolve_path(sc.import_info.registry_class)
        assert target.startswith("lumen_amd.services."), target
        mod, cls = target.rsplit(".", 1)
        assert hasattr(importlib.import_module(mod), cls)
        assert sc.models


@pytest.mark.parametrize("ctype", ["minimal", "light_weight", "basic", "brave"])
@pytest.mark.parametrize("region", ["cn", "other"])
def test_generated_configs_import_strings_resolve(ctype, region):
    """Counterpart of the reference's tests/test_package_init_contract.py: every
    registry_class / add_to_server string the control plane writes into a generated
    config imports (via the hub loader) to a real MI355X object, for every preset."""
    from lumen_amd.app import presets as P
    from lumen_amd.hub.loader import ServiceLoader
    from lumen_amd.resources.config import Region

    for name in P.detection_order():
        c = P.Config("~/.lumen", P.PRESETS[name].create_config(), Region(region), "lumen-ai", 50051)
        lc = getattr(c, ctype)()
        for svc in lc.services.values():
            cls = ServiceLoader.get_class(svc.import_info.registry_class)
            assert hasattr(cls, "from_config"), svc.import_info.registry_class
            assert callable(ServiceLoader.get_class(svc.import_info.add_to_server))
            for m in svc.models.values():
                assert m.model
