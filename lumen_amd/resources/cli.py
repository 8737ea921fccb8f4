"""``lumen-resources`` CLI: download / validate / validate-model-info / list
(reference packages/lumen-resources/src/lumen_resources/cli.py:314-398).

``download`` fetches every enabled service's models into ``<cache_dir>/models``; with
no network (or ``--synthetic`` / ``LUMEN_SYNTHETIC=1``) it writes random-init model
packs of the right architecture so the stack can be exercised end to end.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

from .exceptions import ConfigError, ModelInfoError
from .model_info import load_and_validate_model_info
from .validator import load_and_validate_config


def cmd_download(a) -> int:
    from .downloader import Downloader

    cfg = load_and_validate_config(a.config)
    d = Downloader(cfg, verbose=True, synthetic=True if a.synthetic else None)
    res = d.download_all(force=a.force)
    ok = True
    for key, r in res.items():
        tag = "synthetic" if r.synthetic else ("ok" if r.success else "FAILED")
        print(f"  [{tag}] {key}: {r.model_path or ''} {r.error or ''}".rstrip())
        ok &= r.success
    print(f"{sum(r.success for r in res.values())}/{len(res)} models ready in {cfg.cache_path()}/models")
    return 0 if ok else 1


def cmd_validate(a) -> int:
    if not getattr(a, "strict", True):
        from .validator import ConfigValidator

        ok, errs = ConfigValidator().validate_file(a.config, strict=False)
        if not ok:
            print("invalid configuration (schema):\n  - " + "\n  - ".join(errs))
            return 1
        print(f"valid configuration (schema only): {a.config}")
        return 0
    try:
        cfg = load_and_validate_config(a.config)
    except (ConfigError, Exception) as e:  # noqa: BLE001
        print(f"invalid configuration: {e}")
        return 1
    svcs = ", ".join(cfg.enabled_services())
    print(f"valid configuration ({cfg.deployment.mode} mode; services: {svcs})")
    return 0


def cmd_validate_model_info(a) -> int:
    if not getattr(a, "strict", True):
        import json as _json

        from .model_info import model_info_schema_errors

        p = Path(a.model_info)
        p = p / "model_info.json" if p.is_dir() else p
        try:
            errs = model_info_schema_errors(_json.loads(p.read_text(encoding="utf-8")))
        except (OSError, ValueError) as e:
            errs = [str(e)]
        if errs:
            print("invalid model_info (schema):\n  - " + "\n  - ".join(errs))
            return 1
        print(f"valid model_info (schema only): {p}")
        return 0
    try:
        info = load_and_validate_model_info(a.model_info)
    except (ModelInfoError, Exception) as e:  # noqa: BLE001
        print(f"invalid model_info: {e}")
        return 1
    rts = [k for k, v in info.runtimes.items() if v.available]
    print(f"valid model_info: {info.name} {info.version} ({info.model_type}); runtimes: {', '.join(rts)}")
    return 0


def cmd_list(a) -> int:
    root = Path(a.cache_dir).expanduser() / "models"
    if not root.exists():
        print(f"no models cached in {root}")
        return 0
    for md in sorted(p for p in root.iterdir() if p.is_dir()):
        print(f"  - {md.name}")
        mi = md / "model_info.json"
        if mi.exists():
            try:
                info = json.loads(mi.read_text())
                rts = [k for k, v in info.get("runtimes", {}).items() if v.get("available")]
                print(f"     Type: {info.get('model_type')}  Version: {info.get('version')}")
                if rts:
                    print(f"     Runtimes: {', '.join(rts)}")
            except Exception:  # noqa: BLE001
                pass
        subdirs = [d.name for d in md.iterdir() if d.is_dir()]
        if subdirs:
            print(f"     Contents: {', '.join(subdirs)}")
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="lumen-resources", description="Lumen Resources - Model Resource Manager")
    sub = ap.add_subparsers(dest="command")
    d = sub.add_parser("download", help="Download model resources from configuration")
    d.add_argument("config")
    d.add_argument("--force", action="store_true")
    d.add_argument("--synthetic", action="store_true", help="write random-init model packs (no network)")
    d.set_defaults(func=cmd_download)
    v = sub.add_parser("validate", help="Validate configuration file")
    v.add_argument("config")
    v.add_argument("--strict", action="store_true", default=True)
    v.add_argument("--schema-only", action="store_false", dest="strict")
    v.set_defaults(func=cmd_validate)
    m = sub.add_parser("validate-model-info", help="Validate model_info.json file")
    m.add_argument("model_info")
    m.add_argument("--strict", action="store_true", default=True)
    m.add_argument("--schema-only", action="store_false", dest="strict")
    m.set_defaults(func=cmd_validate_model_info)
    ls = sub.add_parser("list", help="List cached models")
    ls.add_argument("cache_dir", nargs="?", default="~/.lumen/")
    ls.set_defaults(func=cmd_list)
    a = ap.parse_args(argv)
    if not a.command:
        ap.print_help()
        return 1
    return a.func(a)


if __name__ == "__main__":
    sys.exit(main())
