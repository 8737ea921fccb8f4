"""lumen-resources CLI and console entry points."""
import json

import yaml

from lumen_amd import cli
from lumen_amd.resources import cli as rcli


def _cfg(tmp_path):
    return {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(tmp_path)},
            "deployment": {"mode": "hub", "services": ["ocr", "face"]},
            "server": {"port": 50621, "host": "127.0.0.1"},
            "services": {
                "ocr": {"enabled": True, "package": "lumen_ocr",
                        "import_info": {"registry_class": "lumen_ocr.general_ocr.GeneralOcrService",
                                        "add_to_server": "lumen_ocr.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                        "models": {"general": {"model": "ppocr-tiny", "runtime": "onnx"}}},
                "face": {"enabled": True, "package": "lumen_face",
                         "import_info": {"registry_class": "lumen_face.general_face.GeneralFaceService",
                                         "add_to_server": "lumen_face.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                         "models": {"general": {"model": "buffalo_tiny", "runtime": "onnx"}}}}}


def test_resources_cli(tmp_path, capsys):
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(_cfg(tmp_path)))
    assert rcli.main(["validate", str(p)]) == 0
    assert rcli.main(["download", str(p), "--synthetic"]) == 0
    out = capsys.readouterr().out
    assert "2/2 models ready" in out
    mi = tmp_path / "models" / "ppocr-tiny" / "model_info.json"
    assert rcli.main(["validate-model-info", str(mi)]) == 0
    assert rcli.main(["list", str(tmp_path)]) == 0
    out = capsys.readouterr().out
    assert "ppocr-tiny" in out and "buffalo_tiny" in out
    bad = tmp_path / "bad.yaml"
    bad.write_text("metadata: {}\n")
    assert rcli.main(["validate", str(bad)]) == 1
    (tmp_path / "bad_info.json").write_text(json.dumps({"name": "x"}))
    assert rcli.main(["validate-model-info", str(tmp_path / "bad_info.json")]) == 1


def test_entry_points_exist():
    for f in (cli.lumen, cli.clip, cli.face, cli.ocr, cli.vlm, cli.resources, cli.app):
        assert callable(f)
    from pathlib import Path

    text = (Path(__file__).resolve().parents[1] / "pyproject.toml").read_text()
    for name in ("lumen", "lumen-clip", "lumen-face", "lumen-ocr", "lumen-vlm", "lumen-resources", "lumen-app"):
        assert f'\n{name} = "lumen_amd.cli:' in text
