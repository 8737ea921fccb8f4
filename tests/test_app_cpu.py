"""Control plane (FastAPI TestClient): every SURVEY §A.1 endpoint path and response shape."""
import os
import time

import pytest
import yaml
from fastapi.testclient import TestClient

from lumen_amd.app import create_app
from lumen_amd.app.install import InstallOrchestrator


@pytest.fixture()
def client():
    app = create_app()
    with TestClient(app) as c:
        yield c
    app.state.lumen.server.stop(force=True, timeout=5)


def test_health_and_spa(client):
    assert client.get("/health").json() == {"status": "ok", "version": "0.1.0"}
    r = client.get("/some/ui/route")
    assert r.status_code == 200 and "Lumen" in r.text
    assert client.get("/api/v1/nope").status_code == 404


@pytest.mark.parametrize("ctype", ["minimal", "light_weight", "basic", "brave"])
def test_config_generate_current_yaml_load(client, tmp_path, ctype):
    r = client.post("/api/v1/config/generate", json={"cache_dir": str(tmp_path), "preset": "amd_mi355x",
                                                      "config_type": ctype, "port": 50999})
    assert r.status_code == 200, r.text
    d = r.json()
    assert d["success"] and d["config_path"].endswith("lumen-config.yaml")
    cfg = yaml.safe_load(open(d["config_path"]))
    assert cfg["server"]["port"] == 50999 and "ocr" in cfg["services"]
    if ctype == "brave":
        assert cfg["services"]["clip"]["import_info"]["registry_class"].endswith("BioCLIPService")
    cur = client.get("/api/v1/config/current").json()
    assert cur["loaded"] and cur["port"] == 50999 and cur["device"]["runtime"] == "torch"
    y = client.get("/api/v1/config/yaml").json()
    assert y["loaded"] and "services:" in y["yaml"]
    ld = client.post("/api/v1/config/load", params={"config_path": d["config_path"]}).json()
    assert ld["loaded"] and ld["service_name"] == "lumen-ai"
    assert client.post("/api/v1/config/validate", json=cfg).json()["valid"]
    assert client.post("/api/v1/config/generate", json={"preset": "nope"}).status_code == 400


def test_config_validate_and_paths(client, tmp_path):
    bad = client.post("/api/v1/config/validate", json={"metadata": {}}).json()
    assert bad["valid"] is False and bad["errors"]
    v = client.post("/api/v1/config/validate-path", json={"path": str(tmp_path / "new")}).json()
    assert set(v) >= {"valid", "exists", "writable", "free_space_gb", "error", "warning"} and v["writable"]
    assert client.post("/api/v1/config/validate-path", json={"path": ""}).json()["valid"] is False
    assert client.post("/api/v1/config/load", params={"config_path": str(tmp_path / "x.yaml")}).status_code == 404


def test_hardware(client):
    info = client.get("/api/v1/hardware/info").json()
    assert info["platform"] and info["recommended_preset"] and info["presets"]
    pres = client.get("/api/v1/hardware/presets").json()
    names = [p["name"] for p in pres]
    assert names[0] == "amd_mi355x" and "cpu" in names and "nvidia_gpu" in names
    chk = client.get("/api/v1/hardware/presets/amd_mi355x/check").json()
    assert {c["name"] for c in chk} == {"rocm", "hip_runtime", "lumen_native"}
    assert client.get("/api/v1/hardware/presets/zzz/check").status_code == 404
    det = client.post("/api/v1/hardware/detect").json()
    assert det["recommended_preset"] and det["detailed_status"]


def test_install_tasks(client, tmp_path, monkeypatch):
    monkeypatch.setattr(InstallOrchestrator, "_do_build_native",
                        lambda self, t, i: self._step(t, i, "skipped", "prebuilt"))
    monkeypatch.setattr(InstallOrchestrator, "_do_verify_installation",
                        lambda self, t, i: self._step(t, i, "completed", "verified (stub)"))
    st = client.get("/api/v1/install/status", params={"cache_dir": str(tmp_path)}).json()
    assert "missing_components" in st and "drivers" in st
    cp = client.get("/api/v1/install/check-path", params={"path": str(tmp_path)}).json()
    assert cp["recommended_action"] in ("configure_new", "repair", "start_existing")
    r = client.post("/api/v1/install/setup", json={"preset": "cpu", "cache_dir": str(tmp_path / "c")}).json()
    tid = r["task_id"]
    for _ in range(600):
        t = client.get(f"/api/v1/install/tasks/{tid}").json()
        if t["status"] in ("completed", "failed"):
            break
        time.sleep(0.05)
    assert t["status"] == "completed", t
    assert [s["step_id"] for s in t["steps"]] == ["check_python", "build_native", "verify_installation",
                                                  "prepare_cache"]
    assert [s["status"] for s in t["steps"]] == ["completed", "skipped", "completed", "completed"]
    assert (tmp_path / "c" / "models").is_dir()
    assert client.get("/api/v1/install/tasks").json()["total"] == 1
    logs = client.get(f"/api/v1/install/tasks/{tid}/logs", params={"tail": 10}).json()
    assert logs["total_lines"] >= 3
    assert client.post(f"/api/v1/install/tasks/{tid}/cancel").json()["status"] == "completed"
    assert client.post("/api/v1/install/setup", json={"preset": "bogus"}).status_code == 400
    with client.websocket_connect(f"/ws/install/{tid}") as ws:
        msgs = [ws.receive_json(), ws.receive_json()]
    assert msgs[0]["type"] == "status" and msgs[1]["type"] == "complete"


def test_server_lifecycle(client, tmp_path):
    from lumen_amd.resources.synthetic import write_clip_model

    s = client.get("/api/v1/server/status").json()
    assert s["running"] is False
    assert client.post("/api/v1/server/start", json={}).status_code == 400
    write_clip_model(tmp_path / "models" / "clip-tiny", "clip-tiny", preset="tiny", dataset=None)
    cfg = {"metadata": {"version": "1.0.0", "region": "other", "cache_dir": str(tmp_path)},
           "deployment": {"mode": "hub", "services": ["clip"]},
           "server": {"port": 50611, "host": "127.0.0.1"},
           "services": {"clip": {"enabled": True, "package": "lumen_clip",
                                 "import_info": {"registry_class": "lumen_clip.general_clip.clip_service.GeneralCLIPService",
                                                 "add_to_server": "lumen_clip.proto.ml_service_pb2_grpc.add_InferenceServicer_to_server"},
                                 "backend_settings": {"device": "cpu"},
                                 "models": {"general": {"model": "clip-tiny", "runtime": "torch"}}}}}
    p = tmp_path / "lumen-config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = client.post("/api/v1/server/start", json={"config_path": str(p)})
    assert r.status_code == 200 and r.json()["running"] and r.json()["pid"]
    healthy = False
    for _ in range(150):
        if client.get("/api/v1/server/status").json()["health"] == "healthy":
            healthy = True
            break
        time.sleep(0.2)
    logs = client.get("/api/v1/server/logs", params={"lines": 50}).json()
    assert healthy, logs
    assert logs["total_lines"] >= 1 and logs["logs"][0].startswith("[lumen-app] starting")
    assert client.post("/api/v1/server/start", json={"config_path": str(p)}).status_code == 409
    r = client.post("/api/v1/server/restart", json={"config_path": str(p), "timeout": 10}).json()
    assert r["running"]
    r = client.post("/api/v1/server/stop", json={"timeout": 10}).json()
    assert r["running"] is False
    with client.websocket_connect("/ws/logs") as ws:
        assert ws.receive_json()["type"] == "connected"


def test_spa_assets_and_api_coverage(client):
    """The web UI (static/index.html + app.js + app.css) is served, parses, and every
    /api/v1 path it calls is a route of the control-plane app (reference UI views:
    lumen-app/web-ui/src/views/*.tsx, API client lib/api.ts)."""
    import re
    import shutil
    import subprocess
    from pathlib import Path

    from lumen_amd.app.main import STATIC_DIR

    idx = client.get("/")
    assert idx.status_code == 200 and 'src="/app.js"' in idx.text
    for route in ("#/open", "#/session", "#/server", "#/setup/welcome", "#/setup/hardware", "#/setup/config",
                  "#/setup/install"):
        assert route in idx.text
    js = client.get("/app.js")
    assert js.status_code == 200 and "views[\"/setup/install\"]" in js.text
    core = client.get("/lumen.js")
    assert core.status_code == 200
    assert client.get("/app.css").status_code == 200
    if shutil.which("node"):
        for f in ("app.js", "lumen.js"):
            r = subprocess.run(["node", "--check", str(Path(STATIC_DIR) / f)], capture_output=True, text=True)
            assert r.returncode == 0, r.stderr
    # every call("...") path of the UI's API client resolves to a registered route
    routes = list(client.get("/openapi.json").json()["paths"])
    pats = [re.compile("^" + re.sub(r"\{[^}]+\}", "[^/]+", p) + "$") for p in routes]
    used = set(re.findall(r'call\(\s*[`"]([a-z][^`"?]*)', core.text))
    assert len(used) >= 15, used
    for u in used:
        full = "/api/v1/" + u.split("${")[0].rstrip("/")
        if "${" in u:   # templated segment: compare with a placeholder id
            full = "/api/v1/" + re.sub(r"\$\{[^}]+\}", "x", u)
        assert any(p.match(full) for p in pats), f"UI calls {full}, no such route"
    for ws in ("/ws/logs", "/ws/install/"):
        assert ws in js.text


# ----------------------------------------------------------------------------- download integrity
class _Resp:
    def __init__(self, data: bytes):
        import io

        self._b = io.BytesIO(data)

    def read(self, n=-1):
        return self._b.read(n)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _fake_urlopen(table):
    def urlopen(url, timeout=None):
        url = getattr(url, "full_url", url)
        if url not in table:
            raise OSError(f"404 {url}")
        return _Resp(table[url])
    return urlopen


def test_micromamba_mirrors_and_checksum(tmp_path, monkeypatch):
    import hashlib

    from lumen_amd.app.installation import micromamba as mm

    assert all("proxy" not in m for m in mm.mirrors_for("other"))
    assert any(m.startswith("https://gh-proxy.org/") for m in mm.mirrors_for("cn"))
    payload = b"#!/bin/sh\necho 2.0.0\n"
    url = mm.RELEASE.format(plat=mm.platform_tag())
    digest = hashlib.sha256(payload).hexdigest()
    inst = mm.MicromambaInstaller(tmp_path)
    # wrong published digest: the binary is never put in place
    monkeypatch.setattr(mm.urllib.request, "urlopen", _fake_urlopen({url: payload, url + ".sha256": b"0" * 64}))
    with pytest.raises(RuntimeError, match="mismatch"):
        inst._fetch(url)
    assert not inst.local_path.exists()
    # no sidecar: refused
    monkeypatch.setattr(mm.urllib.request, "urlopen", _fake_urlopen({url: payload}))
    with pytest.raises(OSError):
        inst._fetch(url)
    assert not inst.local_path.exists()
    # matching digest: installed and executable
    monkeypatch.setattr(mm.urllib.request, "urlopen",
                        _fake_urlopen({url: payload, url + ".sha256": f"{digest}  micromamba".encode()}))
    inst.local_path.parent.mkdir(parents=True, exist_ok=True)
    inst._fetch(url)
    assert inst.local_path.read_bytes() == payload and os.access(inst.local_path, os.X_OK)


def test_release_wheel_download_requires_matching_digest(tmp_path, monkeypatch):
    import hashlib

    from lumen_amd.app.installation import package_resolver as pr

    data = b"PK\x03\x04 not really a wheel"
    url = "https://github.com/o/r/releases/download/v1/lumen_amd-1.0-py3-none-any.whl"
    res = pr.LumenPackageResolver(tmp_path, region="other")
    monkeypatch.setattr(pr.urllib.request, "urlopen", _fake_urlopen({url: data}))
    with pytest.raises(RuntimeError, match="no SHA-256"):
        res.download(pr.PackageSource("release", url, "v1"))
    with pytest.raises(RuntimeError, match="mismatch"):
        res.download(pr.PackageSource("release", url, "v1", sha256="ab" * 32))
    assert not (tmp_path / "wheels" / url.rsplit("/", 1)[-1]).exists()
    got = res.download(pr.PackageSource("release", url, "v1", sha256=hashlib.sha256(data).hexdigest()))
    assert got.kind == "wheel" and open(got.location, "rb").read() == data
    # the asset digest field of the GitHub API is picked up
    assert res._asset_digest({"name": "x.whl", "digest": "sha256:" + "cd" * 32}, []) == "cd" * 32
