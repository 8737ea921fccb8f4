// The web UI's wizard flow, driven through the real API client (lumen.js) against a live
// control-plane server: node tests/webui/flow.test.js <base-url> <scratch-dir>.
// tests/test_webui_cpu.py starts the server (uvicorn on 127.0.0.1, install build step stubbed)
// and runs this.  Follows the same calls, in the same order, as the views in app.js:
// OpenPath -> Welcome -> Hardware -> Config -> Install -> Server.
"use strict";
const assert = require("assert");
const http = require("http");
const path = require("path");
const L = require(path.join(__dirname, "..", "..", "lumen_amd", "app", "static", "lumen.js"));

const [base, dir] = process.argv.slice(2);

// minimal fetch over node's http module (the Node in the image predates global fetch)
function fetch(url, init) {
  return new Promise((resolve, reject) => {
    const req = http.request(url, { method: init.method, headers: init.headers }, (res) => {
      const chunks = [];
      res.on("data", (c) => chunks.push(c));
      res.on("end", () => {
        const body = Buffer.concat(chunks).toString("utf8");
        resolve({ ok: res.statusCode >= 200 && res.statusCode < 300, status: res.statusCode, statusText: res.statusMessage,
          text: async () => body });
      });
    });
    req.on("error", reject);
    if (init.body !== undefined) req.write(init.body);
    req.end();
  });
}

const sleep = (ms) => new Promise((r) => setTimeout(r, ms));

(async () => {
  const api = L.createApi(fetch, base);
  assert.strictEqual((await api.health()).status, "ok");

  // OpenPath: a fresh directory validates and has no installation yet
  const v = await api.validatePath(dir);
  assert.ok(v.writable && !v.error, JSON.stringify(v));
  const cp = await api.checkPath(dir);
  assert.strictEqual(cp.has_existing_service, false);
  assert.strictEqual(cp.recommended_action, "configure_new");

  // Welcome: basics validate with the UI's rules
  const w = Object.assign({}, L.DEFAULT_WIZARD, { installPath: dir, port: 50777, serviceName: "lumen-ui-test" });
  assert.strictEqual(L.wizardGate(w, "hardware"), null);

  // Hardware: the preset list, a driver check, detection
  const info = await api.hardwareInfo();
  assert.ok(info.presets.length >= 2 && info.recommended_preset);
  const presets = await api.presets();
  assert.ok(presets.some((p) => p.name === "cpu"));
  const drivers = await api.checkPreset("cpu");
  assert.ok(Array.isArray(drivers));
  const det = await api.detect();
  assert.ok(det.recommended_preset);
  w.hardwarePreset = "cpu";
  assert.strictEqual(L.wizardGate(w, "config"), null);
  assert.strictEqual(L.wizardGate(w, "install"), "/setup/config");

  // Config: generate with the light profile + a CLIP model, read back YAML, validate
  w.servicePreset = "light_weight";
  w.clipModel = "MobileCLIP2-S2";
  const g = await api.generateConfig(L.generateRequest(w));
  assert.ok(g.success && g.config_path.endsWith("lumen-config.yaml"), JSON.stringify(g));
  assert.strictEqual(g.config_content.server.port, 50777);
  assert.ok(["ocr", "clip", "face"].every((s) => s in g.config_content.services));
  const y = await api.configYaml();
  assert.ok(y.loaded && y.yaml.indexOf("services:") >= 0 && y.yaml.indexOf("50777") >= 0);
  const cur = await api.currentConfig();
  assert.ok(cur.loaded && cur.port === 50777 && cur.service_name === "lumen-ui-test");
  assert.strictEqual((await api.validateConfig(g.config_content)).valid, true);
  const bad = await api.validateConfig({ metadata: {} });
  assert.ok(!bad.valid && bad.errors.length);
  w.configGenerated = true;
  assert.strictEqual(L.wizardGate(w, "install"), null);

  // business errors surface as ApiError(kind=business) with the server's detail
  try { await api.generateConfig(Object.assign(L.generateRequest(w), { preset: "no-such-preset" })); assert.fail("accepted"); } catch (e) {
    assert.ok(e instanceof L.ApiError && e.kind === "business" && e.status === 400 && /no-such-preset/.test(e.message), e.message);
  }
  try { await api.installTask("no-such-task"); assert.fail("found"); } catch (e) {
    assert.ok(e instanceof L.ApiError && e.status === 404, e.message);
  }

  // Install: start, follow to completion, logs, task list, cancel after completion is a no-op
  const st = await api.installStatus(dir);
  assert.ok(Array.isArray(st.missing_components));
  const t0 = await api.startInstall({ preset: "cpu", cache_dir: dir, environment_name: "lumen_env", force_reinstall: false, env_kind: "current" });
  let t = t0;
  for (let i = 0; i < 400 && !L.taskDone(t.status); i++) { await sleep(50); t = await api.installTask(t0.task_id); }
  assert.strictEqual(t.status, "completed", JSON.stringify(t));
  assert.strictEqual(t.progress, 100);
  const logs = await api.installLogs(t0.task_id, 100);
  assert.ok(logs.total_lines >= 3 && logs.logs.length >= 1);
  assert.ok((await api.installTasks()).tasks.some((x) => x.task_id === t0.task_id));
  assert.strictEqual((await api.cancelInstall(t0.task_id)).status, "completed");

  // Finish: load the generated config; SessionHub now sees an installation
  const ld = await api.loadConfig(g.config_path);
  assert.ok(ld.loaded && ld.port === 50777);
  const cp2 = await api.checkPath(dir);
  assert.ok(cp2.service_status.config, JSON.stringify(cp2));

  // Server view: status + logs endpoints answer; starting without models fails cleanly or starts
  const s = await api.serverStatus();
  assert.strictEqual(s.running, false);
  assert.ok(Array.isArray((await api.serverLogs(10)).logs));
  const stopped = await api.stopServer({ force: true, timeout: 5 });
  assert.strictEqual(stopped.running, false);
  console.log("flow ok");
})().catch((e) => { console.log(e.stack || String(e)); process.exit(1); });
