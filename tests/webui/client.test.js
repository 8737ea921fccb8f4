// DOM-less unit tests of the web UI core (lumen_amd/app/static/lumen.js) under Node.
// Run by tests/test_webui_cpu.py; exits non-zero on the first failed assertion.
"use strict";
const assert = require("assert");
const path = require("path");
const L = require(path.join(__dirname, "..", "..", "lumen_amd", "app", "static", "lumen.js"));

const tests = [];
const test = (name, fn) => tests.push([name, fn]);

// recording fetch: answers from `table[method + " " + url]` (or 200 {} by default)
function recorder(table) {
  const calls = [];
  const fetch = async (url, init) => {
    calls.push({ url, method: init.method, body: init.body === undefined ? undefined : JSON.parse(init.body), headers: init.headers });
    const hit = (table || {})[`${init.method} ${url}`];
    if (hit instanceof Error) throw hit;
    const r = hit || { status: 200, body: {} };
    const text = typeof r.body === "string" ? r.body : JSON.stringify(r.body);
    return { ok: r.status >= 200 && r.status < 300, status: r.status, statusText: r.statusText || "", text: async () => text };
  };
  return { fetch, calls };
}

test("every client method hits the documented route with the right verb and body", async () => {
  const rec = recorder();
  const api = L.createApi(rec.fetch, "http://h:1");
  const expect = [
    [() => api.health(), "GET", "/health"],
    [() => api.generateConfig({ preset: "cpu" }), "POST", "/api/v1/config/generate", { preset: "cpu" }],
    [() => api.currentConfig(), "GET", "/api/v1/config/current"],
    [() => api.loadConfig("/a b/lumen-config.yaml"), "POST", "/api/v1/config/load?config_path=%2Fa%20b%2Flumen-config.yaml"],
    [() => api.configYaml(), "GET", "/api/v1/config/yaml"],
    [() => api.validateConfig({ x: 1 }), "POST", "/api/v1/config/validate", { x: 1 }],
    [() => api.validatePath("~/.lumen"), "POST", "/api/v1/config/validate-path", { path: "~/.lumen" }],
    [() => api.hardwareInfo(), "GET", "/api/v1/hardware/info"],
    [() => api.presets(), "GET", "/api/v1/hardware/presets"],
    [() => api.checkPreset("amd mi355x"), "GET", "/api/v1/hardware/presets/amd%20mi355x/check"],
    [() => api.detect(), "POST", "/api/v1/hardware/detect"],
    [() => api.installStatus("~/.lumen"), "GET", "/api/v1/install/status?cache_dir=~%2F.lumen"],
    [() => api.checkPath("/p"), "GET", "/api/v1/install/check-path?path=%2Fp"],
    [() => api.startInstall({ preset: "cpu" }), "POST", "/api/v1/install/setup", { preset: "cpu" }],
    [() => api.installTasks(), "GET", "/api/v1/install/tasks"],
    [() => api.installTask("t/1"), "GET", "/api/v1/install/tasks/t%2F1"],
    [() => api.cancelInstall("t1"), "POST", "/api/v1/install/tasks/t1/cancel"],
    [() => api.installLogs("t1", 100), "GET", "/api/v1/install/tasks/t1/logs?tail=100"],
    [() => api.installLogs("t1"), "GET", "/api/v1/install/tasks/t1/logs"],
    [() => api.serverStatus(), "GET", "/api/v1/server/status"],
    [() => api.startServer({ port: 5 }), "POST", "/api/v1/server/start", { port: 5 }],
    [() => api.stopServer(), "POST", "/api/v1/server/stop", { force: false, timeout: 30 }],
    [() => api.restartServer({ force: true }), "POST", "/api/v1/server/restart", { force: true }],
    [() => api.serverLogs(), "GET", "/api/v1/server/logs?lines=200"],
    [() => api.serverLogs(50), "GET", "/api/v1/server/logs?lines=50"],
  ];
  for (const [fn, method, url, body] of expect) {
    await fn();
    const c = rec.calls[rec.calls.length - 1];
    assert.strictEqual(c.method, method, url);
    assert.strictEqual(c.url, "http://h:1" + url);
    assert.deepStrictEqual(c.body, body, url);
    assert.strictEqual(c.headers["Content-Type"], body === undefined ? undefined : "application/json", url);
  }
  // the method table covers the whole client (nothing added without a test)
  const methods = Object.keys(api).filter((k) => k !== "call");
  assert.strictEqual(new Set(expect.map(([fn]) => fn.toString().match(/api\.(\w+)/)[1])).size, methods.length);
});

test("errors map to kinds and FastAPI messages", async () => {
  const rec = recorder({
    "GET /api/v1/install/tasks/nope": { status: 404, body: { detail: "Task nope not found" } },
    "POST /api/v1/config/generate": { status: 422, body: { detail: [{ loc: ["body", "preset"], msg: "Field required", type: "missing" }] } },
    "GET /api/v1/server/status": { status: 503, statusText: "Service Unavailable", body: "" },
    "GET /api/v1/hardware/info": { status: 403, body: { message: "nope" } },
    "GET /api/v1/config/yaml": { status: 500, body: { detail: { message: "boom" } } },
    "GET /health": new TypeError("connection refused"),
  });
  const api = L.createApi(rec.fetch);
  const kinds = async (p) => { try { await p; } catch (e) { return e; } throw new Error("did not throw"); };
  let e = await kinds(api.installTask("nope"));
  assert.ok(e instanceof L.ApiError);
  assert.deepStrictEqual([e.kind, e.status, e.message], ["business", 404, "Task nope not found"]);
  e = await kinds(api.generateConfig({}));
  assert.deepStrictEqual([e.kind, e.message], ["business", "preset: Field required"]);
  e = await kinds(api.serverStatus());
  assert.deepStrictEqual([e.kind, e.message], ["server", "HTTP 503: Service Unavailable"]);
  e = await kinds(api.hardwareInfo());
  assert.deepStrictEqual([e.kind, e.message], ["permission", "nope"]);
  e = await kinds(api.configYaml());
  assert.deepStrictEqual([e.kind, e.message], ["server", "boom"]);
  e = await kinds(api.health());
  assert.strictEqual(e.kind, "network");
  assert.deepStrictEqual(L.describeUiError(e, "x").title, "Network error");
  assert.deepStrictEqual(L.describeUiError(new Error(""), "fallback"), { title: "Request failed", message: "fallback" });
  assert.deepStrictEqual(L.describeUiError("weird", "fallback"), { title: "Unknown error", message: "fallback" });
  assert.strictEqual(L.errorKind(302), "unknown");
});

test("204 and non-JSON bodies", async () => {
  const rec = recorder({ "GET /api/v1/server/status": { status: 204, body: "" }, "GET /api/v1/config/yaml": { status: 200, body: "plain" } });
  const api = L.createApi(rec.fetch);
  assert.strictEqual(await api.serverStatus(), undefined);
  assert.strictEqual(await api.configYaml(), "plain");
});

test("port and service-name validation (wizardValidation.ts rules)", () => {
  for (const [v, ok] of [["50051", true], [" 1024 ", true], ["65535", true], ["1023", false], ["65536", false], ["", false],
    ["80a", false], ["-1", false], ["5e4", false], [50051, true]]) {
    assert.strictEqual(L.portError(v) === null, ok, `port ${v}`);
  }
  for (const [v, ok] of [["lumen-ai", true], ["abc", true], ["ab", false], ["-abc", false], ["abc-", false], ["a_b_c", false],
    ["a".repeat(63), true], ["a".repeat(64), false], ["  lumen  ", true], ["", false]]) {
    assert.strictEqual(L.serviceNameError(v) === null, ok, `name ${v}`);
  }
  assert.ok(L.pathError("  "));
  assert.strictEqual(L.pathError("~/.lumen"), null);
});

test("wizard gate walks the steps in order", () => {
  const base = Object.assign({}, L.DEFAULT_WIZARD, { installPath: "/x" });
  assert.strictEqual(L.wizardGate(base, "welcome"), null);
  assert.strictEqual(L.wizardGate(base, "hardware"), null);
  assert.strictEqual(L.wizardGate(base, "config"), "/setup/hardware");
  assert.strictEqual(L.wizardGate(base, "install"), "/setup/hardware");
  assert.strictEqual(L.wizardGate(Object.assign({}, base, { port: 80 }), "hardware"), "/setup/welcome");
  assert.strictEqual(L.wizardGate(Object.assign({}, base, { installPath: "" }), "hardware"), "/setup/welcome");
  const hw = Object.assign({}, base, { hardwarePreset: "amd_mi355x" });
  assert.strictEqual(L.wizardGate(hw, "config"), null);
  assert.strictEqual(L.wizardGate(hw, "install"), "/setup/config");
  assert.strictEqual(L.wizardGate(Object.assign({}, hw, { configGenerated: true }), "install"), null);
  assert.strictEqual(L.wizardGate(hw, "bogus"), "/setup/welcome");
  assert.deepStrictEqual(L.WIZARD_STEPS.map((s) => s.id), ["welcome", "hardware", "config", "install"]);
});

test("config key changes with every generator input; request shape", () => {
  const s = Object.assign({}, L.DEFAULT_WIZARD, { installPath: "/x", hardwarePreset: "cpu", servicePreset: "basic" });
  const k = L.configKey(s);
  for (const patch of [{ region: "cn" }, { port: 50052 }, { serviceName: "other" }, { hardwarePreset: "amd_mi355x" },
    { servicePreset: "brave" }, { installPath: "/y" }, { clipModel: "MobileCLIP2-S4" }]) {
    assert.notStrictEqual(L.configKey(Object.assign({}, s, patch)), k, JSON.stringify(patch));
  }
  assert.deepStrictEqual(L.generateRequest(Object.assign({}, s, { port: "50052", serviceName: " svc " })),
    { cache_dir: "/x", preset: "cpu", region: "other", service_name: "svc", port: 50052, config_type: "basic", clip_model: null });
  // the clip models the UI offers are the ones the generator accepts (app/schemas.py ConfigRequest)
  assert.deepStrictEqual(L.SERVICE_PRESETS.find((p) => p.id === "light_weight").clipModels, ["MobileCLIP2-S2", "CN-CLIP_ViT-B-16"]);
  assert.deepStrictEqual(L.SERVICE_PRESETS.map((p) => p.id), ["minimal", "light_weight", "basic", "brave"]);
});

test("status helpers", () => {
  assert.ok(L.taskDone("completed") && L.taskDone("failed") && L.taskDone("cancelled"));
  assert.ok(!L.taskDone("running") && !L.taskDone("pending"));
  assert.strictEqual(L.statusKind("available"), "ok");
  assert.strictEqual(L.statusKind("missing"), "err");
  assert.strictEqual(L.statusKind("missing_drivers"), "warn");
  assert.strictEqual(L.statusKind("skipped"), "");
  assert.strictEqual(L.formatDuration(5), "5s");
  assert.strictEqual(L.formatDuration(125), "2m 5s");
  assert.strictEqual(L.formatDuration(3 * 3600 + 60), "3h 1m");
  assert.strictEqual(L.formatDuration(2 * 86400 + 3600), "2d 1h");
  assert.strictEqual(L.formatDuration(null), "—");
  assert.deepStrictEqual(L.appendBounded([1, 2, 3], [4, 5], 3), [3, 4, 5]);
  assert.strictEqual(L.wsUrl({ protocol: "https:", host: "a:1" }, "/ws/logs"), "wss://a:1/ws/logs");
  assert.strictEqual(L.wsUrl({ protocol: "http:", host: "a:1" }, "/ws/logs"), "ws://a:1/ws/logs");
});

test("persisted stores and recent paths", () => {
  const mem = {};
  const storage = { getItem: (k) => (k in mem ? mem[k] : null), setItem: (k, v) => { mem[k] = String(v); } };
  const a = L.createStore(storage, "w", { port: 1, x: null });
  a.set({ port: 2 });
  const b = L.createStore(storage, "w", { port: 1, x: null });
  assert.strictEqual(b.get("port"), 2);
  b.reset({ x: 3 });
  assert.deepStrictEqual(L.createStore(storage, "w", { port: 1 }).all(), { port: 1, x: 3 });
  mem.bad = "{not json";
  assert.deepStrictEqual(L.createStore(storage, "bad", { d: 1 }).all(), { d: 1 });
  let r = L.rememberPath([], " /a ");
  r = L.rememberPath(r, "/b");
  r = L.rememberPath(r, "/a");
  assert.deepStrictEqual(r, ["/a", "/b"]);
  assert.strictEqual(L.rememberPath(["1", "2", "3"], "4", 3).length, 3);
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try { await fn(); console.log(`ok - ${name}`); } catch (e) { failed++; console.log(`not ok - ${name}\n${e.stack}`); }
  }
  console.log(`${tests.length - failed}/${tests.length} passed`);
  process.exit(failed ? 1 : 0);
})();
