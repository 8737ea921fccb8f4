// Lumen control-plane SPA (plain ES2020, no build step).
//
// Same flows as the reference web UI (lumen-app/web-ui/src: App.tsx routes, views/*.tsx,
// context/WizardProvider.tsx, hooks/useLumenSession.ts, lib/api.ts): pick a cache
// directory, resume an existing install or walk the setup wizard (welcome -> hardware
// preset -> generated config -> native setup task), then start/stop the hub server and
// follow its logs.  Talks only to the /api/v1 endpoints of lumen_amd.app.main and the
// /ws/logs, /ws/install/{id} websockets.
"use strict";

// ------------------------------------------------------------------ api client (lib/api.ts)
const API = "/api/v1";

async function api(path, opts = {}) {
  const init = { method: opts.method || "GET", headers: {} };
  if (opts.body !== undefined) {
    init.headers["Content-Type"] = "application/json";
    init.body = JSON.stringify(opts.body);
  }
  const r = await fetch(path.startsWith("/") ? path : `${API}/${path}`, init);
  let data = null;
  const text = await r.text();
  try { data = text ? JSON.parse(text) : null; } catch { data = text; }
  if (!r.ok) {
    const detail = data && data.detail ? (typeof data.detail === "string" ? data.detail : JSON.stringify(data.detail)) : r.statusText;
    const e = new Error(`${r.status}: ${detail}`);
    e.status = r.status;
    throw e;
  }
  return data;
}

const qs = (o) => new URLSearchParams(o).toString();
const Api = {
  health: () => api("/health"),
  generateConfig: (req) => api("config/generate", { method: "POST", body: req }),
  currentConfig: () => api("config/current"),
  loadConfig: (p) => api(`config/load?${qs({ config_path: p })}`, { method: "POST" }),
  configYaml: () => api("config/yaml"),
  validateConfig: (cfg) => api("config/validate", { method: "POST", body: cfg }),
  validatePath: (p) => api("config/validate-path", { method: "POST", body: { path: p } }),
  hardwareInfo: () => api("hardware/info"),
  presets: () => api("hardware/presets"),
  checkPreset: (n) => api(`hardware/presets/${encodeURIComponent(n)}/check`),
  detect: () => api("hardware/detect", { method: "POST" }),
  installStatus: (cacheDir) => api(`install/status?${qs({ cache_dir: cacheDir })}`),
  checkPath: (p) => api(`install/check-path?${qs({ path: p })}`),
  startInstall: (req) => api("install/setup", { method: "POST", body: req }),
  installTasks: () => api("install/tasks"),
  installTask: (id) => api(`install/tasks/${id}`),
  cancelInstall: (id) => api(`install/tasks/${id}/cancel`, { method: "POST" }),
  installLogs: (id) => api(`install/tasks/${id}/logs`),
  serverStatus: () => api("server/status"),
  startServer: (req) => api("server/start", { method: "POST", body: req }),
  stopServer: (req) => api("server/stop", { method: "POST", body: req || { force: false, timeout: 30 } }),
  restartServer: (req) => api("server/restart", { method: "POST", body: req }),
  serverLogs: (n) => api(`server/logs?${qs({ lines: n || 200 })}`),
};

// ------------------------------------------------------------------ session + wizard state
const Session = {
  get path() { return localStorage.getItem("lumen.session.path") || ""; },
  set path(p) { p ? localStorage.setItem("lumen.session.path", p) : localStorage.removeItem("lumen.session.path"); },
};
const Wizard = {
  _s: JSON.parse(sessionStorage.getItem("lumen.wizard") || "{}"),
  get(k, d) { return this._s[k] !== undefined ? this._s[k] : d; },
  set(k, v) { this._s[k] = v; sessionStorage.setItem("lumen.wizard", JSON.stringify(this._s)); },
  reset() { this._s = {}; sessionStorage.removeItem("lumen.wizard"); },
};
const STEPS = [["welcome", "Welcome"], ["hardware", "Hardware"], ["config", "Config"], ["install", "Install"]];

// ------------------------------------------------------------------ tiny DOM helpers
function h(tag, attrs = {}, ...kids) {
  const el = document.createElement(tag);
  for (const [k, v] of Object.entries(attrs || {})) {
    if (k === "class") el.className = v;
    else if (k.startsWith("on")) el.addEventListener(k.slice(2), v);
    else if (v === true) el.setAttribute(k, "");
    else if (v !== false && v != null) el.setAttribute(k, v);
  }
  for (const c of kids.flat()) if (c != null && c !== false) el.append(c instanceof Node ? c : document.createTextNode(String(c)));
  return el;
}
const $ = (id) => document.getElementById(id);
function toast(msg, ms = 3500) {
  const t = $("toast");
  t.textContent = msg;
  t.classList.remove("hidden");
  clearTimeout(toast._t);
  toast._t = setTimeout(() => t.classList.add("hidden"), ms);
}
const badge = (text, kind) => h("span", { class: `badge ${kind || ""}` }, text);
const alertBox = (text, kind) => h("div", { class: `alert ${kind || ""}` }, text);
const card = (title, ...kids) => h("div", { class: "card" }, title ? h("h2", {}, title) : null, ...kids);
const skeleton = (n = 3) => Array.from({ length: n }, () => h("div", { class: "skeleton" }));
function debounce(fn, ms) { let t; return (...a) => { clearTimeout(t); t = setTimeout(() => fn(...a), ms); }; }

// cleanup hooks for the current view (websockets, intervals)
let cleanups = [];
function onLeave(fn) { cleanups.push(fn); }

// ------------------------------------------------------------------ views
const views = {};

views["/open"] = async (root) => {
  $("title").textContent = "Open a Lumen directory";
  const input = h("input", { placeholder: "~/.lumen", value: Session.path || "~/.lumen" });
  const status = h("div");
  const openBtn = h("button", { disabled: true }, "Open");
  const check = debounce(async () => {
    status.replaceChildren(...skeleton(1));
    try {
      const r = await Api.validatePath(input.value.trim());
      const kids = [];
      if (r.error) kids.push(alertBox(r.error, "err"));
      if (r.warning) kids.push(alertBox(r.warning, "warn"));
      kids.push(h("div", { class: "row" }, badge(r.exists ? "exists" : "will be created"),
        badge(r.writable ? "writable" : "not writable", r.writable ? "ok" : "err"),
        r.free_space_gb != null ? badge(`${r.free_space_gb} GB free`) : null));
      status.replaceChildren(...kids);
      openBtn.disabled = !r.writable;
    } catch (e) { status.replaceChildren(alertBox(e.message, "err")); openBtn.disabled = true; }
  }, 500);
  input.addEventListener("input", check);
  openBtn.addEventListener("click", async () => {
    const p = input.value.trim();
    Session.path = p;
    Wizard.reset();
    Wizard.set("cacheDir", p);
    refreshChrome();
    try {
      const r = await Api.checkPath(p);
      location.hash = r.has_existing_service ? "#/session" : "#/setup/welcome";
    } catch (e) { toast(e.message); location.hash = "#/setup/welcome"; }
  });
  root.append(card("Lumen directory",
    h("p", { class: "muted" }, "Models, label banks, the generated lumen-config.yaml and logs live here."),
    h("label", {}, "Path"), input, status, h("div", { class: "row", style: "margin-top:12px" }, openBtn)));
  check();
};

views["/session"] = async (root) => {
  $("title").textContent = "Session";
  const p = Session.path;
  const body = h("div", {}, ...skeleton(4));
  root.append(card(`Installation at ${p}`, body));
  try {
    const r = await Api.checkPath(p);
    const s = r.service_status;
    const rows = [["configuration (lumen-config.yaml)", s.config], ["native runtime built", s.environment], ["drivers", s.drivers]]
      .map(([k, v]) => h("tr", {}, h("td", {}, k), h("td", {}, badge(v ? "ok" : "missing", v ? "ok" : "warn"))));
    const actions = h("div", { class: "row", style: "margin-top:12px" });
    const startExisting = h("button", {
      onclick: async () => {
        try {
          await Api.loadConfig(`${p.replace(/\/$/, "")}/lumen-config.yaml`);
          location.hash = "#/server";
        } catch (e) { toast(e.message); }
      },
    }, "Use existing configuration");
    if (r.has_existing_service) actions.append(startExisting);
    actions.append(h("button", { class: "secondary", onclick: () => { Wizard.reset(); Wizard.set("cacheDir", p); location.hash = "#/setup/welcome"; } }, "Configure new"));
    if (r.recommended_action === "repair") actions.append(h("button", { class: "secondary", onclick: () => (location.hash = "#/setup/install") }, "Repair"));
    body.replaceChildren(alertBox(r.message, r.ready_to_start ? "ok" : "warn"), h("table", {}, ...rows),
      h("p", { class: "muted" }, `recommended: ${r.recommended_action.replace("_", " ")}`), actions);
  } catch (e) { body.replaceChildren(alertBox(e.message, "err")); }
};

views["/setup/welcome"] = async (root) => {
  $("title").textContent = "Setup";
  root.append(card("Welcome",
    h("p", {}, "This wizard prepares a Lumen hub on this machine in four steps:"),
    h("ol", {},
      h("li", {}, "pick a hardware preset (AMD MI355X / ROCm, or CPU),"),
      h("li", {}, "generate lumen-config.yaml (services, models, batch sizes),"),
      h("li", {}, "build the native gfx950 kernels and fetch models,"),
      h("li", {}, "start the gRPC hub and watch its logs.")),
    h("p", { class: "muted" }, `Directory: ${Session.path}`),
    h("div", { class: "row" }, h("button", { onclick: () => (location.hash = "#/setup/hardware") }, "Start"))));
};

views["/setup/hardware"] = async (root) => {
  $("title").textContent = "Hardware";
  const sys = h("div", {}, ...skeleton(3));
  const list = h("div", { class: "grid" }, ...skeleton(4));
  const drivers = h("div");
  const next = h("button", { disabled: !Wizard.get("preset") }, "Next: configuration");
  next.addEventListener("click", () => (location.hash = "#/setup/config"));
  const detectBtn = h("button", { class: "secondary" }, "Detect");
  root.append(card("This machine", sys), card("Presets", h("div", { class: "row", style: "margin-bottom:10px" }, detectBtn), list, drivers),
    h("div", { class: "row" }, h("button", { class: "ghost", onclick: () => (location.hash = "#/setup/welcome") }, "Back"), next));

  const select = async (name) => {
    Wizard.set("preset", name);
    next.disabled = false;
    list.querySelectorAll(".preset").forEach((c) => c.classList.toggle("selected", c.dataset.name === name));
    drivers.replaceChildren(...skeleton(2));
    try {
      const ds = await Api.checkPreset(name);
      drivers.replaceChildren(h("h3", {}, `Drivers for ${name}`), h("table", {}, ...ds.map((d) =>
        h("tr", {}, h("td", {}, d.name), h("td", {}, badge(d.status, d.status === "available" ? "ok" : "warn")), h("td", { class: "muted" }, d.details)))));
    } catch (e) { drivers.replaceChildren(alertBox(e.message, "err")); }
  };
  try {
    const info = await Api.hardwareInfo();
    const gpus = (info.gpus || []).map((g) => h("li", {}, Object.entries(g).map(([k, v]) => `${k}: ${v}`).join(" · ")));
    sys.replaceChildren(h("table", {},
      h("tr", {}, h("td", {}, "platform"), h("td", {}, `${info.platform} ${info.machine}`)),
      h("tr", {}, h("td", {}, "processor"), h("td", {}, info.processor || "—")),
      h("tr", {}, h("td", {}, "python"), h("td", {}, info.python_version)),
      h("tr", {}, h("td", {}, "recommended preset"), h("td", {}, badge(info.recommended_preset || "cpu", "ok")))),
      gpus.length ? h("ul", {}, gpus) : h("p", { class: "muted" }, "no AMD GPU detected"));
    const cur = Wizard.get("preset", info.recommended_preset);
    list.replaceChildren(...info.presets.map((p) => {
      const c = h("div", { class: "card preset", "data-name": p.name },
        h("h3", {}, p.name), h("div", { class: "muted" }, p.description),
        h("div", { class: "row", style: "margin-top:6px" }, badge(p.runtime), badge(p.availability.replace("_", " "),
          p.ready ? "ok" : p.availability === "not_checked" ? "" : "warn"),
          p.supported_on_current_platform ? null : badge("unsupported OS", "err")));
      c.addEventListener("click", () => select(p.name));
      return c;
    }));
    if (cur) select(cur);
  } catch (e) { sys.replaceChildren(alertBox(e.message, "err")); }
  detectBtn.addEventListener("click", async () => {
    detectBtn.disabled = true;
    try {
      const r = await Api.detect();
      toast(`recommended preset: ${r.recommended_preset}`);
      select(r.recommended_preset);
    } catch (e) { toast(e.message); }
    detectBtn.disabled = false;
  });
};

views["/setup/config"] = async (root) => {
  $("title").textContent = "Configuration";
  const preset = Wizard.get("preset");
  if (!preset) { location.hash = "#/setup/hardware"; return; }
  const f = (label, el) => h("div", {}, h("label", {}, label), el);
  const region = h("select", {}, h("option", { value: "other" }, "other"), h("option", { value: "cn" }, "cn"));
  region.value = Wizard.get("region", "other");
  const svc = h("input", { value: Wizard.get("serviceName", "lumen-ai") });
  const port = h("input", { type: "number", value: Wizard.get("port", 50051) });
  const ctype = h("select", {}, ...["minimal", "light_weight", "basic", "brave"].map((t) => h("option", { value: t }, t.replace("_", " "))));
  ctype.value = Wizard.get("configType", "minimal");
  const clip = h("select");
  const fillClip = () => {
    const opts = ctype.value === "light_weight" ? ["MobileCLIP2-S2", "CN-CLIP_ViT-B-16"] : ctype.value === "basic" ? ["MobileCLIP2-S4", "CN-CLIP_ViT-L-14"] : [];
    clip.replaceChildren(h("option", { value: "" }, opts.length ? "default for region" : "n/a"), ...opts.map((o) => h("option", { value: o }, o)));
    clip.disabled = !opts.length;
  };
  ctype.addEventListener("change", fillClip);
  fillClip();
  const out = h("div");
  const gen = h("button", {}, "Generate lumen-config.yaml");
  const next = h("button", { disabled: !Wizard.get("configGenerated") }, "Next: install");
  next.addEventListener("click", () => (location.hash = "#/setup/install"));
  const showYaml = async (warnings) => {
    const y = await Api.configYaml();
    const val = h("button", { class: "secondary" }, "Validate");
    val.addEventListener("click", async () => {
      try {
        const cur = Wizard.get("configContent");
        const r = await Api.validateConfig(cur || {});
        toast(r.valid ? "configuration is valid" : `invalid: ${r.errors.join("; ")}`);
      } catch (e) { toast(e.message); }
    });
    out.replaceChildren(...(warnings || []).map((w) => alertBox(w, "warn")), h("h3", {}, "lumen-config.yaml"), h("pre", {}, y.yaml || ""),
      h("div", { class: "row", style: "margin-top:8px" }, val));
  };
  gen.addEventListener("click", async () => {
    gen.disabled = true;
    Wizard.set("region", region.value); Wizard.set("serviceName", svc.value); Wizard.set("port", Number(port.value)); Wizard.set("configType", ctype.value);
    try {
      const r = await Api.generateConfig({ cache_dir: Session.path, preset, region: region.value, service_name: svc.value,
        port: Number(port.value) || 50051, config_type: ctype.value, clip_model: clip.value || null });
      Wizard.set("configGenerated", true); Wizard.set("configPath", r.config_path); Wizard.set("configContent", r.config_content);
      toast(r.message);
      next.disabled = false;
      await showYaml(r.warnings);
    } catch (e) { out.replaceChildren(alertBox(e.message, "err")); }
    gen.disabled = false;
  });
  root.append(card(`Configuration for preset ${preset}`,
    h("div", { class: "grid" }, f("Region (model mirrors)", region), f("Service name (mDNS)", svc), f("gRPC port", port), f("Profile", ctype), f("CLIP model", clip)),
    h("div", { class: "row", style: "margin-top:12px" }, gen)), out,
    h("div", { class: "row" }, h("button", { class: "ghost", onclick: () => (location.hash = "#/setup/hardware") }, "Back"), next));
  if (Wizard.get("configGenerated")) showYaml().catch(() => {});
};

views["/setup/install"] = async (root) => {
  $("title").textContent = "Install";
  const preset = Wizard.get("preset", "cpu");
  const status = h("div", {}, ...skeleton(3));
  const bar = h("div", { class: "progress" }, h("div", { style: "width:0%" }));
  const stepsTbl = h("table");
  const logs = h("pre", { class: "logs" });
  const startBtn = h("button", {}, "Run setup");
  const cancelBtn = h("button", { class: "secondary", disabled: true }, "Cancel");
  const toServer = h("button", { class: "hidden", onclick: () => (location.hash = "#/server") }, "Go to server");
  root.append(card("Environment", status),
    card("Setup task", h("div", { class: "row" }, startBtn, cancelBtn, toServer), h("div", { style: "margin:12px 0" }, bar), stepsTbl, h("h3", {}, "Logs"), logs));
  const loadStatus = async () => {
    try {
      const s = await Api.installStatus(Session.path);
      status.replaceChildren(h("table", {},
        h("tr", {}, h("td", {}, "native runtime"), h("td", {}, badge(s.environment_exists ? "built" : "not built", s.environment_exists ? "ok" : "warn"))),
        h("tr", {}, h("td", {}, "ready for preset"), h("td", {}, s.ready_for_preset || "—")),
        ...Object.entries(s.drivers || {}).map(([k, v]) => h("tr", {}, h("td", {}, `driver ${k}`), h("td", {}, badge(v, v === "available" ? "ok" : "warn"))))),
        s.missing_components.length ? alertBox(`missing: ${s.missing_components.join(", ")}`, "warn") : alertBox("all components present", "ok"));
    } catch (e) { status.replaceChildren(alertBox(e.message, "err")); }
  };
  const render = (t) => {
    bar.firstChild.style.width = `${t.progress}%`;
    stepsTbl.replaceChildren(...t.steps.map((s) => h("tr", {}, h("td", {}, s.name),
      h("td", {}, badge(s.status, s.status === "completed" ? "ok" : s.status === "failed" ? "err" : s.status === "running" ? "warn" : "")),
      h("td", { class: "muted" }, s.message))));
    const done = ["completed", "failed", "cancelled"].includes(t.status);
    cancelBtn.disabled = done;
    startBtn.disabled = !done;
    if (t.status === "completed") toServer.classList.remove("hidden");
    if (t.error) stepsTbl.append(h("tr", {}, h("td", { colspan: 3 }, alertBox(t.error, "err"))));
  };
  const follow = (id) => {
    Wizard.set("installTask", id);
    cancelBtn.onclick = async () => { try { render(await Api.cancelInstall(id)); } catch (e) { toast(e.message); } };
    const pullLogs = async () => { try { logs.textContent = (await Api.installLogs(id)).logs.join("\n"); logs.scrollTop = logs.scrollHeight; } catch { /* task gone */ } };
    const iv = setInterval(pullLogs, 1000);
    onLeave(() => clearInterval(iv));
    let ws;
    try {
      ws = new WebSocket(`${location.protocol === "https:" ? "wss" : "ws"}://${location.host}/ws/install/${id}`);
      ws.onmessage = (ev) => {
        const m = JSON.parse(ev.data);
        if (m.task) render(m.task);
        if (m.type === "complete" || m.type === "error") { pullLogs(); loadStatus(); clearInterval(iv); }
      };
      onLeave(() => ws.close());
    } catch {
      const pv = setInterval(async () => { try { render(await Api.installTask(id)); } catch { clearInterval(pv); } }, 1000);
      onLeave(() => clearInterval(pv));
    }
  };
  startBtn.addEventListener("click", async () => {
    startBtn.disabled = true;
    try {
      const t = await Api.startInstall({ preset, cache_dir: Session.path, environment_name: "lumen_env", force_reinstall: false });
      render(t);
      follow(t.task_id);
    } catch (e) { toast(e.message); startBtn.disabled = false; }
  });
  await loadStatus();
  const prev = Wizard.get("installTask");
  if (prev) {
    try { const t = await Api.installTask(prev); render(t); if (!["completed", "failed", "cancelled"].includes(t.status)) follow(prev); } catch { Wizard.set("installTask", null); }
  }
};

views["/server"] = async (root) => {
  $("title").textContent = "Server";
  const st = h("div", {}, ...skeleton(4));
  const logs = h("pre", { class: "logs" });
  const cfgPath = h("input", { placeholder: "lumen-config.yaml (defaults to the loaded configuration)" });
  const portIn = h("input", { type: "number", placeholder: "port (from config)" });
  const startB = h("button", {}, "Start");
  const stopB = h("button", { class: "secondary" }, "Stop");
  const restartB = h("button", { class: "secondary" }, "Restart");
  const forceStop = h("input", { type: "checkbox", style: "width:auto" });
  root.append(card("Hub server", st,
    h("div", { class: "grid", style: "margin-top:10px" }, h("div", {}, h("label", {}, "Config path"), cfgPath), h("div", {}, h("label", {}, "Port override"), portIn)),
    h("div", { class: "row", style: "margin-top:12px" }, startB, stopB, restartB, h("label", { style: "display:flex;gap:6px;align-items:center;margin:0" }, forceStop, "force"))),
    card("Logs", logs));
  const show = (s) => {
    st.replaceChildren(h("table", {},
      h("tr", {}, h("td", {}, "state"), h("td", {}, badge(s.running ? "running" : "stopped", s.running ? "ok" : ""))),
      h("tr", {}, h("td", {}, "health"), h("td", {}, badge(s.health, s.health === "healthy" ? "ok" : s.health === "unhealthy" ? "err" : ""))),
      h("tr", {}, h("td", {}, "pid"), h("td", {}, s.pid != null ? s.pid : "—")),
      h("tr", {}, h("td", {}, "address"), h("td", {}, `${s.host}:${s.port}`)),
      h("tr", {}, h("td", {}, "uptime"), h("td", {}, s.uptime_seconds != null ? `${Math.round(s.uptime_seconds)} s` : "—")),
      h("tr", {}, h("td", {}, "config"), h("td", {}, s.config_path || "—"))),
      s.last_error ? alertBox(s.last_error, "err") : null);
    startB.disabled = s.running;
    stopB.disabled = !s.running;
  };
  const poll = async () => { try { show(await Api.serverStatus()); } catch (e) { st.replaceChildren(alertBox(e.message, "err")); } };
  const body = () => ({ config_path: cfgPath.value.trim() || null, port: portIn.value ? Number(portIn.value) : null, environment: "lumen_env" });
  startB.addEventListener("click", async () => { try { show(await Api.startServer(body())); toast("server starting"); } catch (e) { toast(e.message); } });
  stopB.addEventListener("click", async () => { try { show(await Api.stopServer({ force: forceStop.checked, timeout: 30 })); } catch (e) { toast(e.message); } });
  restartB.addEventListener("click", async () => { try { show(await Api.restartServer({ ...body(), force: forceStop.checked, timeout: 30 })); } catch (e) { toast(e.message); } });
  try { const c = await Api.currentConfig(); if (c.loaded) cfgPath.placeholder = c.config_path; } catch { /* none loaded */ }
  await poll();
  const iv = setInterval(poll, 3000);
  onLeave(() => clearInterval(iv));
  try { logs.textContent = (await Api.serverLogs(200)).logs.join("\n"); } catch { /* no logs yet */ }
  try {
    const ws = new WebSocket(`${location.protocol === "https:" ? "wss" : "ws"}://${location.host}/ws/logs`);
    ws.onmessage = (ev) => {
      const m = JSON.parse(ev.data);
      if (m.type === "log") { logs.textContent += (logs.textContent ? "\n" : "") + m.message; logs.scrollTop = logs.scrollHeight; }
    };
    onLeave(() => ws.close());
  } catch { /* websocket unavailable: status polling still works */ }
};

// ------------------------------------------------------------------ router (App.tsx)
function refreshChrome() {
  const p = Session.path;
  $("session-path").textContent = p || "—";
  const route = location.hash.replace(/^#/, "") || "/open";
  document.querySelectorAll("#nav a").forEach((a) => {
    a.classList.toggle("active", a.dataset.route === route);
    a.classList.toggle("disabled", a.hasAttribute("data-needs-session") && !p);
  });
  const steps = $("steps");
  if (route.startsWith("/setup/")) {
    const cur = STEPS.findIndex(([k]) => route === `/setup/${k}`);
    steps.replaceChildren(...STEPS.map(([, label], i) => h("div", { class: `s ${i < cur ? "done" : i === cur ? "cur" : ""}` }, `${i + 1}. ${label}`)));
    steps.classList.remove("hidden");
  } else steps.classList.add("hidden");
}

async function route() {
  cleanups.forEach((f) => { try { f(); } catch { /* ignore */ } });
  cleanups = [];
  let r = location.hash.replace(/^#/, "") || "/open";
  if (r === "/" || r === "/setup") r = r === "/" ? "/open" : "/setup/welcome";
  if (!views[r]) { location.hash = "#/open"; return; }
  if (r !== "/open" && !Session.path) { location.hash = "#/open"; return; }   // RequireSessionPath
  refreshChrome();
  const root = $("view");
  root.replaceChildren();
  try { await views[r](root); } catch (e) { root.append(alertBox(e.message, "err")); }
}

async function health() {
  const b = $("api-health");
  try { const r = await Api.health(); b.textContent = `API ${r.status} · v${r.version}`; b.className = "badge ok"; }
  catch { b.textContent = "API unreachable"; b.className = "badge err"; }
}

$("theme").addEventListener("click", () => {
  document.documentElement.classList.toggle("dark");
  localStorage.setItem("lumen.theme", document.documentElement.classList.contains("dark") ? "dark" : "light");
});
if (localStorage.getItem("lumen.theme") === "dark") document.documentElement.classList.add("dark");
window.addEventListener("hashchange", route);
health();
setInterval(health, 15000);
route();
