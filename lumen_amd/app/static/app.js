// Lumen control-plane SPA (plain ES2019, no build step).  The DOM-free core -- API client,
// error presentation, wizard gating, validation -- lives in lumen.js (window.Lumen) and is
// unit-tested under Node; this file is the views and the hash router.
//
// Routes (reference lumen-app/web-ui/src/App.tsx:27-71):
//   /open           OpenPath: pick/validate the Lumen directory, recent paths
//   /session        SessionHub: what is installed there, resume or reconfigure
//   /setup/welcome  wizard 1: directory, region, mDNS service name, gRPC port
//   /setup/hardware wizard 2: hardware preset + driver checks
//   /setup/config   wizard 3: service profile -> generated lumen-config.yaml
//   /setup/install  wizard 4: setup task with per-step progress, logs, cancel/retry/finish
//   /server         hub server start/stop/restart, health, config YAML, live logs
"use strict";

const L = window.Lumen;
const Api = L.createApi(window.fetch.bind(window), "");

// ------------------------------------------------------------------ persisted state
const Session = L.createStore(window.localStorage, "lumen.session", { path: "", recent: [] });
const Wizard = L.createStore(window.sessionStorage, "lumen.wizard", L.DEFAULT_WIZARD);

function setSessionPath(p) {
  const n = String(p || "").trim();
  Session.set({ path: n, recent: n ? L.rememberPath(Session.get("recent") || [], n) : Session.get("recent") });
  if (Wizard.get("installPath") !== n) Wizard.reset({ installPath: n });
  refreshChrome();
}

// ------------------------------------------------------------------ DOM helpers
function h(tag, attrs, ...kids) {
  const el = document.createElement(tag);
  Object.entries(attrs || {}).forEach(([k, v]) => {
    if (k === "class") el.className = v;
    else if (k.startsWith("on") && typeof v === "function") el.addEventListener(k.slice(2), v);
    else if (v === true) el.setAttribute(k, "");
    else if (v !== false && v != null) el.setAttribute(k, v);
  });
  kids.flat(3).forEach((c) => {
    if (c != null && c !== false) el.append(c instanceof Node ? c : document.createTextNode(String(c)));
  });
  return el;
}
const $ = (id) => document.getElementById(id);
function toast(msg, kind, ms) {
  const t = $("toast");
  t.textContent = msg;
  t.className = `toast ${kind || ""}`;
  clearTimeout(toast._t);
  toast._t = setTimeout(() => t.classList.add("hidden"), ms || 3500);
}
const badge = (text, kind) => h("span", { class: `badge ${kind === undefined ? L.statusKind(text) : kind}` }, String(text).replace(/_/g, " "));
const alertBox = (text, kind, title) => h("div", { class: `alert ${kind || ""}` }, title ? h("strong", {}, title, " ") : null, text);
const errorBox = (e, fallback) => { const d = L.describeUiError(e, fallback || "request failed"); return alertBox(d.message, "err", d.title); };
const card = (title, ...kids) => h("div", { class: "card" }, title ? h("h2", {}, title) : null, ...kids);
const skeleton = (n) => Array.from({ length: n || 3 }, () => h("div", { class: "skeleton" }));
const row = (...kids) => h("div", { class: "row" }, ...kids);
const kv = (pairs) => h("table", { class: "kv" }, pairs.filter(Boolean).map(([k, v]) => h("tr", {}, h("td", {}, k), h("td", {}, v))));
const field = (label, input, hint) => h("div", { class: "field" }, h("label", {}, label), input, hint || null);
function debounce(fn, ms) { let t; return (...a) => { clearTimeout(t); t = setTimeout(() => fn(...a), ms); }; }
const go = (path) => { location.hash = `#${path}`; };
async function busy(btn, fn) {
  btn.disabled = true;
  btn.classList.add("busy");
  try { return await fn(); } finally { btn.disabled = false; btn.classList.remove("busy"); }
}
function copyText(text) {
  if (navigator.clipboard && window.isSecureContext) return navigator.clipboard.writeText(text);
  const ta = h("textarea", { style: "position:fixed;opacity:0" });
  ta.value = text;
  document.body.append(ta);
  ta.select();
  document.execCommand("copy");
  ta.remove();
  return Promise.resolve();
}
function modal(title, body, actions) {
  const close = () => wrap.remove();
  const wrap = h("div", { class: "modal-wrap", onclick: (e) => { if (e.target === wrap) close(); } },
    h("div", { class: "modal" }, h("h2", {}, title), body, row(...(actions || []), h("button", { class: "ghost", onclick: close }, "Close"))));
  document.body.append(wrap);
  onLeave(close);
  return close;
}
function openSocket(path, onMessage) {
  try {
    const ws = new WebSocket(L.wsUrl(location, path));
    ws.onmessage = (ev) => { try { onMessage(JSON.parse(ev.data)); } catch (e) { /* non-JSON frame */ } };
    onLeave(() => ws.close());
    return ws;
  } catch (e) { return null; }
}

// cleanup hooks for the current view (websockets, intervals, dialogs)
let cleanups = [];
function onLeave(fn) { cleanups.push(fn); }
function every(ms, fn) { const iv = setInterval(fn, ms); onLeave(() => clearInterval(iv)); return iv; }

// ------------------------------------------------------------------ views
const views = {};

views["/open"] = async (root) => {
  $("title").textContent = "Open a Lumen directory";
  const input = h("input", { id: "path", placeholder: "~/.lumen or /opt/lumen", value: Session.get("path") || "~/.lumen" });
  const status = h("div", { class: "status" });
  const openBtn = h("button", { disabled: true }, "Open");
  let last = null;
  const check = debounce(async () => {
    const p = input.value.trim();
    const err = L.pathError(p);
    if (err) { status.replaceChildren(alertBox(err, "err")); openBtn.disabled = true; return; }
    status.replaceChildren(...skeleton(1));
    try {
      const [v, inst] = await Promise.all([Api.validatePath(p), Api.checkPath(p).catch(() => null)]);
      if (input.value.trim() !== p) return;        // superseded by a newer keystroke
      last = { v, inst };
      const kids = [];
      if (v.error) kids.push(alertBox(v.error, "err"));
      if (v.warning) kids.push(alertBox(v.warning, "warn"));
      kids.push(row(badge(v.exists ? "exists" : "will be created", ""), badge(v.writable ? "writable" : "not writable", v.writable ? "ok" : "err"),
        v.free_space_gb != null ? badge(`${v.free_space_gb} GB free`, v.free_space_gb >= 10 ? "" : "warn") : null,
        inst && inst.has_existing_service ? badge("existing installation", "ok") : null));
      if (inst && inst.message) kids.push(h("p", { class: "muted" }, inst.message));
      status.replaceChildren(...kids);
      openBtn.disabled = !v.writable;
      openBtn.textContent = inst && inst.has_existing_service ? "Open installation" : "Set up here";
    } catch (e) { status.replaceChildren(errorBox(e)); openBtn.disabled = true; }
  }, 400);
  input.addEventListener("input", check);
  input.addEventListener("keydown", (e) => { if (e.key === "Enter" && !openBtn.disabled) openBtn.click(); });
  openBtn.addEventListener("click", () => {
    const p = input.value.trim();
    setSessionPath(p);
    go(last && last.inst && last.inst.has_existing_service ? "/session" : "/setup/welcome");
  });
  const recent = Session.get("recent") || [];
  root.append(card("Lumen directory",
    h("p", { class: "muted" }, "Models, label banks, the generated lumen-config.yaml and server logs live here. " +
      "An existing directory is opened as a session; an empty one starts the setup wizard."),
    field("Path", input), status, row(openBtn)),
  recent.length ? card("Recent", h("ul", { class: "links" }, recent.map((p) => h("li", {},
    h("a", { href: "#", onclick: (e) => { e.preventDefault(); input.value = p; check(); } }, p))))) : null);
  check();
};

views["/session"] = async (root) => {
  $("title").textContent = "Session";
  const p = Session.get("path");
  const body = h("div", {}, ...skeleton(4));
  const srv = h("div", {}, ...skeleton(2));
  root.append(card(`Installation at ${p}`, body), card("Hub server", srv));
  try {
    const [r, cur] = await Promise.all([Api.checkPath(p), Api.currentConfig().catch(() => ({ loaded: false }))]);
    const s = r.service_status;
    const cfgFile = `${p.replace(/\/+$/, "")}/lumen-config.yaml`;
    const actions = row();
    if (r.has_existing_service) {
      const useBtn = h("button", {}, "Use this configuration");
      useBtn.addEventListener("click", () => busy(useBtn, async () => {
        try { await Api.loadConfig(cfgFile); toast("configuration loaded", "ok"); go("/server"); } catch (e) { body.append(errorBox(e, "could not load the configuration")); }
      }));
      actions.append(useBtn);
    }
    actions.append(h("button", { class: "secondary", onclick: () => { Wizard.reset({ installPath: p }); go("/setup/welcome"); } }, "Configure new"));
    if (r.recommended_action === "repair") {
      actions.append(h("button", { class: "secondary", onclick: () => { Wizard.set({ installPath: p }); go("/setup/hardware"); } }, "Repair"));
    }
    actions.append(h("button", { class: "ghost", onclick: () => { Session.set({ path: "" }); Wizard.reset(); go("/open"); } }, "Switch directory"));
    body.replaceChildren(alertBox(r.message, r.ready_to_start ? "ok" : "warn"),
      kv([["configuration (lumen-config.yaml)", badge(s.config ? "ok" : "missing")],
        ["runtime environment", badge(s.environment ? "ok" : "missing")],
        ["drivers", badge(s.drivers ? "ok" : "missing")],
        ["micromamba", badge(s.micromamba ? "ok" : "not installed", s.micromamba ? "ok" : "")],
        ["recommended", r.recommended_action.replace(/_/g, " ")],
        cur.loaded ? ["loaded configuration", h("code", {}, cur.config_path)] : null]),
      actions);
  } catch (e) { body.replaceChildren(errorBox(e)); }
  try {
    const s = await Api.serverStatus();
    srv.replaceChildren(kv([["state", badge(s.running ? "running" : "stopped", s.running ? "ok" : "")], ["health", badge(s.health)],
      ["address", `${s.host}:${s.port}`]]), row(h("button", { class: "secondary", onclick: () => go("/server") }, "Open server view")));
  } catch (e) { srv.replaceChildren(errorBox(e)); }
};

// ---- wizard chrome (WizardLayout.tsx): step guard + back/next bar
function wizardGuard(stepId) {
  const to = L.wizardGate(Wizard.all(), stepId);
  if (to) { go(to); return false; }
  return true;
}
function navBar(backPath, next) {
  return h("div", { class: "row navbar" }, backPath ? h("button", { class: "ghost", onclick: () => go(backPath) }, "Back") : null,
    h("span", { class: "spacer" }), next);
}

views["/setup/welcome"] = async (root) => {
  $("title").textContent = "Setup · basics";
  if (!Wizard.get("installPath")) Wizard.set({ installPath: Session.get("path") });
  const w = Wizard.all();
  const region = h("select", { id: "region" }, h("option", { value: "other" }, "International (Hugging Face)"), h("option", { value: "cn" }, "China mainland (ModelScope, mirrors)"));
  region.value = w.region;
  const port = h("input", { id: "port", inputmode: "numeric", value: String(w.port) });
  const name = h("input", { id: "serviceName", placeholder: "lumen-ai", value: w.serviceName });
  const portMsg = h("div", { class: "hint err" });
  const nameMsg = h("div", { class: "hint err" });
  const next = h("button", {}, "Next: hardware");
  const validate = () => {
    const pe = L.portError(port.value), ne = L.serviceNameError(name.value);
    portMsg.textContent = pe || "";
    nameMsg.textContent = ne || "";
    next.disabled = Boolean(pe || ne);
    return !next.disabled;
  };
  [port, name].forEach((el) => el.addEventListener("input", validate));
  next.addEventListener("click", () => {
    if (!validate()) return;
    const patch = { region: region.value, port: parseInt(port.value, 10), serviceName: name.value.trim() };
    const changed = Object.keys(patch).some((k) => Wizard.get(k) !== patch[k]);
    Wizard.set(changed ? Object.assign(patch, { configGenerated: false, configPath: null, configKey: null }) : patch);
    go("/setup/hardware");
  });
  root.append(card("Welcome",
    h("p", {}, "This wizard prepares a Lumen hub on this machine:"),
    h("ol", {}, h("li", {}, "basics: where models come from and how clients find the hub,"),
      h("li", {}, "a hardware preset (AMD MI355X / ROCm, or CPU) and its driver checks,"),
      h("li", {}, "the services to run, written to lumen-config.yaml,"),
      h("li", {}, "the setup task: runtime environment, native gfx950 kernels, model cache.")),
    kv([["directory", h("code", {}, w.installPath)]])),
  card("Basics",
    h("div", { class: "grid" }, field("Region *", region, h("div", { class: "hint" }, "selects model mirrors")),
      field("gRPC port *", port, portMsg), field("Service name (mDNS) *", name, nameMsg))),
  navBar(null, next));
  validate();
};

views["/setup/hardware"] = async (root) => {
  $("title").textContent = "Setup · hardware";
  if (!wizardGuard("hardware")) return;
  const sys = h("div", {}, ...skeleton(3));
  const list = h("div", { class: "grid presets" }, ...skeleton(4));
  const drivers = h("div");
  const next = h("button", { disabled: !Wizard.get("hardwarePreset") }, "Next: services");
  next.addEventListener("click", () => go("/setup/config"));
  const detectBtn = h("button", { class: "secondary" }, "Detect hardware");
  root.append(card("This machine", sys), card("Hardware preset", row(detectBtn), list, drivers), navBar("/setup/welcome", next));

  let presets = [];
  const select = async (name) => {
    if (Wizard.get("hardwarePreset") !== name) Wizard.set({ hardwarePreset: name, configGenerated: false, configPath: null, configKey: null });
    next.disabled = false;
    list.querySelectorAll(".preset").forEach((c) => c.classList.toggle("selected", c.dataset.name === name));
    const p = presets.find((x) => x.name === name);
    drivers.replaceChildren(...skeleton(2));
    try {
      const ds = await Api.checkPreset(name);
      drivers.replaceChildren(h("h3", {}, `Driver checks for ${name}`),
        h("table", {}, ds.map((d) => h("tr", {}, h("td", {}, d.name), h("td", {}, badge(d.status)), h("td", { class: "muted" }, d.details),
          h("td", {}, d.installable_via_mamba ? badge("installable by setup", "") : null)))),
        ds.some((d) => d.status !== "available") ? alertBox("Some drivers are missing; the setup task installs the installable ones, " +
          "the others need a system install (ROCm).", "warn") : alertBox("All drivers available.", "ok"),
        p && p.providers && p.providers.length ? h("p", { class: "muted" }, `providers: ${p.providers.join(", ")}`) : null);
    } catch (e) { drivers.replaceChildren(errorBox(e)); }
  };
  try {
    const info = await Api.hardwareInfo();
    presets = info.presets || [];
    const gpus = (info.gpus || []).map((g) => h("li", {}, Object.entries(g).map(([k, v]) => `${k}: ${v}`).join(" · ")));
    sys.replaceChildren(kv([["platform", `${info.platform} ${info.machine}`], ["processor", info.processor || "—"],
      ["python", info.python_version], ["recommended preset", badge(info.recommended_preset || "cpu", "ok")]]),
    gpus.length ? h("ul", {}, gpus) : h("p", { class: "muted" }, "no AMD GPU detected"));
    list.replaceChildren(...presets.map((p) => {
      const c = h("div", { class: "card preset", "data-name": p.name, tabindex: "0" },
        h("h3", {}, p.name, p.name === info.recommended_preset ? badge("recommended", "ok") : null), h("div", { class: "muted" }, p.description),
        row(badge(p.runtime, ""), badge(p.availability), p.supported_on_current_platform ? null : badge("unsupported OS", "err")));
      c.addEventListener("click", () => select(p.name));
      c.addEventListener("keydown", (e) => { if (e.key === "Enter") select(p.name); });
      return c;
    }));
    const cur = Wizard.get("hardwarePreset") || info.recommended_preset;
    if (cur) select(cur);
  } catch (e) { sys.replaceChildren(errorBox(e)); list.replaceChildren(); }
  detectBtn.addEventListener("click", () => busy(detectBtn, async () => {
    try { const r = await Api.detect(); toast(`recommended preset: ${r.recommended_preset}`, "ok"); select(r.recommended_preset); } catch (e) { toast(L.describeUiError(e).message, "err"); }
  }));
};

views["/setup/config"] = async (root) => {
  $("title").textContent = "Setup · services";
  if (!wizardGuard("config")) return;
  const out = h("div");
  const next = h("button", { disabled: !Wizard.get("configGenerated") }, "Next: install");
  next.addEventListener("click", () => go("/setup/install"));
  const clip = h("select", { id: "clipModel" });
  const svcList = h("div", { class: "services" });
  let inflight = false;

  const showYaml = async (warnings) => {
    try {
      const y = await Api.configYaml();
      const val = h("button", { class: "secondary" }, "Validate");
      const valOut = h("div");
      val.addEventListener("click", () => busy(val, async () => {
        try {
          const r = await Api.validateConfig(Wizard.get("configContent") || {});
          valOut.replaceChildren(r.valid ? alertBox("configuration is valid", "ok") : alertBox(r.errors.join("; "), "err", "Invalid:"));
        } catch (e) { valOut.replaceChildren(errorBox(e)); }
      }));
      out.replaceChildren(...(warnings || []).map((w) => alertBox(w, "warn")),
        card(`Generated ${Wizard.get("configPath") || "lumen-config.yaml"}`, h("pre", { class: "yaml" }, y.yaml || ""),
          row(val, h("button", { class: "ghost", onclick: () => copyText(y.yaml || "").then(() => toast("copied", "ok")) }, "Copy")), valOut));
    } catch (e) { out.replaceChildren(errorBox(e)); }
  };

  const generate = async (force) => {
    const s = Wizard.all();
    if (!s.servicePreset || inflight) return;
    const key = L.configKey(s);
    if (!force && s.configGenerated && key === s.configKey) { showYaml(); return; }
    inflight = true;
    next.disabled = true;
    Wizard.set({ configGenerated: false, configPath: null, configKey: null });
    out.replaceChildren(...skeleton(3));
    try {
      const r = await Api.generateConfig(L.generateRequest(s));
      if (!r.success) { out.replaceChildren(alertBox(r.message, "err", "Rejected:")); return; }
      Wizard.set({ configGenerated: true, configPath: r.config_path, configKey: key, configContent: r.config_content });
      next.disabled = false;
      await showYaml(r.warnings);
    } catch (e) {
      out.replaceChildren(errorBox(e, "configuration generation failed"),
        row(h("button", { class: "secondary", onclick: () => generate(true) }, "Retry")));
    } finally { inflight = false; }
  };

  const renderServices = () => {
    const p = L.SERVICE_PRESETS.find((x) => x.id === Wizard.get("servicePreset"));
    const on = p ? p.services : [];
    svcList.replaceChildren(...L.SERVICES.map((s) => h("div", { class: `svc ${on.indexOf(s.id) >= 0 ? "on" : "off"}` },
      h("strong", {}, s.name), " ", h("code", {}, s.package), h("div", { class: "muted" }, s.description))));
    const opts = (p && p.clipModels) || [];
    clip.replaceChildren(h("option", { value: "" }, opts.length ? "default for the region" : "n/a for this profile"), ...opts.map((o) => h("option", { value: o }, o)));
    clip.disabled = !opts.length;
    clip.value = opts.indexOf(Wizard.get("clipModel")) >= 0 ? Wizard.get("clipModel") : "";
  };
  clip.addEventListener("change", () => { Wizard.set({ clipModel: clip.value || null }); generate(false); });

  const cards = L.SERVICE_PRESETS.map((p) => {
    const c = h("div", { class: "card preset", "data-name": p.id, tabindex: "0" },
      h("h3", {}, p.name, p.recommended ? badge("recommended", "ok") : null), h("div", {}, p.description),
      h("div", { class: "muted" }, p.requirements), row(...p.services.map((s) => badge(s, ""))));
    const pick = () => {
      const again = Wizard.get("servicePreset") === p.id;
      Wizard.set({ servicePreset: p.id, clipModel: again ? Wizard.get("clipModel") : null });
      cards.forEach((x) => x.classList.toggle("selected", x.dataset.name === p.id));
      renderServices();
      generate(again);            // clicking the selected profile again regenerates
    };
    c.addEventListener("click", pick);
    c.addEventListener("keydown", (e) => { if (e.key === "Enter") pick(); });
    return c;
  });
  root.append(card(`Services for hardware preset ${Wizard.get("hardwarePreset")}`,
    h("p", { class: "muted" }, "Pick a profile; lumen-config.yaml is generated in the Lumen directory as soon as you do."),
    h("div", { class: "grid presets" }, cards), h("h3", {}, "Services in this profile"), svcList, field("CLIP model", clip)),
  out, navBar("/setup/hardware", next));
  cards.forEach((x) => x.classList.toggle("selected", x.dataset.name === Wizard.get("servicePreset")));
  renderServices();
  if (Wizard.get("servicePreset")) generate(false);
};

views["/setup/install"] = async (root) => {
  $("title").textContent = "Setup · install";
  if (!wizardGuard("install")) return;
  const preset = Wizard.get("hardwarePreset");
  const dir = Wizard.get("installPath");
  const status = h("div", {}, ...skeleton(3));
  const bar = h("div", { class: "progress" }, h("div", { style: "width:0%" }));
  const pct = h("span", { class: "muted" }, "");
  const stepsTbl = h("table", { class: "steps-table" });
  const logs = h("pre", { class: "logs" });
  const envKind = h("select", { id: "envKind" }, h("option", { value: "current" }, "this Python (ROCm PyTorch already here)"),
    h("option", { value: "venv" }, "isolated venv over the host PyTorch"), h("option", { value: "micromamba" }, "micromamba env (envs/rocm.yaml)"));
  envKind.value = Wizard.get("envKind") || "current";
  envKind.addEventListener("change", () => Wizard.set({ envKind: envKind.value }));
  const force = h("input", { type: "checkbox", class: "inline" });
  const startBtn = h("button", {}, "Run setup");
  const cancelBtn = h("button", { class: "secondary", disabled: true }, "Cancel");
  const retryBtn = h("button", { class: "secondary hidden" }, "Retry");
  const finishBtn = h("button", { class: "hidden" }, "Finish: load config and open server");
  const err = h("div");
  root.append(card("Environment", status),
    card("Setup task", h("div", { class: "grid" }, field("Runtime environment", envKind),
      field("Options", h("label", { class: "check" }, force, "force reinstall"))),
    row(startBtn, cancelBtn, retryBtn, finishBtn), h("div", { class: "progress-row" }, bar, pct), err, stepsTbl),
    card("Logs", logs), navBar("/setup/config", null));

  let taskId = null, cancelRequested = false, stopFollow = null;
  const loadStatus = async () => {
    try {
      const s = await Api.installStatus(dir);
      status.replaceChildren(kv([["directory", h("code", {}, dir)], ["hardware preset", preset],
        ["runtime environment", badge(s.environment_exists ? "ready" : "not created", s.environment_exists ? "ok" : "warn")],
        ["ready for preset", s.ready_for_preset || "—"],
        ...Object.entries(s.drivers || {}).map(([k, v]) => [`driver ${k}`, badge(v)])]),
      s.missing_components.length ? alertBox(`missing: ${s.missing_components.join(", ")}`, "warn") : alertBox("all components present", "ok"));
    } catch (e) { status.replaceChildren(errorBox(e)); }
  };
  const render = (t) => {
    bar.firstChild.style.width = `${t.progress}%`;
    pct.textContent = `${t.progress}% · ${t.status}${t.current_step ? ` · ${t.current_step}` : ""}`;
    stepsTbl.replaceChildren(h("tr", {}, h("th", {}, "step"), h("th", {}, "status"), h("th", {}, "progress"), h("th", {}, "detail")),
      t.steps.map((s) => h("tr", { class: s.status }, h("td", {}, s.name), h("td", {}, badge(s.status)), h("td", {}, `${s.progress}%`),
        h("td", { class: "muted" }, s.message))));
    const done = L.taskDone(t.status);
    cancelBtn.disabled = done || cancelRequested;
    cancelBtn.textContent = cancelRequested && !done ? "Cancelling…" : "Cancel";
    startBtn.disabled = !done && taskId !== null;
    retryBtn.classList.toggle("hidden", !(t.status === "failed" || t.status === "cancelled"));
    finishBtn.classList.toggle("hidden", t.status !== "completed");
    err.replaceChildren(t.error ? alertBox(t.error, "err", "Setup failed:") : null);
    if (t.status === "completed") Wizard.set({ installationComplete: true });
    if (done) { cancelRequested = false; if (stopFollow) { stopFollow(); stopFollow = null; } }
  };
  const pullLogs = async () => {
    if (!taskId) return;
    try { logs.textContent = (await Api.installLogs(taskId, 500)).logs.join("\n"); logs.scrollTop = logs.scrollHeight; } catch (e) { /* task gone */ }
  };
  const follow = (id) => {
    taskId = id;
    Wizard.set({ installTask: id });
    const iv = every(1500, pullLogs);
    let ws = openSocket(`/ws/install/${encodeURIComponent(id)}`, (m) => {
      if (m.task) render(m.task);
      if (m.type === "complete" || m.type === "error") { pullLogs(); loadStatus(); }
    });
    const pv = ws ? null : every(1000, async () => { try { render(await Api.installTask(id)); } catch (e) { /* gone */ } });
    stopFollow = () => { clearInterval(iv); if (pv) clearInterval(pv); if (ws) { ws.close(); ws = null; } };
  };
  const start = () => busy(startBtn, async () => {
    err.replaceChildren();
    cancelRequested = false;
    try {
      const t = await Api.startInstall({ preset, cache_dir: dir, environment_name: "lumen_env", force_reinstall: force.checked,
        env_kind: envKind.value });
      render(t);
      follow(t.task_id);
    } catch (e) { err.replaceChildren(errorBox(e, "could not start the setup task")); }
  });
  startBtn.addEventListener("click", start);
  retryBtn.addEventListener("click", () => { Wizard.set({ installationComplete: false }); start(); });
  cancelBtn.addEventListener("click", async () => {
    if (!taskId || cancelRequested) return;
    cancelRequested = true;
    cancelBtn.disabled = true;
    try { render(await Api.cancelInstall(taskId)); Wizard.set({ installationComplete: false }); loadStatus(); } catch (e) { cancelRequested = false; err.replaceChildren(errorBox(e)); }
  });
  finishBtn.addEventListener("click", () => busy(finishBtn, async () => {
    const cfg = Wizard.get("configPath") || `${dir.replace(/\/+$/, "")}/lumen-config.yaml`;
    try { await Api.loadConfig(cfg); go("/server"); } catch (e) { err.replaceChildren(errorBox(e, "could not load the generated configuration")); }
  }));
  await loadStatus();
  const prev = Wizard.get("installTask");
  if (prev) {
    try {
      const t = await Api.installTask(prev);
      taskId = prev;
      render(t);
      pullLogs();
      if (!L.taskDone(t.status)) follow(prev);
    } catch (e) { Wizard.set({ installTask: null }); }
  }
};

views["/server"] = async (root) => {
  $("title").textContent = "Server";
  const cfgCard = h("div", {}, ...skeleton(2));
  const st = h("div", {}, ...skeleton(4));
  const logs = h("pre", { class: "logs" });
  const cfgPath = h("input", { id: "cfgPath", placeholder: "lumen-config.yaml (default: the loaded configuration)" });
  const portIn = h("input", { id: "portOverride", inputmode: "numeric", placeholder: "from config" });
  const hostIn = h("input", { id: "hostOverride", placeholder: "from config" });
  const startB = h("button", {}, "Start");
  const stopB = h("button", { class: "secondary" }, "Stop");
  const restartB = h("button", { class: "secondary" }, "Restart");
  const forceStop = h("input", { type: "checkbox", class: "inline" });
  const follow = h("input", { type: "checkbox", class: "inline", checked: true });
  const filter = h("input", { placeholder: "filter lines" });
  const err = h("div");
  let lines = [];
  const drawLogs = () => {
    const f = filter.value.trim().toLowerCase();
    logs.textContent = (f ? lines.filter((l) => l.toLowerCase().indexOf(f) >= 0) : lines).join("\n");
    if (follow.checked) logs.scrollTop = logs.scrollHeight;
  };
  filter.addEventListener("input", drawLogs);
  root.append(card("Configuration", cfgCard),
    card("Hub server", st,
      h("div", { class: "grid" }, field("Config path", cfgPath), field("Port override", portIn), field("Host override", hostIn)),
      row(startB, stopB, restartB, h("label", { class: "check" }, forceStop, "force stop")), err),
    card("Logs", row(filter, h("label", { class: "check" }, follow, "follow"),
      h("button", { class: "ghost", onclick: () => copyText(lines.join("\n")).then(() => toast("copied", "ok")) }, "Copy"),
      h("button", { class: "ghost", onclick: () => { lines = []; drawLogs(); } }, "Clear view")), logs));

  const showCfg = async () => {
    try {
      const c = await Api.currentConfig();
      if (!c.loaded) {
        cfgCard.replaceChildren(alertBox("No configuration loaded: finish the setup wizard or open an existing installation.", "warn"),
          row(h("button", { class: "secondary", onclick: () => go("/session") }, "Back to session")));
        return;
      }
      cfgPath.placeholder = c.config_path;
      const view = h("button", { class: "secondary" }, "View YAML");
      view.addEventListener("click", () => busy(view, async () => {
        try {
          const y = await Api.configYaml();
          modal(c.config_path, h("pre", { class: "yaml" }, y.yaml), [h("button", { onclick: () => copyText(y.yaml).then(() => toast("copied", "ok")) }, "Copy")]);
        } catch (e) { toast(L.describeUiError(e).message, "err"); }
      }));
      const d = c.device || {};
      cfgCard.replaceChildren(kv([["file", h("code", {}, c.config_path)], ["cache dir", h("code", {}, c.cache_dir)],
        ["region", c.region], ["service name", c.service_name], ["port", c.port],
        d.runtime ? ["runtime", `${d.runtime} · batch ${d.batch_size} · ${d.precision}`] : null]), row(view));
    } catch (e) { cfgCard.replaceChildren(errorBox(e)); }
  };
  const show = (s) => {
    st.replaceChildren(kv([["state", badge(s.running ? "running" : "stopped", s.running ? "ok" : "")], ["health", badge(s.health)],
      ["pid", s.pid != null ? s.pid : "—"], ["address", `${s.host}:${s.port}`], ["mDNS name", s.service_name],
      ["uptime", L.formatDuration(s.uptime_seconds)], ["config", s.config_path || "—"]]),
    s.last_error ? alertBox(s.last_error, "err", "Last error:") : null);
    startB.disabled = s.running;
    stopB.disabled = !s.running;
  };
  const poll = async () => { try { show(await Api.serverStatus()); } catch (e) { st.replaceChildren(errorBox(e)); } };
  const body = () => {
    const pe = portIn.value.trim() ? L.portError(portIn.value) : null;
    if (pe) throw new Error(pe);
    return { config_path: cfgPath.value.trim() || null, port: portIn.value.trim() ? parseInt(portIn.value, 10) : null,
      host: hostIn.value.trim() || null, environment: "lumen_env" };
  };
  const act = (btn, fn, msg) => btn.addEventListener("click", () => busy(btn, async () => {
    err.replaceChildren();
    try { show(await fn()); if (msg) toast(msg, "ok"); } catch (e) { err.replaceChildren(errorBox(e)); }
    poll();
  }));
  act(startB, () => Api.startServer(body()), "server starting");
  act(stopB, () => Api.stopServer({ force: forceStop.checked, timeout: 30 }), "server stopped");
  act(restartB, () => Api.restartServer(Object.assign(body(), { force: forceStop.checked, timeout: 30 })), "server restarting");
  await Promise.all([showCfg(), poll()]);
  every(3000, poll);
  try { lines = (await Api.serverLogs(500)).logs; drawLogs(); } catch (e) { /* no logs yet */ }
  const ws = openSocket("/ws/logs", (m) => { if (m.type === "log") { lines = L.appendBounded(lines, [m.message], 5000); drawLogs(); } });
  if (!ws) every(2000, async () => { try { lines = (await Api.serverLogs(500)).logs; drawLogs(); } catch (e) { /* ignore */ } });
};

// ------------------------------------------------------------------ router (App.tsx)
function refreshChrome() {
  const p = Session.get("path");
  $("session-path").textContent = p || "—";
  const r = location.hash.replace(/^#/, "") || "/open";
  document.querySelectorAll("#nav a").forEach((a) => {
    a.classList.toggle("active", a.dataset.route === r);
    a.classList.toggle("disabled", a.hasAttribute("data-needs-session") && !p);
  });
  const steps = $("steps");
  const cur = L.WIZARD_STEPS.findIndex((s) => s.path === r);
  if (cur >= 0) {
    const w = Wizard.all();
    steps.replaceChildren(...L.WIZARD_STEPS.map((s, i) => {
      const reachable = !L.wizardGate(w, s.id);
      return h(reachable ? "a" : "span", { class: `s ${i < cur ? "done" : i === cur ? "cur" : ""}`, href: reachable ? `#${s.path}` : null }, `${i + 1}. ${s.name}`);
    }));
    steps.classList.remove("hidden");
  } else steps.classList.add("hidden");
}

async function route() {
  cleanups.forEach((f) => { try { f(); } catch (e) { /* ignore */ } });
  cleanups = [];
  let r = location.hash.replace(/^#/, "") || "/open";
  if (r === "/") r = "/open";
  if (r === "/setup") r = "/setup/welcome";
  if (!views[r]) { go("/open"); return; }
  if (r !== "/open" && !Session.get("path")) { go("/open"); return; }   // RequireSessionPath
  refreshChrome();
  const root = $("view");
  root.replaceChildren();
  try { await views[r](root); } catch (e) { root.append(errorBox(e)); }
  refreshChrome();
}

async function health() {
  const b = $("api-health");
  try { const r = await Api.health(); b.textContent = `API ${r.status} · v${r.version}`; b.className = "badge ok"; } catch (e) { b.textContent = "API unreachable"; b.className = "badge err"; }
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
