// Lumen control-plane UI core: API client, error presentation, wizard state machine and
// input validation.  DOM-free on purpose: the browser loads it as a classic script
// (window.Lumen), Node loads it with require() for the UI tests (tests/webui/*.test.js).
// Written to ES2019 so the Node in the build image runs it unchanged.
//
// Parity map (reference lumen-app/web-ui/src):
//   createApi / ApiError          lib/api.ts:1-456 (fetchApi, resolveErrorMessage/Kind)
//   describeUiError               lib/errorPresentation.ts
//   portError / serviceNameError  lib/wizardValidation.ts
//   WIZARD_STEPS / wizardGate     context/wizardConfig.ts + components/wizard/WizardLayout.tsx
//   SERVICE_PRESETS / SERVICES    views/Config.tsx:54-127
//   createStore / Session         hooks/useLumenSession.ts, context/WizardProvider.tsx
(function (root, factory) {
  if (typeof module === "object" && module.exports) module.exports = factory();
  else root.Lumen = factory();
})(typeof self !== "undefined" ? self : this, function () {
  "use strict";

  // ---------------------------------------------------------------------- errors
  class ApiError extends Error {
    constructor(message, kind, status) {
      super(message);
      this.name = "ApiError";
      this.kind = kind;       // network | permission | business | server | unknown
      this.status = status;
    }
  }

  function errorKind(status) {
    if (status === 401 || status === 403) return "permission";
    if (status >= 400 && status < 500) return "business";
    if (status >= 500) return "server";
    return "unknown";
  }

  const nonEmpty = (s) => typeof s === "string" && s.trim() !== "";

  // FastAPI puts the message in `detail` (string, or a list of pydantic errors for 422)
  function errorMessage(payload, fallback) {
    if (nonEmpty(payload)) return payload;
    if (payload && typeof payload === "object") {
      if (nonEmpty(payload.message)) return payload.message;
      const d = payload.detail;
      if (nonEmpty(d)) return d;
      if (Array.isArray(d) && d.length) {
        return d.map((e) => {
          const loc = Array.isArray(e.loc) ? e.loc.filter((x) => x !== "body").join(".") : "";
          return loc ? `${loc}: ${e.msg}` : String(e.msg || JSON.stringify(e));
        }).join("; ");
      }
      if (d && typeof d === "object" && nonEmpty(d.message)) return d.message;
    }
    return fallback;
  }

  const ERROR_TITLES = {
    network: "Network error", permission: "Permission denied", business: "Request rejected",
    server: "Server error",
  };

  function describeUiError(error, fallback) {
    if (error instanceof ApiError && ERROR_TITLES[error.kind]) {
      return { title: ERROR_TITLES[error.kind], message: error.message || fallback };
    }
    if (error instanceof Error) return { title: "Request failed", message: error.message || fallback };
    return { title: "Unknown error", message: fallback };
  }

  // ---------------------------------------------------------------------- API client
  const API = "/api/v1";

  function query(q) {
    const parts = [];
    Object.keys(q || {}).forEach((k) => {
      const v = q[k];
      if (v !== undefined && v !== null) parts.push(`${encodeURIComponent(k)}=${encodeURIComponent(String(v))}`);
    });
    return parts.length ? `?${parts.join("&")}` : "";
  }

  // Every control-plane call the UI makes.  `fetchImpl` is window.fetch in the browser and a
  // recording/HTTP shim in the tests; `base` prefixes every path ("" = same origin).
  function createApi(fetchImpl, base) {
    const prefix = base || "";

    async function call(path, opts) {
      const o = opts || {};
      const init = { method: o.method || "GET", headers: { Accept: "application/json" } };
      if (o.body !== undefined) {
        init.headers["Content-Type"] = "application/json";
        init.body = JSON.stringify(o.body);
      }
      const url = prefix + (path.charAt(0) === "/" ? path : `${API}/${path}`) + query(o.query);
      let r;
      try {
        r = await fetchImpl(url, init);
      } catch (e) {
        throw new ApiError("Cannot reach the Lumen control plane; is `lumen-app` running?", "network");
      }
      const text = await r.text();
      let data = null;
      try { data = text ? JSON.parse(text) : null; } catch (e) { data = text; }
      if (!r.ok) {
        throw new ApiError(errorMessage(data, `HTTP ${r.status}: ${r.statusText || ""}`.trim()), errorKind(r.status), r.status);
      }
      return r.status === 204 ? undefined : data;
    }

    const id = encodeURIComponent;
    return {
      call,
      health: () => call("/health"),
      // config (lib/api.ts:143-253)
      generateConfig: (req) => call("config/generate", { method: "POST", body: req }),
      currentConfig: () => call("config/current"),
      loadConfig: (configPath) => call("config/load", { method: "POST", query: { config_path: configPath } }),
      configYaml: () => call("config/yaml"),
      validateConfig: (cfg) => call("config/validate", { method: "POST", body: cfg }),
      validatePath: (path) => call("config/validate-path", { method: "POST", body: { path } }),
      // hardware (:255-317)
      hardwareInfo: () => call("hardware/info"),
      presets: () => call("hardware/presets"),
      checkPreset: (name) => call(`hardware/presets/${id(name)}/check`),
      detect: () => call("hardware/detect", { method: "POST" }),
      // install (:319-407)
      installStatus: (cacheDir) => call("install/status", { query: { cache_dir: cacheDir } }),
      checkPath: (path) => call("install/check-path", { query: { path } }),
      startInstall: (req) => call("install/setup", { method: "POST", body: req }),
      installTasks: () => call("install/tasks"),
      installTask: (taskId) => call(`install/tasks/${id(taskId)}`),
      cancelInstall: (taskId) => call(`install/tasks/${id(taskId)}/cancel`, { method: "POST" }),
      installLogs: (taskId, tail) => call(`install/tasks/${id(taskId)}/logs`, { query: { tail } }),
      // server (:409-456)
      serverStatus: () => call("server/status"),
      startServer: (req) => call("server/start", { method: "POST", body: req || {} }),
      stopServer: (req) => call("server/stop", { method: "POST", body: req || { force: false, timeout: 30 } }),
      restartServer: (req) => call("server/restart", { method: "POST", body: req || {} }),
      serverLogs: (lines) => call("server/logs", { query: { lines: lines || 200 } }),
    };
  }

  // websocket URLs (app/main.py /ws/logs, /ws/install/{id})
  function wsUrl(loc, path) {
    return `${loc.protocol === "https:" ? "wss" : "ws"}://${loc.host}${path}`;
  }

  // ---------------------------------------------------------------------- validation
  const SERVICE_NAME_RE = /^[a-zA-Z0-9](?:[a-zA-Z0-9-]{0,61}[a-zA-Z0-9])?$/;

  function portError(raw) {
    const s = String(raw == null ? "" : raw).trim();
    if (!s) return "port is required";
    if (!/^\d+$/.test(s)) return "port must be a number";
    const p = parseInt(s, 10);
    if (p < 1024 || p > 65535) return "port must be between 1024 and 65535";
    return null;
  }

  function serviceNameError(raw) {
    const s = String(raw == null ? "" : raw).trim();
    if (!s) return "service name is required";
    if (s.length < 3 || s.length > 63) return "service name must be 3-63 characters";
    if (!SERVICE_NAME_RE.test(s)) return "letters, digits and '-' only; no leading or trailing '-'";
    return null;
  }

  function pathError(raw) {
    const s = String(raw == null ? "" : raw).trim();
    if (!s) return "path is required";
    if (/[\u0000]/.test(s)) return "path contains a NUL byte";
    return null;
  }

  // ---------------------------------------------------------------------- wizard model
  const WIZARD_STEPS = [
    { id: "welcome", name: "Basics", path: "/setup/welcome" },
    { id: "hardware", name: "Hardware", path: "/setup/hardware" },
    { id: "config", name: "Services", path: "/setup/config" },
    { id: "install", name: "Install", path: "/setup/install" },
  ];

  // service profiles the generator knows (app/presets.py Config.minimal/light_weight/basic/brave)
  const SERVICE_PRESETS = [
    { id: "minimal", name: "Minimal", services: ["ocr"], recommended: false,
      description: "Text recognition only: classify documents and receipts, search text in photos.",
      requirements: "smallest footprint" },
    { id: "light_weight", name: "Light", services: ["ocr", "clip", "face"], recommended: true,
      description: "OCR, semantic search, face recognition and scene classification.",
      requirements: "balanced; fits most machines", clipModels: ["MobileCLIP2-S2", "CN-CLIP_ViT-B-16"] },
    { id: "basic", name: "Basic", services: ["ocr", "clip", "face", "vlm"], recommended: true,
      description: "Everything in Light plus image captioning (FastVLM).",
      requirements: "full feature set", clipModels: ["MobileCLIP2-S4", "CN-CLIP_ViT-L-14"] },
    { id: "brave", name: "Brave", services: ["ocr", "clip", "face", "vlm"], recommended: false,
      description: "Largest models of every service (BioCLIP-2, antelopev2, PP-OCRv5 server).",
      requirements: "an MI355X-class GPU" },
  ];

  const SERVICES = [
    { id: "ocr", name: "Text recognition", package: "lumen-ocr", description: "DB detection + CTC recognition" },
    { id: "clip", name: "Image/text understanding", package: "lumen-clip", description: "embeddings, zero-shot labels, search" },
    { id: "face", name: "Face recognition", package: "lumen-face", description: "detection, landmarks, 512-d identity embeddings" },
    { id: "vlm", name: "Image description", package: "lumen-vlm", description: "captions and chat about an image" },
  ];

  const DEFAULT_WIZARD = {
    installPath: "", region: "other", serviceName: "lumen-ai", port: 50051,
    hardwarePreset: null, servicePreset: null, clipModel: null, configGenerated: false, configPath: null,
    configKey: null, installTask: null, installationComplete: false,
  };

  // The last wizard step a state may show (WizardLayout's guards): basics must validate
  // before hardware, a preset must be chosen before services, a config generated before
  // install.  Returns the path to redirect to, or null when `stepId` is allowed.
  function wizardGate(state, stepId) {
    const s = Object.assign({}, DEFAULT_WIZARD, state || {});
    const order = WIZARD_STEPS.map((x) => x.id);
    const want = order.indexOf(stepId);
    if (want < 0) return WIZARD_STEPS[0].path;
    const basicsOk = !pathError(s.installPath) && !portError(s.port) && !serviceNameError(s.serviceName);
    const reached = !basicsOk ? 0 : !s.hardwarePreset ? 1 : !s.configGenerated ? 2 : 3;
    return want <= reached ? null : WIZARD_STEPS[reached].path;
  }

  // identity of a generated config: changing any input invalidates it (Config.tsx:182-193)
  function configKey(s) {
    return [s.servicePreset, s.hardwarePreset, s.installPath, s.region, String(s.port), s.serviceName,
      s.clipModel || ""].join("|");
  }

  function generateRequest(s) {
    return { cache_dir: s.installPath, preset: s.hardwarePreset, region: s.region,
      service_name: String(s.serviceName).trim(), port: parseInt(s.port, 10), config_type: s.servicePreset,
      clip_model: s.clipModel || null };
  }

  const TERMINAL = ["completed", "failed", "cancelled"];
  const taskDone = (status) => TERMINAL.indexOf(String(status)) >= 0;

  // badge colour for any status string the API returns
  function statusKind(status) {
    switch (String(status)) {
      case "completed": case "available": case "healthy": case "running": case "ok": case "ready":
        return "ok";
      case "failed": case "unhealthy": case "error": case "missing": case "incompatible":
        return "err";
      case "pending": case "cancelled": case "skipped": case "unknown": case "not_checked":
        return "";
      default:
        return "warn";
    }
  }

  function formatDuration(sec) {
    if (sec == null || !isFinite(sec)) return "—";
    const s = Math.max(0, Math.floor(sec));
    const d = Math.floor(s / 86400), h = Math.floor((s % 86400) / 3600), m = Math.floor((s % 3600) / 60);
    if (d) return `${d}d ${h}h`;
    if (h) return `${h}h ${m}m`;
    if (m) return `${m}m ${s % 60}s`;
    return `${s}s`;
  }

  // keep the tail of a log list bounded (Server/Install views stream lines into it)
  function appendBounded(lines, more, cap) {
    const out = lines.concat(more);
    return out.length > cap ? out.slice(out.length - cap) : out;
  }

  // ---------------------------------------------------------------------- persisted state
  // localStorage-like store with JSON values and defaults (WizardProvider persists to
  // sessionStorage, useLumenSession to localStorage)
  function createStore(storage, key, defaults) {
    let s = Object.assign({}, defaults || {});
    try { Object.assign(s, JSON.parse(storage.getItem(key) || "{}")); } catch (e) { /* corrupt: defaults */ }
    const save = () => { try { storage.setItem(key, JSON.stringify(s)); } catch (e) { /* quota */ } };
    return {
      get: (k) => s[k],
      all: () => Object.assign({}, s),
      set(patch) { s = Object.assign({}, s, patch); save(); return s; },
      reset(patch) { s = Object.assign({}, defaults || {}, patch || {}); save(); return s; },
    };
  }

  // most-recently-used install paths for the Open view
  function rememberPath(list, p, cap) {
    const n = String(p).trim();
    if (!n) return list.slice();
    return [n].concat(list.filter((x) => x !== n)).slice(0, cap || 6);
  }

  return {
    ApiError, errorKind, errorMessage, describeUiError, createApi, wsUrl, query,
    portError, serviceNameError, pathError,
    WIZARD_STEPS, SERVICE_PRESETS, SERVICES, DEFAULT_WIZARD, wizardGate, configKey, generateRequest,
    taskDone, statusKind, formatDuration, appendBounded, createStore, rememberPath,
  };
});
