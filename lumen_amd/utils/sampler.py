"""Statistical stack sampler for the serving processes (all Python threads -- the gRPC handler pool
included, which cProfile, bound to one thread, never sees).  Every ``interval_s`` it records each
thread's innermost frame and innermost ``lumen_amd`` frame; :meth:`report` writes the hottest ones.

Enabled in the front-end / engine processes by ``LUMEN_SAMPLE_DIR=<dir>`` (hub/server.py,
parallel/engine.py): ``<dir>/<name>-<pid>.txt`` at process exit.  The reference has no serving
profiler; this is the MI355X box's way to see where a CPU-bound front end spends its time.
"""
from __future__ import annotations

import collections
import os
import sys
import threading


class StackSampler:
    def __init__(self, interval_s: float = 0.002):
        self.interval = interval_s
        self.leaf = collections.Counter()
        self.own = collections.Counter()
        self.samples = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="lumen-sampler", daemon=True)

    def start(self) -> "StackSampler":
        self._t.start()
        return self

    def _run(self) -> None:
        me = threading.get_ident()
        while not self._stop.wait(self.interval):
            for tid, f in sys._current_frames().items():
                if tid == me:
                    continue
                self.samples += 1
                code = f.f_code
                self.leaf[f"{os.path.basename(code.co_filename)}:{f.f_lineno} {code.co_name}"] += 1
                g = f
                while g is not None and "lumen_amd" not in g.f_code.co_filename:
                    g = g.f_back
                if g is not None:
                    c = g.f_code
                    self.own[f"{os.path.relpath(c.co_filename, os.path.dirname(os.path.dirname(__file__)))}:"
                             f"{g.f_lineno} {c.co_name}"] += 1

    def report(self, path: str, top: int = 40) -> None:
        self._stop.set()
        self._t.join(timeout=1.0)
        n = max(self.samples, 1)
        with open(path, "w") as fh:
            fh.write(f"# {self.samples} thread samples every {self.interval * 1e3:.1f} ms "
                     f"(idle threads blocked in waits count too)\n# innermost frame:\n")
            for k, v in self.leaf.most_common(top):
                fh.write(f"{100.0 * v / n:6.2f}%  {k}\n")
            fh.write("# innermost lumen_amd frame:\n")
            for k, v in self.own.most_common(top):
                fh.write(f"{100.0 * v / n:6.2f}%  {k}\n")


def maybe_start(name: str):
    """Start a sampler when LUMEN_SAMPLE_DIR is set; returns a ``stop()`` callable writing the report."""
    d = os.environ.get("LUMEN_SAMPLE_DIR")
    if not d:
        return lambda: None
    os.makedirs(d, exist_ok=True)
    s = StackSampler(float(os.environ.get("LUMEN_SAMPLE_INTERVAL_MS", "2")) / 1e3).start()

    def stop():
        s.report(os.path.join(d, f"{name}-{os.getpid()}.txt"))
    return stop
