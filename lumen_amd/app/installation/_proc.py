"""Child-process helper shared by the installers: stream output lines to a log callback,
stop the process group when a cancel event is set, return (rc, tail of output)."""
from __future__ import annotations

import os
import signal
import subprocess
import threading
from typing import Callable, Optional, Sequence

LogFn = Callable[[str], None]


class Cancelled(Exception):
    pass


def run(cmd: Sequence[str], log: Optional[LogFn] = None, cancel: Optional[threading.Event] = None,
        env: Optional[dict] = None, cwd: Optional[str] = None, timeout: Optional[float] = None) -> tuple[int, list[str]]:
    tail: list[str] = []
    try:
        p = subprocess.Popen(list(cmd), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=cwd,
                             start_new_session=True)
    except OSError as e:
        if log:
            log(f"cannot start {cmd[0]}: {e}")
        return 127, [str(e)]
    timer = None
    if timeout:
        timer = threading.Timer(timeout, lambda: _kill(p))
        timer.start()
    try:
        for raw in iter(p.stdout.readline, b""):
            line = raw.decode("utf-8", "replace").rstrip()
            tail = (tail + [line])[-50:]
            if log:
                log(line)
            if cancel is not None and cancel.is_set():
                _kill(p)
                p.wait(timeout=30)
                raise Cancelled()
        return p.wait(), tail
    finally:
        if timer:
            timer.cancel()


def _kill(p: subprocess.Popen) -> None:
    try:
        os.killpg(p.pid, signal.SIGTERM)     # the child's own process group (start_new_session)
    except (ProcessLookupError, PermissionError):
        pass
