"""Host shared-memory step bus from TP rank 0 to its follower ranks (``csrc/host/step_bus.cpp``).

:class:`lumen_amd.runtime.engine.TPSync` sends every engine step through it when the whole TP
group lives on one node (always, for :class:`~lumen_amd.parallel.tp.TPServingGroup`): the
followers' hosts read the step descriptor straight from shared memory -- no device collective,
no device->host copy per token -- and launch their decode graphs while the leader launches its
own.  The bus is created collectively: rank 0 makes a uniquely named region, the followers map
it, and rank 0 unlinks the name once every rank holds a mapping (nothing is left in /dev/shm
even if a rank dies later).
"""
from __future__ import annotations

import ctypes
import os
import uuid
from typing import Optional

import numpy as np

from .._native import load_host


class BusClosed(RuntimeError):
    """The writer closed the bus (engine shut down)."""


def _lib():
    lib = load_host()
    if lib is None or not hasattr(lib, "lumen_bus_create"):
        raise RuntimeError("lumen host library without the step bus (run lumen_amd._build)")
    if not getattr(lib, "_bus_typed", False):
        vp, u64, i32, i64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
        sig = {"lumen_bus_region_bytes": (u64, [i32, u64]),
               "lumen_bus_create": (vp, [ctypes.c_char_p, i32, u64, i32]),
               "lumen_bus_open": (vp, [ctypes.c_char_p]), "lumen_bus_unlink": (i32, [ctypes.c_char_p]),
               "lumen_bus_unmap": (None, [vp]), "lumen_bus_slot_bytes": (u64, [vp]),
               "lumen_bus_writer_pid": (u32, [vp]), "lumen_bus_head": (u64, [vp]),
               "lumen_bus_publish": (i32, [vp, vp, u64, i32]),
               "lumen_bus_next": (i64, [vp, i32, vp, u64, i32, i32]), "lumen_bus_close": (None, [vp])}
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        lib._bus_typed = True
    return lib


def available() -> bool:
    try:
        _lib()
        return True
    except RuntimeError:
        return False


class StepBus:
    """One writer, ``nreaders`` readers.  ``reader`` is None for the writer, else 0..nreaders-1."""

    def __init__(self, name: str, reader: Optional[int], nslots: int = 64, slot_bytes: int = 1 << 18,
                 nreaders: int = 1):
        self.lib = _lib()
        self.name = name.encode()
        self.reader = reader
        if reader is None:
            self.base = self.lib.lumen_bus_create(self.name, int(nslots), int(slot_bytes), int(nreaders))
        else:
            self.base = self.lib.lumen_bus_open(self.name)
        if not self.base:
            raise RuntimeError(f"step bus {name}: {'create' if reader is None else 'open'} failed")
        self.slot_bytes = int(self.lib.lumen_bus_slot_bytes(self.base))
        self.buf = np.empty(self.slot_bytes, np.uint8)
        self.closed = False

    @staticmethod
    def unique_name() -> str:
        return f"/lumen_tp_{os.getpid()}_{uuid.uuid4().hex[:12]}"

    def unlink(self) -> None:
        self.lib.lumen_bus_unlink(self.name)

    def publish(self, data, timeout_ms: int = 60000) -> None:
        """Writer: ``data`` = bytes / contiguous numpy array (at most ``slot_bytes``)."""
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data)
            ptr, n = a.ctypes.data, a.nbytes
        else:
            a = bytes(data)
            ptr, n = ctypes.cast(ctypes.c_char_p(a), ctypes.c_void_p).value, len(a)
        r = self.lib.lumen_bus_publish(self.base, ptr, n, int(timeout_ms))
        if r == -1:
            raise TimeoutError("step bus: a follower stopped reading")
        if r == -2:
            raise ValueError(f"step bus: {n} bytes > slot {self.slot_bytes} or bus closed")

    def next(self, timeout_ms: int = 1000, spin_us: int = 200) -> Optional[memoryview]:
        """Reader: the next message (a view of this reader's buffer, valid until the next call),
        or None on timeout."""
        n = self.lib.lumen_bus_next(self.base, int(self.reader), self.buf.ctypes.data, self.slot_bytes,
                                    int(timeout_ms), int(spin_us))
        if n == -1:
            return None
        if n == -2:
            raise BusClosed("step bus closed")
        if n < 0:
            raise RuntimeError(f"step bus read failed ({n})")
        return memoryview(self.buf)[:n]

    def writer_alive(self) -> bool:
        pid = int(self.lib.lumen_bus_writer_pid(self.base))
        try:
            os.kill(pid, 0)
            return True
        except ProcessLookupError:
            return False
        except PermissionError:
            return True

    def close(self) -> None:
        """Writer: wake every reader with BusClosed.  Both sides: drop the mapping."""
        if self.closed:
            return
        self.closed = True
        if self.reader is None:
            self.lib.lumen_bus_close(self.base)
        self.lib.lumen_bus_unmap(self.base)
        self.base = None
