"""Shared-memory request channel: serving front ends -> one GPU engine process per device.

Python side of ``csrc/host/shm_channel.cpp`` (C ABI, ``_lumen_host.so``).  The region lives in a
``memfd`` created by the launcher and handed to every child at spawn
(:class:`multiprocessing.resource_sharer.DupFd`), so nothing depends on the size of
``/dev/shm``; each process maps it at its own address.  A request occupies one slot from
submission to result: payload (a numpy array -- a decoded uint8 HWC image, int64 token ids --
or opaque bytes), a ``kind`` code, a short JSON ``meta`` string; the engine answers with an
array or bytes in the slot's result area.

Front end (any thread)::

    res = ch.call("image_u8", img_hwc, meta={"k": 5})      # blocks this thread only (futex)

Engine::

    for slot in ch.pop_batch(max_n=256, wait_ms=100, linger_us=2000):
        arr, meta = ch.request(slot)                       # zero-copy view into the slot
        ...; ch.complete(slot, result_array)

Streaming (a VLM's tokens): the engine appends partial records to a running slot
(``ch.partial(slot, b"...")``) and the front end iterates ``ch.call_stream(...)``, which yields
``("partial", bytes)`` as each record lands and ends with ``("result", value)``.

The reference has no cross-process serving path at all (``src/lumen/server.py:232-235``: one
process, a 10-thread gRPC pool, batch 1).
"""
from __future__ import annotations

import ctypes
import itertools
import json
import mmap
import os
import threading
from dataclasses import dataclass
from typing import Any, Optional, Sequence

import numpy as np

from .._native import load_host

FREE, FILLING, QUEUED, RUNNING, DONE, ERROR, ABANDONED_Q, ABANDONED_R = range(8)

_DTYPES = [np.uint8, np.float32, np.int64, np.int32, np.float16, np.int8]
BYTES = 255            # dtype code of an opaque byte payload / result


class ChannelError(RuntimeError):
    """The engine reported an error for this request (message from the engine)."""


class EngineUnavailable(RuntimeError):
    """No engine answered in time (dead, hung or restarting): maps to gRPC UNAVAILABLE."""


class _SlotDesc(ctypes.Structure):
    """Mirror of ``Slot`` in shm_channel.cpp (the state word is read through the C ABI)."""
    _fields_ = [("state", ctypes.c_uint32), ("kind", ctypes.c_uint32), ("dtype", ctypes.c_uint32),
                ("ndim", ctypes.c_uint32), ("shape", ctypes.c_uint32 * 4), ("nbytes", ctypes.c_uint64),
                ("rdtype", ctypes.c_uint32), ("rndim", ctypes.c_uint32), ("rshape", ctypes.c_uint32 * 4),
                ("rbytes", ctypes.c_uint64), ("status", ctypes.c_uint32), ("gen", ctypes.c_uint32),
                ("tag", ctypes.c_uint64), ("meta", ctypes.c_char * 128), ("pseq", ctypes.c_uint32),
                ("pflags", ctypes.c_uint32), ("plen", ctypes.c_uint64), ("roff", ctypes.c_uint64),
                ("_pad", ctypes.c_char * 16)]


def _lib():
    lib = load_host()
    if lib is None or not hasattr(lib, "lumen_ch_init"):
        raise RuntimeError("lumen host library without the shm channel (run lumen_amd._build)")
    if not getattr(lib, "_ch_typed", False):
        vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
        sig = {"lumen_ch_region_bytes": (u64, [i32, u64, u64]), "lumen_ch_init": (i32, [vp, i32, u64, u64]),
               "lumen_ch_check": (i32, [vp]), "lumen_ch_nslots": (i32, [vp]), "lumen_ch_slot_bytes": (u64, [vp]),
               "lumen_ch_result_bytes": (u64, [vp]), "lumen_ch_total_bytes": (u64, [vp]),
               "lumen_ch_slot_desc_off": (u64, [vp, i32]), "lumen_ch_payload_off": (u64, [vp, i32]),
               "lumen_ch_result_off": (u64, [vp, i32]), "lumen_ch_slot_desc_size": (i32, []),
               "lumen_ch_slot_state": (i32, [vp, i32]), "lumen_ch_depth": (i32, [vp]),
               "lumen_ch_acquire": (i32, [vp, i32]), "lumen_ch_submit": (i32, [vp, i32, u64]),
               "lumen_ch_wait": (i32, [vp, i32, i32]), "lumen_ch_release": (None, [vp, i32]),
               "lumen_ch_abandon": (i32, [vp, i32]),
               "lumen_ch_pop_batch": (i32, [vp, ctypes.POINTER(ctypes.c_int), i32, i32, i32]),
               "lumen_ch_complete": (None, [vp, i32, i32]), "lumen_ch_heartbeat": (None, [vp, u32]),
               "lumen_ch_heartbeat_age_ns": (u64, [vp]), "lumen_ch_engine_start": (i32, [vp, u32]),
               "lumen_ch_partial": (i32, [vp, i32, vp, u64]), "lumen_ch_plen": (u64, [vp, i32]),
               "lumen_ch_wait_partial": (i32, [vp, i32, u64, i32])}
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        if lib.lumen_ch_slot_desc_size() != ctypes.sizeof(_SlotDesc):
            raise RuntimeError(f"shm channel slot layout mismatch: C {lib.lumen_ch_slot_desc_size()} "
                               f"vs Python {ctypes.sizeof(_SlotDesc)} bytes")
        lib._ch_typed = True
    return lib


@dataclass
class ChannelSpec:
    """Picklable handle to a channel for a spawned child (the fd travels as a DupFd)."""
    name: str
    fd: Any
    size: int
    kinds: tuple


class ShmChannel:
    def __init__(self, name: str, fd: int, size: int, kinds: Sequence[str], create: bool = False,
                 nslots: int = 0, slot_bytes: int = 0, result_bytes: int = 0):
        self.lib = _lib()
        self.name = name
        self.fd = fd
        self.size = size
        self.kinds = tuple(kinds)
        self._kind_code = {k: i for i, k in enumerate(self.kinds)}
        self.mm = mmap.mmap(fd, size, flags=mmap.MAP_SHARED)
        self._buf = (ctypes.c_char * size).from_buffer(self.mm)
        self.base = ctypes.addressof(self._buf)
        if create:
            if self.lib.lumen_ch_init(self.base, nslots, slot_bytes, result_bytes) != 0:
                raise RuntimeError("lumen_ch_init failed")
        if self.lib.lumen_ch_check(self.base) != 0:
            raise RuntimeError(f"channel {name}: not an initialised lumen channel")
        self.nslots = self.lib.lumen_ch_nslots(self.base)
        self.slot_bytes = int(self.lib.lumen_ch_slot_bytes(self.base))
        self.result_bytes = int(self.lib.lumen_ch_result_bytes(self.base))
        self._desc = [_SlotDesc.from_address(self.base + self.lib.lumen_ch_slot_desc_off(self.base, i))
                      for i in range(self.nslots)]
        self._pay = [int(self.lib.lumen_ch_payload_off(self.base, i)) for i in range(self.nslots)]
        self._res = [int(self.lib.lumen_ch_result_off(self.base, i)) for i in range(self.nslots)]
        self._seq = itertools.count(1)
        self._registered = None

    # ------------------------------------------------------------------ lifecycle
    @classmethod
    def create(cls, name: str, kinds: Sequence[str], nslots: int = 128, slot_bytes: int = 8 << 20,
               result_bytes: int = 64 << 10) -> "ShmChannel":
        lib = _lib()
        size = int(lib.lumen_ch_region_bytes(nslots, slot_bytes, result_bytes))
        fd = os.memfd_create(f"lumen-ch-{name}", os.MFD_CLOEXEC)
        os.ftruncate(fd, size)
        return cls(name, fd, size, kinds, create=True, nslots=nslots, slot_bytes=slot_bytes,
                   result_bytes=result_bytes)

    def spec(self) -> ChannelSpec:
        """A one-shot handle for ONE child process (build a new one per spawn)."""
        from multiprocessing.resource_sharer import DupFd

        return ChannelSpec(self.name, DupFd(self.fd), self.size, self.kinds)

    @classmethod
    def attach(cls, spec: ChannelSpec) -> "ShmChannel":
        fd = spec.fd.detach() if hasattr(spec.fd, "detach") else int(spec.fd)
        return cls(spec.name, fd, spec.size, spec.kinds)

    def close(self) -> None:
        if self._registered is not None:
            try:
                import torch

                torch.cuda.cudart().cudaHostUnregister(self._registered)
            except Exception:  # noqa: BLE001
                pass
            self._registered = None
        self._desc = []
        del self._buf
        try:
            self.mm.close()
        except BufferError:   # a view is still alive: the mapping goes with the process
            pass
        try:
            os.close(self.fd)
        except OSError:
            pass

    def register_host(self) -> bool:
        """Pin the region for DMA (engine side): device copies read payload slots directly."""
        try:
            import torch

            if not torch.cuda.is_available():
                return False
            err = torch.cuda.cudart().cudaHostRegister(self.base, self.size, 0)
            if int(err) == 0:
                self._registered = self.base
                return True
        except Exception:  # noqa: BLE001 - pinning is an optimisation only
            pass
        return False

    # ------------------------------------------------------------------ helpers
    def depth(self) -> int:
        return int(self.lib.lumen_ch_depth(self.base))

    def heartbeat_age(self) -> float:
        ns = int(self.lib.lumen_ch_heartbeat_age_ns(self.base))
        return float("inf") if ns >= (1 << 63) else ns / 1e9

    def _payload(self, slot: int, nbytes: int) -> np.ndarray:
        return np.frombuffer(self.mm, np.uint8, nbytes, self._pay[slot])

    def _result(self, slot: int, nbytes: int, off: int = 0) -> np.ndarray:
        return np.frombuffer(self.mm, np.uint8, nbytes, self._res[slot] + off)

    @staticmethod
    def _code(x) -> tuple:
        if isinstance(x, (bytes, bytearray, memoryview)):
            return BYTES, ()
        a = np.asarray(x)
        for i, d in enumerate(_DTYPES):
            if a.dtype == d:
                return i, a.shape
        raise TypeError(f"shm channel: unsupported dtype {a.dtype}")

    @staticmethod
    def _decode(buf: np.ndarray, code: int, shape, copy: bool):
        if code == BYTES:
            return bytes(buf)
        a = buf.view(_DTYPES[code]).reshape(shape)
        return a.copy() if copy else a

    # ------------------------------------------------------------------ front end
    def _fill_submit(self, kind: str, payload, meta: Optional[dict], timeout: float) -> int:
        """Acquire a slot, write the request and queue it; returns the slot (released on error)."""
        lib, base = self.lib, self.base
        slot = lib.lumen_ch_acquire(base, int(timeout * 1000))
        if slot < 0:
            raise EngineUnavailable(f"channel {self.name}: no free slot in {timeout:.0f} s")
        try:
            d = self._desc[slot]
            code, shape = self._code(payload)
            if code == BYTES:
                nbytes = len(payload)
                if nbytes > self.slot_bytes:
                    raise ValueError(f"payload {nbytes} B exceeds the channel slot ({self.slot_bytes} B)")
                self._payload(slot, nbytes)[:] = np.frombuffer(payload, np.uint8)
            else:
                a = np.ascontiguousarray(payload)
                nbytes = a.nbytes
                if nbytes > self.slot_bytes:
                    raise ValueError(f"payload {nbytes} B exceeds the channel slot ({self.slot_bytes} B)")
                if len(shape) > 4:
                    raise ValueError("payload rank > 4")
                self._payload(slot, nbytes)[:] = a.reshape(-1).view(np.uint8)
                for i, s in enumerate(shape):
                    d.shape[i] = s
            d.kind = self._kind_code[kind]
            d.dtype = code
            d.ndim = len(shape)
            d.nbytes = nbytes
            m = json.dumps(meta, separators=(",", ":")).encode() if meta else b""
            if len(m) > 127:
                raise ValueError("request meta exceeds 127 bytes")
            d.meta = m
            tag = (os.getpid() << 32) | (next(self._seq) & 0xFFFFFFFF)
            if lib.lumen_ch_submit(base, slot, tag) != 0:
                raise RuntimeError("shm channel submit failed")
        except BaseException:
            lib.lumen_ch_release(base, slot)
            raise
        return slot

    def _final(self, slot: int, st: int):
        d = self._desc[slot]
        rb = int(d.rbytes)
        buf = np.frombuffer(self.mm, np.uint8, rb, self._res[slot] + int(d.roff))
        if st == ERROR:
            raise ChannelError(bytes(buf).decode("utf-8", "replace"))
        return self._decode(buf, d.rdtype, tuple(d.rshape[:d.rndim]), copy=True)

    def call(self, kind: str, payload, meta: Optional[dict] = None, timeout: float = 120.0):
        """Submit one request and wait for its result (array or bytes).  Raises
        :class:`ChannelError` with the engine's message, :class:`EngineUnavailable` on timeout."""
        lib, base = self.lib, self.base
        slot = self._fill_submit(kind, payload, meta, timeout)
        try:
            st = lib.lumen_ch_wait(base, slot, int(timeout * 1000))
            if st < 0:
                # the engine may still write this slot: abandon it (the engine frees it when it
                # pops or completes it; a finished one is freed here) instead of releasing it
                lib.lumen_ch_abandon(base, slot)
                slot = -1
                raise EngineUnavailable(f"channel {self.name}: no answer in {timeout:.0f} s")
            return self._final(slot, st)
        finally:
            if slot >= 0:
                lib.lumen_ch_release(base, slot)

    def call_stream(self, kind: str, payload, meta: Optional[dict] = None, timeout: float = 120.0):
        """Submit one streaming request; yields ``("partial", bytes)`` for every record the engine
        appends, as it lands, then ``("result", value)``.  ``timeout`` bounds the wait for EACH
        record.  Closing the generator early (a cancelled client) abandons the slot: the engine's
        next append to it fails and it stops generating."""
        lib, base = self.lib, self.base
        slot = self._fill_submit(kind, payload, meta, timeout)
        done = False
        seen = 0
        try:
            while True:
                st = lib.lumen_ch_wait_partial(base, slot, seen, int(timeout * 1000))
                if st < 0:
                    raise EngineUnavailable(f"channel {self.name}: no answer in {timeout:.0f} s")
                end = int(lib.lumen_ch_plen(base, slot))
                off = self._res[slot]
                while seen < end:
                    n = int(np.frombuffer(self.mm, np.uint32, 1, off + seen)[0])
                    yield "partial", bytes(self.mm[off + seen + 4: off + seen + 4 + n])
                    seen += (4 + n + 7) & ~7
                if st in (DONE, ERROR) and int(lib.lumen_ch_plen(base, slot)) == seen:
                    done = True
                    value = self._final(slot, st)
                    yield "result", value
                    return
        finally:
            if done:
                lib.lumen_ch_release(base, slot)
            else:
                lib.lumen_ch_abandon(base, slot)

    # ------------------------------------------------------------------ engine
    def engine_start(self) -> int:
        """A (re)started engine: new generation, fail what a predecessor left running."""
        return int(self.lib.lumen_ch_engine_start(self.base, os.getpid()))

    def heartbeat(self) -> None:
        self.lib.lumen_ch_heartbeat(self.base, os.getpid())

    def pop_batch(self, max_n: int, wait_ms: int = 100, linger_us: int = 0) -> list[int]:
        """Engine: up to max_n RUNNING slots (thread-safe: several batch loops may pop)."""
        k = min(max_n, self.nslots)
        out = (ctypes.c_int * k)()
        n = self.lib.lumen_ch_pop_batch(self.base, out, k, int(wait_ms), int(linger_us))
        return [out[i] for i in range(n)]

    def tag(self, slot: int) -> int:
        """Submitter tag of a slot: (front-end pid << 32) | sequence."""
        return int(self._desc[slot].tag)

    def request(self, slot: int):
        """(kind, payload view, meta dict) of a RUNNING slot (the view is valid until complete())."""
        d = self._desc[slot]
        buf = self._payload(slot, int(d.nbytes))
        meta = json.loads(d.meta.decode()) if d.meta else {}
        return self.kinds[d.kind], self._decode(buf, d.dtype, tuple(d.shape[:d.ndim]), copy=False), meta

    def partial(self, slot: int, data: bytes) -> int:
        """Engine: append one partial record to a running slot (streaming).  0 ok, -1 the result
        area is full (record dropped), -2 the front end abandoned the request: stop producing."""
        data = bytes(data)
        return int(self.lib.lumen_ch_partial(self.base, slot, data if data else None, len(data)))

    def complete(self, slot: int, result=None, error: Optional[str] = None) -> None:
        d = self._desc[slot]
        # the final result goes after any partial records (a streaming front end may still read them)
        roff = (int(self.lib.lumen_ch_plen(self.base, slot)) + 63) & ~63
        room = self.result_bytes - roff
        if error is not None:
            msg = error.encode("utf-8", "replace")[: max(room, 0)]
            self._result(slot, len(msg), roff)[:] = np.frombuffer(msg, np.uint8)
            d.roff = roff
            d.rbytes, d.rdtype, d.rndim = len(msg), BYTES, 0
            self.lib.lumen_ch_complete(self.base, slot, 1)
            return
        code, shape = self._code(result if result is not None else b"")
        if code == BYTES:
            raw = bytes(result or b"")
            nb = len(raw)
            if nb > room:
                return self.complete(slot, error=f"result {nb} B exceeds the channel result area")
            self._result(slot, nb, roff)[:] = np.frombuffer(raw, np.uint8)
        else:
            a = np.ascontiguousarray(result)
            nb = a.nbytes
            if nb > room or a.ndim > 4:
                return self.complete(slot, error=f"result {a.shape} exceeds the channel result area")
            self._result(slot, nb, roff)[:] = a.reshape(-1).view(np.uint8)
            for i, s in enumerate(a.shape):
                d.rshape[i] = s
        d.roff = roff
        d.rbytes, d.rdtype, d.rndim = nb, code, len(shape)
        self.lib.lumen_ch_complete(self.base, slot, 0)


class ChannelGroup:
    """The channels of one service across its engines (one per GPU): each call goes to the
    least-loaded live engine (queue depth from the region; a stale heartbeat skips an engine)."""

    def __init__(self, channels: Sequence[ShmChannel], dead_after_s: float = 30.0):
        self.channels = list(channels)
        self.dead_after_s = dead_after_s
        self._rr = itertools.count()
        self._lock = threading.Lock()

    def pick(self) -> ShmChannel:
        live = [c for c in self.channels if c.heartbeat_age() < self.dead_after_s] or self.channels
        with self._lock:
            start = next(self._rr)
        n = len(live)
        return min((live[(start + i) % n] for i in range(n)), key=lambda c: c.depth())

    def call(self, kind: str, payload, meta: Optional[dict] = None, timeout: float = 120.0):
        return self.pick().call(kind, payload, meta, timeout)
