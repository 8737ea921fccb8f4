"""Host shared-memory TP step bus (csrc/host/step_bus.cpp, parallel/step_bus.py): one writer, two
reader processes; every reader sees every message in order through ring wrap-around (more
messages than slots), a writer blocked on a full ring times out instead of hanging, and closing
the bus wakes readers with BusClosed after the pending messages."""
import multiprocessing as mp

import numpy as np
import pytest

from lumen_amd.parallel import step_bus

pytestmark = pytest.mark.skipif(not step_bus.available(), reason="host library without the step bus")


def _reader(name, idx, n, q):
    bus = step_bus.StepBus(name, idx)
    got = []
    try:
        for _ in range(n):
            m = bus.next(timeout_ms=20000)
            got.append(None if m is None else bytes(m))
        try:
            while bus.next(timeout_ms=20000) is not None:
                pass
            closed = False
        except step_bus.BusClosed:
            closed = True
        q.put((idx, got, closed))
    finally:
        bus.close()


def test_step_bus_two_readers_wraparound_and_close():
    name = step_bus.StepBus.unique_name()
    w = step_bus.StepBus(name, None, nslots=4, slot_bytes=4096, nreaders=2)
    n = 37
    msgs = [np.arange(k % 50 + 1, dtype=np.int32) * (k + 1) for k in range(n)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reader, args=(name, i, n, q)) for i in range(2)]
    for p in ps:
        p.start()
    try:
        for m in msgs:
            w.publish(m, timeout_ms=20000)
        w.close()
        res = sorted(q.get(timeout=60) for _ in ps)
    finally:
        for p in ps:
            p.join(30)
        w.unlink()
    for idx, got, closed in res:
        assert closed
        assert got == [m.tobytes() for m in msgs]


def test_step_bus_full_ring_times_out_and_rejects_oversize():
    name = step_bus.StepBus.unique_name()
    w = step_bus.StepBus(name, None, nslots=2, slot_bytes=256, nreaders=1)
    try:
        w.publish(b"a")
        w.publish(b"b")
        with pytest.raises(TimeoutError):          # the one reader never consumed: ring full
            w.publish(b"c", timeout_ms=50)
        with pytest.raises(ValueError):
            w.publish(b"x" * 1000)
        r = step_bus.StepBus(name, 0)
        assert bytes(r.next(timeout_ms=100)) == b"a"
        w.publish(b"c", timeout_ms=1000)            # a slot freed
        assert bytes(r.next(timeout_ms=100)) == b"b" and bytes(r.next(timeout_ms=100)) == b"c"
        assert r.next(timeout_ms=20) is None          # nothing pending: timeout
        r.close()
    finally:
        w.close()
        w.unlink()


def test_h2d_cpu_paths():
    """utils.h2d on a CPU target: lists, numpy arrays and tensors keep values and dtypes."""
    import torch

    from lumen_amd.utils.h2d import h2d

    assert torch.equal(h2d([[1, 2], [3, 4]], "cpu", torch.long), torch.tensor([[1, 2], [3, 4]]))
    a = np.arange(6, dtype=np.float32).reshape(2, 3)[:, ::2]          # non-contiguous view
    t = h2d(a, "cpu")
    assert t.dtype == torch.float32 and torch.equal(t, torch.from_numpy(np.ascontiguousarray(a)))
    assert h2d(torch.ones(3, dtype=torch.int32), "cpu", torch.float32).dtype == torch.float32
