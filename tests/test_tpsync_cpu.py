"""TPSync (runtime/engine.py): the TP step channel from rank 0 to followers, world 2 (gloo).
``bcast`` transport: small decode steps travel in the 4 KiB prefix, a long block table in prefix +
sized remainder, control messages as objects.  ``bus`` transport (host shared-memory ring,
csrc/host/step_bus.cpp): every step is one message, and the follower makes no device->host copy.
Either way the follower decodes exactly what the leader sent, flags included (graph replay,
look-ahead ids from the device, in-graph sampler)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _steps():
    rng = np.random.default_rng(0)
    out = []
    for B, W in [(1, 3), (16, 8), (32, 64), (4, 600)]:     # the last two exceed the prefix
        out.append((rng.integers(0, 1000, B), rng.integers(0, 5000, B).astype(np.int32),
                    rng.integers(0, 9000, B), rng.integers(0, 300, (B, W)).astype(np.int32),
                    rng.integers(1, 5000, B).astype(np.int32)))
    return out


def _worker(rank, port, q, transport):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from lumen_amd.runtime.engine import TPSync

    ts = TPSync(device=torch.device("cpu"), capacity=4 * 600 + 4 * 4 + 64, transport=transport)
    steps = _steps()
    big = ("pbuild", 7, {"blob": bytes(range(256)) * 4096})          # 1 MiB: larger than a bus slot
    if rank == 0:
        for i, (ids, pos, slots, bt, ctx) in enumerate(steps):
            ts.send_decode(None if i == 2 else ids, pos, slots, bt, ctx, {"k": 8, "inv": None, "pen": None},
                           graph=i % 2 == 0, ingraph=i >= 2)
        ts.send(big)
        ts.send(("stop", {"why": "done"}))
        q.put(dict(ts.stats, transport=ts.transport))
    else:
        ok = True
        for i, (ids, pos, slots, bt, ctx) in enumerate(steps):
            m = ts.recv()
            ok &= m[0] == "decode" and (m[1] is None if i == 2 else np.array_equal(m[1], ids))
            ok &= np.array_equal(m[2], pos)
            ok &= np.array_equal(m[3], slots) and np.array_equal(m[4], bt) and np.array_equal(m[5], ctx)
            ok &= m[6]["k"] == 8 and m[7] == (i % 2 == 0) and m[8] == (i >= 2)
        ok &= ts.recv() == big
        ok &= ts.recv() == ("stop", {"why": "done"})
        q.put({"ok": ok, "d2h": ts.stats["d2h"], "transport": ts.transport})
        ts.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["bcast", "bus"])
def test_tpsync_transports(transport):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q, transport)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    stats = [r for r in res if "tensor_steps" in r][0]
    fol = [r for r in res if "ok" in r][0]
    assert fol["ok"] and stats["transport"] == fol["transport"] == transport
    assert stats["tensor_steps"] == 4 and stats["object_steps"] == 2
    if transport == "bcast":
        assert stats["two_part_steps"] == 2 and fol["d2h"] >= 6
    else:
        assert stats["two_part_steps"] == 0 and fol["d2h"] == 0
